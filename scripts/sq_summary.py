#!/usr/bin/env python3
"""Summarise scripts/pmc_kernel.sh output: per CRC kernel, LDS busy fraction,
bank-conflict fraction and VALU issue fraction of the kernel's cycles.
GRBM_GUI_ACTIVE is summed over the 8 XCDs, SQ_* over all CUs/SIMDs."""
import collections
import csv
import os
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(list)
    for p in sorted(os.listdir(d)):
        f = os.path.join(d, p, "p_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "crc" not in k or "fill" in k:
                continue
            agg[(k.split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    kern = sorted({k for k, _ in agg})
    for k in kern:
        v = {c: sum(x[-3:]) / len(x[-3:]) for (kk, c), x in agg.items() if kk == k}
        cyc = v["GRBM_GUI_ACTIVE"] / 8
        print(f"{d}: {k}: cycles/XCD {cyc:.4g}  LDS busy {v['SQ_LDS_IDX_ACTIVE'] / 256 / cyc:.2f}  "
              f"bank-conflict {v['SQ_LDS_BANK_CONFLICT'] / 256 / cyc:.3f}  "
              f"VALU issue {v['SQ_INSTS_VALU'] / 1024 * 2 / cyc:.2f}  "
              f"VALU/LDS instr {v['SQ_INSTS_VALU'] / v['SQ_INSTS_LDS']:.2f}  "
              f"per KiB of a 4 GiB launch: VALU {v['SQ_INSTS_VALU'] / 4194304:.1f} LDS {v['SQ_INSTS_LDS'] / 4194304:.1f} "
              f"wave-cycles {v['SQ_WAVE_CYCLES'] / 4194304:.0f} wait-any {v['SQ_WAIT_ANY'] / 4194304:.0f} "
              f"clock {cyc / (v.get('_dur_ns', 0) or 1):.2f}")
