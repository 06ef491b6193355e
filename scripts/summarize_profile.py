#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output for the CRC kernels into profiles/*.json.

  --stats DIR   : a `rocprofv3 --kernel-trace --stats --output-format csv` run
  --pmc DIR     : a `rocprofv3 --pmc FETCH_SIZE ... --output-format csv` run
Per kernel: launches, average duration (ns) and, from the PMC pass, HBM read
bytes per launch = FETCH_SIZE (KiB) * 1024 * 2 -- FETCH_SIZE counts half the
bytes of wide coalesced reads on gfx950 (MI355X_MICROARCH.md, HBM section).
"""
import argparse
import csv
import glob
import json
import os
import statistics


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats")
    ap.add_argument("--pmc")
    ap.add_argument("--kernel", default="crc32c")
    ap.add_argument("--payload-bytes", type=float, required=True, help="algorithmic bytes per launch")
    ap.add_argument("--out", required=True)
    ap.add_argument("--last", type=int, default=0, help="average only the last N launches (the timed steps)")
    args = ap.parse_args()
    res = {"payload_bytes_per_launch": args.payload_bytes}
    if args.stats:
        kt = [r for r in rows(os.path.join(args.stats, "**", "*kernel_trace.csv")) if args.kernel in r["Kernel_Name"]]
        durs = {}
        for r in sorted(kt, key=lambda r: int(r["Start_Timestamp"])):
            durs.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        if args.last:
            durs = {k: v[-args.last:] for k, v in durs.items()}
        res["kernels"] = {k: {"launches": len(v), "avg_ns": statistics.mean(v), "min_ns": min(v),
                              "achieved_GBps": args.payload_bytes / statistics.mean(v)}
                          for k, v in durs.items()}
        st = rows(os.path.join(args.stats, "**", "*kernel_stats.csv"))
        res["kernel_stats_csv"] = [r for r in st if args.kernel in r.get("Name", "")]
    if args.pmc:
        pc = [r for r in rows(os.path.join(args.pmc, "**", "*counter_collection.csv"))
              if args.kernel in r["Kernel_Name"]]
        per = {}
        for r in pc:
            if r["Counter_Name"] == "FETCH_SIZE":
                per.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
        res["pmc"] = {k: {"launches": len(v), "FETCH_SIZE_KiB_avg": statistics.mean(v),
                          "hbm_read_bytes_per_launch": statistics.mean(v) * 1024 * 2,
                          "traffic_over_payload": statistics.mean(v) * 1024 * 2 / args.payload_bytes}
                      for k, v in per.items()}
        main_k = max(per, key=lambda k: statistics.mean(per[k])) if per else None
        if main_k:
            res["hbm_bytes_per_launch"] = res["pmc"][main_k]["hbm_read_bytes_per_launch"]
            res["hbm_kernel"] = main_k
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernel_stats_csv"}, indent=1))


if __name__ == "__main__":
    main()
