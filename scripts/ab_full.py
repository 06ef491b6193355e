#!/usr/bin/env python3
"""A/B of the batch kernels on whole-step uniform batches, in ONE process
with interleaved rounds: the generic batch kernel (mode 0) against the
full-row kernel (crc32c_full_kernel / crc64_full_kernel, mode 1) and its
cross-buffer-prefetch form (mode 2), rows per step as given (0 = the batch
kernel's). Every variant's CRCs must equal the first variant's (the generic
kernel, which the GPU parity suite pins to the oracle). CRC-64 only: the
CRC-32C form of the full-row kernel measured slower than the generic batch
kernel on C2/C3/C4 (profiles/r05b_ab_full32_*.jsonl) and was removed. One JSON line per
variant: mean / median launch time (HIP events on the launch stream) and the
fraction of 8 TB/s."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from photonlibos_amd import checksum as ck  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3", choices=["c2", "c3", "c4"])
ap.add_argument("--crc", type=int, default=64, choices=[64])  # (round 5's CRC-32C full-row kernel measured slower: removed)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--variants", default="0:2,1:2,2:2,1:4,2:4",
                help="mode:rows[:lanes] per variant (lanes 0 = --lanes / automatic)")
ap.add_argument("--lanes", type=int, default=0)
ap.add_argument("--no-check", action="store_true", help="ablation builds (PHOTON_CRC_LIB): results are not CRCs")
args = ap.parse_args()

nbytes, count = {"c2": (65536, 65536), "c3": (4096, 1 << 20), "c4": (1 << 20, 4096)}[args.config]
st = torch.cuda.current_stream()
buf = torch.empty(nbytes * count, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(buf, nbytes, nbytes, count, 0x5EED0001)
out = torch.zeros(count, dtype=torch.int64 if args.crc == 64 else torch.int32, device="cuda")
setk = ck.set_full_rows64
run = ck.batch64_strided if args.crc == 64 else ck.batch_strided
ck.set_lanes_per_buffer(args.lanes)
variants = [tuple(int(x) for x in (v + ":0").split(":")[:3]) if v.count(":") == 1 else tuple(int(x) for x in v.split(":"))
            for v in args.variants.split(",")]
ref = None
times = {v: [] for v in variants}
for r in range(args.rounds):
    for v in (variants if r % 2 == 0 else variants[::-1]):
        setk(v[0], v[1])
        ck.set_lanes_per_buffer(v[2] or args.lanes)
        run(buf, nbytes, nbytes, count, out, stream=st)  # warm this shape
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.reps + 1)]
        ev[0].record(st)
        for k in range(args.reps):
            run(buf, nbytes, nbytes, count, out, stream=st)
            ev[k + 1].record(st)
        torch.cuda.synchronize()
        times[v] += [ev[k].elapsed_time(ev[k + 1]) for k in range(args.reps)]
        o = out.cpu().numpy().copy()
        if ref is None:
            ref = o
        assert args.no_check or np.array_equal(o, ref), f"variant {v} disagrees with the first variant"
setk(3, 2)
ck.set_lanes_per_buffer(0)
for v in variants:
    ms = np.asarray(times[v])
    print(json.dumps({"config": args.config + ("_crc64" if args.crc == 64 else ""), "mode": v[0], "rows": v[1],
                      "lanes": v[2] or args.lanes or "auto",
                      "launches": int(ms.size), "ms_mean": round(float(ms.mean()), 5),
                      "ms_median": round(float(np.median(ms)), 5),
                      "frac_mean": round(nbytes * count / (ms.mean() * 1e-3) / 8e12, 4),
                      "frac_median": round(nbytes * count / (np.median(ms) * 1e-3) / 8e12, 4)}), flush=True)
