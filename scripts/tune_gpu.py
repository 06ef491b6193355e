#!/usr/bin/env python3
"""A/B the CRC32C kernel variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24). Prints a table of GB/s per variant
(algorithmic payload bytes / kernel time from HIP events on the launch stream)
next to the read-only HBM stream probe."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from photonlibos_amd import checksum as ck  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--variants", default="generic,generic:2,generic:4,generic:8,g64")
ap.add_argument("--lanes", default="0")
ap.add_argument("--count", type=int, default=0, help="override buffer count")
args = ap.parse_args()

shapes = {"c2": (65536, 65536), "c3": (4096, 1 << 20), "c4": (1 << 20, 4096), "c5seg": (8192, 1 << 19)}
nbytes, count = shapes[args.config]
count = args.count or count
stream = torch.cuda.current_stream()
buf = torch.empty(nbytes * count, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(buf, nbytes, nbytes, count, 0x5EED0001)
out = torch.zeros(count, dtype=torch.int32, device="cuda")
out64 = torch.zeros(count, dtype=torch.int64, device="cuda")
sink = torch.zeros(256 * 256 * 8, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
total = nbytes * count


def timed(fn):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(args.reps):
        fn()
    b.record(stream)
    b.synchronize()
    return a.elapsed_time(b) / args.reps


def make(v, lanes):
    if v == "read":
        return lambda: ck.read_stream(buf, total, sink, sink.numel(), stream=stream)
    if v.startswith("g64"):  # g64[:MODE:ROWS]: CRC-64, full-row mode and rows per step (photon_crc64_set_full_rows)
        mode, rows = (int(x) for x in v.split(":")[1:3]) if ":" in v else (3, 2)

        def f64():
            ck.set_lanes_per_buffer(lanes)
            ck.set_full_rows64(mode, rows)
            ck.batch64_strided(buf, nbytes, nbytes, count, out64, stream=stream)
        return f64

    def f():
        ck.set_lanes_per_buffer(lanes)
        ck.set_generic_rows(int(v.split(":")[1]) if ":" in v else -1)
        ck.batch_strided(buf, nbytes, nbytes, count, out, stream=stream)
    return f


variants = [(v, int(l)) for v in args.variants.split(",") for l in args.lanes.split(",")] + [("read", 0)]
refs = {}
res = {f"{v}/G{l}": [] for v, l in variants}
for r in range(args.rounds):
    # alternate the order every round (the first launches after a switch can
    # run at a different clock; do not always hand that to the same variant)
    for v, l in (variants if r % 2 == 0 else variants[::-1]):
        ms = timed(make(v, l))
        res[f"{v}/G{l}"].append(ms)
        if v != "read":
            torch.cuda.synchronize()
            is64 = v.startswith("g64")
            o = (out64 if is64 else out).cpu().numpy().copy()
            key = "64" if is64 else "32"
            if key not in refs:
                refs[key] = o
            assert np.array_equal(o, refs[key]), f"variant {v}/G{l} disagrees"
ck.set_generic_rows(-1)
ck.set_lanes_per_buffer(0)
ck.set_full_rows64(3, 2)
rows = []
for k, ms in res.items():
    med, best = float(np.median(ms)), float(np.min(ms))
    rows.append({"variant": k, "ms_median": round(med, 4), "ms_best": round(best, 4),
                 "GBps_median": round(total / med / 1e6, 1), "GBps_best": round(total / best / 1e6, 1),
                 "frac_of_8TBps": round(total / med / 1e6 / 8000, 4)})
for row in rows:
    print(json.dumps(row))
