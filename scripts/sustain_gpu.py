#!/usr/bin/env python3
"""Back-to-back launches of one variant with per-launch HIP events: shows how
the per-launch time drifts under sustained load (DVFS / power management).
Prints one JSON line per variant: per-launch ms list, first/last/median."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from photonlibos_amd import checksum as ck  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=40)
ap.add_argument("--rest", type=float, default=2.0, help="idle seconds between variants")
ap.add_argument("--variants", default="read,crc:0:1:4:3,crc:32:1:4:3,crc:64:1:4:3,crc:32:0:0:0")
ap.add_argument("--repeat", type=int, default=1)
ap.add_argument("--shape", default="65536x65536", help="nbytes x count")
args = ap.parse_args()
nbytes, count = (int(x) for x in args.shape.split("x"))
total = nbytes * count
st = torch.cuda.current_stream()
buf = torch.empty(total, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(buf, nbytes, nbytes, count, 0x5EED0001)
out = torch.zeros(count, dtype=torch.int32, device="cuda")
sink = torch.zeros(256 * 256 * 8, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
for v in args.variants.split(",") * args.repeat:
    if v == "read":
        fn = lambda: ck.read_stream(buf, total, sink, sink.numel(), stream=st)  # noqa: E731
    else:
        _, g = v.split(":")[:2]
        ck.set_lanes_per_buffer(int(g))
        fn = lambda: ck.batch_strided(buf, nbytes, nbytes, count, out, stream=st)  # noqa: E731
    time.sleep(args.rest)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.n)]
    for a, b_ in ev:
        a.record(st)
        fn()
        b_.record(st)
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b_) for a, b_ in ev]
    print(json.dumps({"variant": v, "first5": [round(x, 3) for x in ms[:5]], "last5": [round(x, 3) for x in ms[-5:]],
                      "median_ms": round(float(np.median(ms)), 4),
                      "median_GBps": round(total / float(np.median(ms)) / 1e6, 1)}), flush=True)
ck.set_lanes_per_buffer(0)
