#!/usr/bin/env python3
"""Per-launch fixed cost of the batch kernels (LDS table building in the
prologue + launch): time a batch whose payload is negligible (4096 buffers of
64 B, i.e. one 16-byte block per lane and a persistent grid of one workgroup
per CU) with HIP events, CRC32C per lane-group size and CRC-64."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from photonlibos_amd import checksum as ck  # noqa: E402

st = torch.cuda.current_stream()
nbytes, count = 64, 4096 * 16
buf = torch.zeros(nbytes * count, dtype=torch.uint8, device="cuda")
out = torch.zeros(count, dtype=torch.int32, device="cuda")
out64 = torch.zeros(count, dtype=torch.int64, device="cuda")


def timed(f, reps=200):
    for _ in range(10):
        f()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        f()
    b.record(st)
    b.synchronize()
    return a.elapsed_time(b) / reps * 1000.0


res = {}
for g in (4, 8, 16, 32, 64):
    ck.set_lanes_per_buffer(g)
    res[f"crc32c G{g}"] = timed(lambda: ck.batch_strided(buf, nbytes, nbytes, count, out, stream=st))
    res[f"crc64 G{g}"] = timed(lambda: ck.batch64_strided(buf, nbytes, nbytes, count, out64, stream=st))
ck.set_lanes_per_buffer(0)
for k, v in res.items():
    print(json.dumps({"kernel": k, "us_per_launch": round(v, 2), "buffers": count, "nbytes": nbytes}))
