#!/usr/bin/env python3
"""One long buffer (photon_crc32c_extend_device / photon_crc64ecma_extend_device)
in every long-kernel shape (tuning.h photon_crc_set_long_shape: lanes per
chunk x chunks per lane group of the grid), beside the strided batch kernel
and the read-only stream over the same bytes (bench-only tuning sweep).
Buffers at base+1 like the reference's perf test (test_checksum.cpp:125-168).
One JSON line per (size, shape); every shape's CRC must equal the first's."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from photonlibos_amd import checksum as ck  # noqa: E402

st = torch.cuda.current_stream()
N = int(os.environ.get("LAUNCHES", "30"))
SHAPES = [tuple(int(v) for v in x.split("/")) for x in
          os.environ.get("SHAPES", "64/1,64/2,64/4,32/1,32/2,32/4").split(",")]
SIZES = [int(x) << 20 for x in os.environ.get("SIZES_MIB", "1024,256,64").split(",")]


def host_us(fn, k=200):
    # submission cost per call (the queue absorbs the launches; no wait inside)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return round((t1 - t0) / k * 1e6, 2)


def timed(fn):
    for _ in range(5):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(N)]
    for a, b in ev:
        a.record(st)
        fn()
        b.record(st)
    torch.cuda.synchronize()
    t = np.array([a.elapsed_time(b) for a, b in ev])
    return float(np.mean(t)), float(np.median(t))


big = max(SIZES)
d = torch.empty(big + 4096, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(d, big + 4096, big + 4096, 1, 0x5EED0B00, stream=st)
out = torch.zeros(1, dtype=torch.int32, device="cuda")
out64 = torch.zeros(1, dtype=torch.int64, device="cuda")
sink = torch.zeros(1 << 22, dtype=torch.int32, device="cuda")
for n in SIZES:
    base = d.data_ptr() + 1
    lib = os.environ.get("PHOTON_CRC_LIB", "in-tree")
    mean, med = timed(lambda: ck.read_stream(d.data_ptr(), n, sink, sink.numel(), stream=st))
    hus = host_us(lambda: ck.read_stream(d.data_ptr(), n, sink, sink.numel(), stream=st))
    print(json.dumps({"n": n, "kernel": "read_stream", "ms": round(mean, 4), "frac": round(n / mean / 8e9, 4),
                      "host_us_per_call": hus}),
          flush=True)
    pieces = torch.zeros(n >> 16, dtype=torch.int32, device="cuda")
    mean, med = timed(lambda: ck.batch_strided(d.data_ptr(), 65536, 65536, n >> 16, pieces, stream=st))
    print(json.dumps({"n": n, "kernel": "strided 64 KiB pieces", "ms": round(mean, 4),
                      "frac": round(n / mean / 8e9, 4)}), flush=True)
    ref = ref64 = None
    for lanes, rounds in SHAPES:
        ck.set_long_shape(lanes, rounds)
        mean, med = timed(lambda: ck.extend_device(base, n, 7, out, stream=st))
        crc = int(out.cpu().numpy().view(np.uint32)[0])
        mean64, _ = timed(lambda: ck.extend64_device(base, n, out64, seed=7, stream=st))
        crc64 = int(out64.cpu().numpy().view(np.uint64)[0])
        hus = host_us(lambda: ck.extend_device(base, n, 7, out, stream=st))
        ref = crc if ref is None else ref
        ref64 = crc64 if ref64 is None else ref64
        print(json.dumps({"n": n, "lib": lib, "kernel": "long", "lanes": lanes, "rounds": rounds, "ms": round(mean, 4),
                          "ms_median": round(med, 4), "frac": round(n / mean / 8e9, 4),
                          "crc64_ms": round(mean64, 4), "crc64_frac": round(n / mean64 / 8e9, 4),
                          "host_us_per_call": hus, "same_crc": crc == ref and crc64 == ref64}), flush=True)
    ck.set_long_shape(0, 0)
