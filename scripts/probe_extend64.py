#!/usr/bin/env python3
"""CRC-64/ECMA on one device buffer at base+1 (the reference's perf shapes,
test_checksum.cpp:204-216: 128 KiB and 1 GiB through crc64ecma_hw):
photon_crc64ecma_extend_device kernel time (HIP events, median of 200 / 50
launches) and enqueue + wait, and the routed crc64ecma_extend on a device
pointer (128 KiB and 1 GiB). Bench-only probe; prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from photonlibos_amd import checksum as ck  # noqa: E402

st = torch.cuda.current_stream()
n1 = 1 << 30
d = torch.empty(n1 + 64, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(d, n1 + 64, n1 + 64, 1, 0x5EED0964, stream=st)
out = torch.zeros(64, dtype=torch.int64, device="cuda")
res = {"metric": "photon_crc64ecma_extend_device at base+1"}
for label, n, k in (("128KiB", 128 << 10, 200), ("1GiB", n1, 50)):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]
    ev[0].record(st)
    for i in range(k):
        ck.extend64_device(d.data_ptr() + 1, n, out[i % 64:i % 64 + 1], seed=7, stream=st)
        ev[i + 1].record(st)
    torch.cuda.synchronize()
    t = np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(k)])
    lat = []
    for _ in range(50):
        t0 = time.perf_counter()
        ck.extend64_device(d.data_ptr() + 1, n, out[:1], seed=7, stream=st)
        st.synchronize()
        lat.append(time.perf_counter() - t0)
    res[label] = {"kernel_us_median": round(float(np.median(t)) * 1e3, 2),
                  "frac_median": round(n / (float(np.median(t)) * 1e-3) / 8e12, 4),
                  "call_wait_us_median": round(float(np.median(lat)) * 1e6, 1)}
ck.set_device_dispatch(True)
routed = []
for _ in range(50):
    t0 = time.perf_counter()
    r = ck.crc64ecma_extend_at(d.data_ptr() + 1, 128 << 10, 7)
    routed.append(time.perf_counter() - t0)
routed_1g = []
for _ in range(10):  # the long kernel, result as two tagged words
    t0 = time.perf_counter()
    r1 = ck.crc64ecma_extend_at(d.data_ptr() + 1, n1, 7)
    routed_1g.append(time.perf_counter() - t0)
ck.set_device_dispatch(False)
want = ck.crc64ecma_extend(d[1:1 + (128 << 10)].cpu().numpy().tobytes(), 7)
ck.extend64_device(d.data_ptr() + 1, n1, out[:1], seed=7, stream=st)
st.synchronize()
res["routed_128KiB_us_median"] = round(float(np.median(routed)) * 1e6, 1)
res["routed_1GiB_us_median"] = round(float(np.median(routed_1g)) * 1e6, 1)
res["self_check"] = r == want and r1 == int(out[0].item()) & 0xFFFFFFFFFFFFFFFF
print(json.dumps(res))
