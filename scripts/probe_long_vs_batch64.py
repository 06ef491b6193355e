#!/usr/bin/env python3
"""CRC-64/ECMA: 1 GiB as one long buffer vs as a batch of 64 KiB pieces,
where the long kernel's extra time sits (bench-only probe; the CRC-32C twin
is probe_long_vs_batch.py). Interleaved rounds, one process:
  long<L>x<R> = crc64_long_stamped_kernel (the product's crc64_long_run +
          stamps), base+1, the product's plan for that shape (0x0 automatic);
  batch<G> = crc64_batch_stamped_kernel (crc64_batch_run + stamps), 16 Ki x
          64 KiB from an aligned base.
Stamps per wave (s_memrealtime, 100 MHz): start, tables built, [long: basis
words done], loop done, end. Per launch: HIP-event time; medians over waves
of table build, basis words and the first-start -> loop-end time; the p90 /
max of loop ends; the last end (span). One JSON line per variant (medians
over launches)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from photonlibos_amd import checksum as ck  # noqa: E402

P = ctypes.CDLL(os.path.join(REPO, "photonlibos_amd", "lib", "libphoton_probes.so"))
vp, u64, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
P.probe_crc64_long_stamped.argtypes = [vp, u64, u64, vp, vp, vp, ci, ci, ci, vp, vp]
P.probe_crc64_long_stamped.restype = ci
P.probe_crc64_batch_stamped.argtypes = [vp, u64, u64, vp, vp, ci, ci, vp]
P.probe_crc64_batch_stamped.restype = ci

st = torch.cuda.current_stream()
cus = torch.cuda.get_device_properties(0).multi_processor_count
n = 1 << 30
N = int(os.environ.get("LAUNCHES", "8"))
ROUNDS = int(os.environ.get("ROUNDS", "6"))
VARIANTS = os.environ.get("VARIANTS", "long0x0,long32x2,batch32,batch64").split(",")
d = torch.empty(n + 8192, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(d, n + 8192, n + 8192, 1, 0x5EED0B00, stream=st)
out = torch.zeros(1 << 14, dtype=torch.int64, device="cuda")
state = torch.zeros(1024, dtype=torch.int64, device="cuda")
nw = cus * 16
ts = {v: [torch.zeros(8 * nw, dtype=torch.int64, device="cuda") for _ in range(N)] for v in VARIANTS}
grid = ctypes.c_int(0)


def run(v, k):
    t = ts[v][k].data_ptr()
    if v.startswith("long"):
        lanes, rounds = (int(x) for x in v[4:].split("x"))
        rc = P.probe_crc64_long_stamped(d.data_ptr() + 1, n, 7, out.data_ptr(), state.data_ptr(), t, cus, lanes,
                                        rounds, ctypes.byref(grid), ctypes.c_void_p(st.cuda_stream))
    else:
        rc = P.probe_crc64_batch_stamped(d.data_ptr(), 65536, n >> 16, out.data_ptr(), t, int(v[5:]), cus,
                                         ctypes.c_void_p(st.cuda_stream))
    assert rc == 0, (v, rc)


def stats(v, k):
    t = ts[v][k].cpu().numpy().reshape(-1, 8).astype(np.int64)
    t = t[t[:, 4] > 0]
    b = t[:, 0].min()
    us = lambda x: float(x) / 100.0  # noqa: E731
    r = {"waves": int(len(t)), "start_max_us": us((t[:, 0] - b).max()),
         "tables_p50_us": us(np.median(t[:, 1] - t[:, 0]))}
    if v.startswith("long"):
        r["basis_p50_us"] = us(np.median(t[:, 2] - t[:, 1]))
    loop_end = t[:, 3] - b
    r.update({"loop_end_p50_us": us(np.median(loop_end)), "loop_end_p90_us": us(np.percentile(loop_end, 90)),
              "loop_end_max_us": us(loop_end.max()), "span_us": us((t[:, 4] - b).max()),
              "tail_after_loops_us": us(t[:, 4].max() - t[:, 3].max())})
    xcc = t[:, 6] & 7
    r["xcc_loop_end_p50_us"] = [us(np.median(loop_end[xcc == x])) if (xcc == x).any() else None for x in range(8)]
    return r


res = {v: [] for v in VARIANTS}
for r in range(ROUNDS):
    for v in (VARIANTS if r % 2 == 0 else VARIANTS[::-1]):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(N)]
        for k in range(N):
            ts[v][k].zero_()
        for k in range(N):
            ev[k][0].record(st)
            run(v, k)
            ev[k][1].record(st)
        torch.cuda.synchronize()
        for k in range(N // 2, N):
            s = stats(v, k)
            s["event_us"] = ev[k][0].elapsed_time(ev[k][1]) * 1e3
            res[v].append(s)
for v, rows in res.items():
    agg = {key: round(float(np.median([r[key] for r in rows])), 2) for key in rows[0] if key != "xcc_loop_end_p50_us"}
    agg["xcc_loop_end_p50_us"] = [round(float(np.median([r["xcc_loop_end_p50_us"][x] for r in rows
                                                          if r["xcc_loop_end_p50_us"][x] is not None])), 1)
                                  for x in range(8)]
    print(json.dumps({"variant": v, "n": n, **agg}), flush=True)
