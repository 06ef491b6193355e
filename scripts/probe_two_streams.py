#!/usr/bin/env python3
"""The driver's window (fresh process, fill, 5 warmup + 20 timed steps) with
the C2 batch launched three ways (bench-only probe; one variant per process):
  single : one launch of the whole batch per step on one stream (the product);
  forkjoin: per step, two launches of half the batch on two streams forked from
            and joined back to the main stream by events;
  free   : the two half-batch launches on two streams with no join between
            steps (as two ranks sharing one GPU).
Prints one JSON line: GiB/s over the timed steps (wall, synchronised), ms per
step, and the CRCs checked against the single-stream result of step 0.

  python scripts/probe_two_streams.py single|forkjoin|free|shape:G:U
  (shape:G:U = single with lanes per buffer G and rows per step U, tuning.h)
"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from photonlibos_amd import checksum as ck  # noqa: E402

mode = sys.argv[1]
if mode.startswith("shape:"):
    _, g_, u_ = mode.split(":")
    ck.set_lanes_per_buffer(int(g_))
    ck.set_generic_rows(int(u_))
W, K = 5, 20
n, cnt = 65536, 65536
h = cnt // 2
buf = torch.empty(n * cnt, dtype=torch.uint8, device="cuda")
out = torch.zeros(cnt, dtype=torch.int32, device="cuda")
main = torch.cuda.current_stream()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
ck.fill_splitmix(buf, n, n, cnt, 0x5EED0001, stream=main)
want = torch.zeros(cnt, dtype=torch.int32, device="cuda")


def step():
    if mode == "single" or mode.startswith("shape:"):
        ck.batch_strided(buf, n, n, cnt, out, stream=main)
        return
    if mode == "forkjoin":
        e = torch.cuda.Event()
        e.record(main)
        s1.wait_event(e)
        s2.wait_event(e)
    ck.batch_strided(buf.data_ptr(), n, n, h, out[:h], stream=s1)
    ck.batch_strided(buf.data_ptr() + h * n, n, n, h, out[h:], stream=s2)
    if mode == "forkjoin":
        a, b = torch.cuda.Event(), torch.cuda.Event()
        a.record(s1)
        b.record(s2)
        main.wait_event(a)
        main.wait_event(b)


for _ in range(W):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    step()
torch.cuda.synchronize()
t1 = time.perf_counter()
ck.batch_strided(buf, n, n, cnt, want, stream=main)
torch.cuda.synchronize()
ms = (t1 - t0) / K * 1e3
print(json.dumps({"mode": mode, "GiB_per_s": round(n * cnt / (ms * 1e-3) / 2 ** 30, 1), "ms_per_step": round(ms, 4),
                  "frac_wall": round(n * cnt / (ms * 1e-3) / 8e12, 4), "same_crc": bool(torch.equal(out, want))}))
