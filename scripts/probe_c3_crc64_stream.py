#!/usr/bin/env python3
"""CRC-64/ECMA on the C3 shape (1 Mi x 4 KiB, strided, aligned): the generic
batch kernel (the product) against the opt-in streaming kernel
(crc64_uniform_kernel: rows in flight ACROSS buffer boundaries) at several
shapes, interleaved in rounds in one process after a 3 s warm-up. Bench-only
probe; one JSON line per variant (median launch by HIP events, fraction of
8 TB/s, CRCs equal to the generic kernel's).

  VARIANTS="gen:16,gen:8,st:16:2:2:1:1,..."  (st:G:U:D:V:B)"""
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
n, cnt = 4096, 1 << 20
VARIANTS = os.environ.get("VARIANTS", "gen:16,st:16:2:2:1:1,st:16:2:3:1:1,st:16:4:2:1:1,st:16:2:4:1:1,"
                                      "st:8:4:2:1:1,st:16:4:2:2:1,st:8:2:4:1:1").split(",")
N, ROUNDS = 10, 6
buf = torch.empty(n * cnt, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(buf, n, n, cnt, 0x5EED0C30, stream=st)
outs = {v: torch.zeros(cnt, dtype=torch.int64, device="cuda") for v in VARIANTS}


def configure(v):
    f = v.split(":")
    ck.set_lanes_per_buffer(int(f[1]))
    if f[0] == "gen":
        ck.set_stream64_config(0, 0)
    else:
        u, d, vv, b = (int(x) for x in f[2:6])
        ck.set_stream64_config(u, d)
        ck.set_stream64_interleave(vv)
        ck.set_stream64_run_blocks(b)


def launch(v):
    ck.batch64_strided(buf, n, n, cnt, outs[v], stream=st)


configure(VARIANTS[0])
t_end = time.time() + 3.0
while time.time() < t_end:
    for _ in range(10):
        launch(VARIANTS[0])
    torch.cuda.synchronize()
res = {v: [] for v in VARIANTS}
for r in range(ROUNDS):
    for v in (VARIANTS if r % 2 == 0 else VARIANTS[::-1]):
        configure(v)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(N + 1)]
        ev[0].record(st)
        for k in range(N):
            launch(v)
            ev[k + 1].record(st)
        torch.cuda.synchronize()
        res[v] += [ev[k].elapsed_time(ev[k + 1]) for k in range(N)]
ck.set_stream64_config(0, 0)
ck.set_lanes_per_buffer(0)
ref = outs[VARIANTS[0]]
for v in VARIANTS:
    m = float(np.median(res[v]))
    print(json.dumps({"variant": v, "launch_us_median": round(m * 1e3, 1), "frac": round(n * cnt / (m * 1e-3) / 8e12, 4),
                      "same_crc": bool(torch.equal(outs[v], ref))}), flush=True)
