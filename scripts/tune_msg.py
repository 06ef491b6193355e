#!/usr/bin/env python3
"""A/B of the message-batch forms on the C5 layout (65,536 messages x 8
scattered 8 KiB segments): one fused kernel vs segment kernel + fold kernel,
with and without per-segment CRC output. One process, interleaved rounds;
kernel time from HIP events on the launch stream."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from photonlibos_amd import checksum as ck  # noqa: E402

nmsg, nseg, n = 65536, 8, 8192
slots = nmsg * nseg
st = torch.cuda.current_stream()
pool = torch.empty(slots * n, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(pool, n, n, slots, 0x5EED0001)
perm = np.random.default_rng(0x5EED0005).permutation(slots).astype(np.uint64)
iov = np.empty((slots, 2), np.uint64)
iov[:, 0] = np.uint64(pool.data_ptr()) + perm * np.uint64(n)
iov[:, 1] = n
d_iov = torch.from_numpy(iov.view(np.int64)).cuda()
d_start = torch.from_numpy(np.arange(0, slots + 1, nseg, dtype=np.uint64).view(np.int64)).cuda()
seg = torch.zeros(slots, dtype=torch.int32, device="cuda")
out = torch.zeros(nmsg, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--lanes", default="0", help="comma list of lane-group sizes (0 = product choice)")
ap.add_argument("--rows", default="2", help="comma list of message rows per step")
ap.add_argument("--forms", default="fused+seg,fused-noseg,two+seg,two-noseg")
args = ap.parse_args()
forms = {"fused+seg": (1, seg), "fused-noseg": (1, None), "two+seg": (2, seg), "two-noseg": (2, None)}
variants = {f"{f}/G{g}/U{u}": (forms[f][0], forms[f][1], int(g), int(u))
            for f in args.forms.split(",") for g in args.lanes.split(",") for u in args.rows.split(",")}
res = {k: [] for k in variants}
ref = None
for r in range(args.rounds):
    for k, (mode, so, g, u) in (list(variants.items()) if r % 2 == 0 else list(variants.items())[::-1]):
        ck.set_msg_mode(mode)
        ck.set_lanes_per_buffer(g)
        ck.set_msg_rows(u)
        f = lambda: ck.batch_msg_n(d_iov, d_start, nmsg, slots, so, out, stream=st)  # noqa: E731
        f()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(args.reps):
            f()
        b.record(st)
        b.synchronize()
        res[k].append(a.elapsed_time(b) / args.reps)
        o = out.cpu().numpy().copy()
        if ref is None:
            ref = o
        assert np.array_equal(o, ref), k
ck.set_msg_mode(0)
ck.set_lanes_per_buffer(0)
ck.set_msg_rows(2)
for k, ms in res.items():
    med = float(np.median(ms))
    print(json.dumps({"variant": k, "ms_median": round(med, 4), "GBps": round(slots * n / med / 1e6, 1),
                      "frac_of_8TBps": round(slots * n / med / 1e6 / 8000, 4)}))
