#!/usr/bin/env python3
"""HBM read-ceiling probes (bench-only libphoton_probes.so): grid-stride
streaming reads and the CRC kernels' one-wave-per-buffer row pattern, with
and without the nontemporal hint. Prints GB/s per variant (median of rounds)."""
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
P.probe_read_gridstride.argtypes = [vp, u64, vp, ci, ci, ci, vp]
P.probe_read_rows.argtypes = [vp, u64, u64, u64, vp, ci, ci, ci, vp]

nbytes, count = 65536, 65536
total = nbytes * count
buf = torch.empty(total, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(buf, nbytes, nbytes, count, 1)
sink = torch.zeros(256 * 1024 * 8, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()
s = st.cuda_stream


def timed(fn, reps=5):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        fn()
    b.record(st)
    b.synchronize()
    return a.elapsed_time(b) / reps


variants = {}
for blocks in (1024, 2048, 4096):
    for unr in (8, 16):
        for nt in (0, 1):
            variants[f"gridstride b{blocks} u{unr} nt{nt}"] = (lambda b=blocks, u=unr, n=nt:
                P.probe_read_gridstride(buf.data_ptr(), total, sink.data_ptr(), b, u, n, s))
for u in (4, 8, 16):
    for nt in (0, 1):
        variants[f"rows u{u} nt{nt}"] = (lambda u=u, n=nt:
            P.probe_read_rows(buf.data_ptr(), nbytes, nbytes // 1024, count, sink.data_ptr(), 256, u, n, s))
res = {k: [] for k in variants}
for r in range(4):
    for k, f in variants.items():
        res[k].append(timed(f))
for k, ms in res.items():
    med = float(np.median(ms))
    print(json.dumps({"probe": k, "ms": round(med, 4), "GBps": round(total / med / 1e6, 1),
                      "frac_of_8TBps": round(total / med / 1e6 / 8000, 4)}))

# (The round-1 ablations of the retired streaming CRC kernels, probe_crc_ablate /
# probe_crc64_ablate, were removed with those kernels in round 6; their numbers
# stay in repo:profiles/r01_hbm_probes.jsonl and DESIGN.md §4 / §4.1. The
# product kernels' ablations are PCRC_ABL / PCRC64_ABL builds, scripts/gpu.sh abn.)
