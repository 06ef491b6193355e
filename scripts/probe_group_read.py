#!/usr/bin/env python3
"""What the CRC kernels' lane-group read pattern can read (bench-only probe,
libphoton_probes.so group_rows_kernel: G lanes per buffer, 64/G buffers per
wave, U rows per step + U in flight, nt loads, XOR instead of CRC) for the
C3 shape (1 Mi x 4 KiB) and the C2 shape (64 Ki x 64 KiB), next to the CRC
kernel itself on the same buffers. Interleaved rounds, median ms."""
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
P.probe_group_rows.argtypes = [vp, u64, u64, u64, vp, ci, ci, ci, vp]
P.probe_group_rows.restype = ci
P.probe_group_rows_slots.argtypes = [vp, u64, u64, u64, vp, ci, ci, ci, vp, vp]
P.probe_group_rows_slots.restype = ci
st = torch.cuda.current_stream()
cus = torch.cuda.get_device_properties(0).multi_processor_count
sink = torch.zeros(cus * 1024, dtype=torch.int32, device="cuda")


def timed(fn, reps=20):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        fn()
    b.record(st)
    b.synchronize()
    return a.elapsed_time(b) / reps


SHAPES = {"c3": (4096, 1 << 20, (8, 16, 32)), "c2": (65536, 65536, (8, 16, 32, 64)), "c5": (8192, 1 << 19, (8, 16)),
          "c4": (1 << 20, 4096, (16, 32, 64)),
          # one 1 GiB buffer's worth (the reference's perf shape) as the long
          # kernel cuts it: 16 Ki x 64 KiB and 4 Ki x 256 KiB pieces
          "g1_64k": (65536, 16384, (32, 64)), "g1_256k": (1 << 18, 4096, (32, 64))}
wanted = sys.argv[1].split(",") if len(sys.argv) > 1 else ["c3", "c2"]


def c5_product(buf, n, cnt):
    # the C5 message batch (bench.py's layout): 65,536 messages x 8 segments
    # at permuted 8 KiB slots, segment CRCs + per-message fold
    perm = np.random.default_rng(0x5EED0005).permutation(cnt).astype(np.uint64)
    iov = np.empty((cnt, 2), np.uint64)
    iov[:, 0] = np.uint64(buf.data_ptr()) + perm * np.uint64(n)
    iov[:, 1] = n
    d_iov = torch.from_numpy(iov.view(np.int64)).cuda()
    d_start = torch.from_numpy(np.arange(0, cnt + 1, 8, dtype=np.uint64).view(np.int64)).cuda()
    seg = torch.zeros(cnt, dtype=torch.int32, device="cuda")
    mout = torch.zeros(cnt // 8, dtype=torch.int32, device="cuda")
    slots = torch.from_numpy(perm.view(np.int64)).cuda()
    return slots, (lambda: ck.batch_msg_n(d_iov, d_start, cnt // 8, cnt, seg, mout, stream=st))


for name in wanted:
    n, cnt, gs = SHAPES[name]
    buf = torch.empty(n * cnt, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(buf, n, n, cnt, 0x5EED0001)
    out = torch.zeros(cnt, dtype=torch.int32, device="cuda")
    variants = {}
    slots, product = (c5_product(buf, n, cnt) if name == "c5" else
                      (None, lambda: ck.batch_strided(buf, n, n, cnt, out, stream=st)))
    sp = slots.data_ptr() if slots is not None else None
    for g in gs:
        for u in (2, 4, 8):
            rows = n // (16 * g)
            if rows % u:
                continue
            variants[f"read G{g} U{u}"] = (lambda g=g, u=u, rows=rows: P.probe_group_rows_slots(
                buf.data_ptr(), n, rows, cnt, sink.data_ptr(), cus, g, u, sp, st.cuda_stream))
    variants["crc (product)"] = product
    res = {k: [] for k in variants}
    for r in range(6):
        for k, f in (list(variants.items()) if r % 2 == 0 else list(variants.items())[::-1]):
            res[k].append(timed(f))
    for k, ms in res.items():
        med = float(np.median(ms))
        print(json.dumps({"shape": name, "variant": k, "ms": round(med, 4), "GBps": round(n * cnt / med / 1e6, 1),
                          "frac_of_8TBps": round(n * cnt / med / 1e6 / 8000, 4)}), flush=True)
    del buf
    torch.cuda.empty_cache()
