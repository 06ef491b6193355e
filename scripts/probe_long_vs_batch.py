#!/usr/bin/env python3
"""1 GiB as one long buffer vs as a batch of 64 KiB pieces: where the long
kernel's extra time sits (bench-only probe). Interleaved rounds, one process:
  long  = long_stamped_kernel (the product's long_run + stamps), base+1, the
          product's plan for 32 lanes x 2 rounds;
  batch = crc_wave_times_kernel (the product's batch kernel + stamps), 16 Ki x
          64 KiB from an aligned base, 32 lanes.
Per launch: HIP-event time, stamp span (first wave start -> last wave end),
the spread of wave END times (p50, p90, max minus first start) and per-XCC
median end. Prints one JSON line per variant (medians over launches)."""
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
vp, u64, u32, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
P.probe_long_stamped.argtypes = [vp, u64, u32, vp, vp, vp, ci, ci, ci, u64, vp, vp]
P.probe_long_stamped.restype = ci
P.probe_crc_wave_times.argtypes = [vp, u64, u64, vp, vp, vp, ci, ci, ci, ci, vp]
P.probe_crc_wave_times.restype = ci

st = torch.cuda.current_stream()
cus = torch.cuda.get_device_properties(0).multi_processor_count
n = 1 << 30
N = int(os.environ.get("LAUNCHES", "8"))
ROUNDS = int(os.environ.get("ROUNDS", "6"))
d = torch.empty(n + 8192, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(d, n + 8192, n + 8192, 1, 0x5EED0B00, stream=st)
out = torch.zeros(1 << 14, dtype=torch.int32, device="cuda")
state = torch.zeros(1024, dtype=torch.int32, device="cuda")
ticket = torch.zeros(256, dtype=torch.int32, device="cuda")
nw = cus * 16
tl = [torch.zeros(8 * nw, dtype=torch.int64, device="cuda") for _ in range(N)]
tb = [torch.zeros(6 * nw, dtype=torch.int64, device="cuda") for _ in range(N)]
grid = ctypes.c_int(0)


def run(kind, k):
    if kind == "long":
        rc = P.probe_long_stamped(d.data_ptr() + 1, n, 7, out.data_ptr(), state.data_ptr(), tl[k].data_ptr(), cus,
                                  32, 2, 0, ctypes.byref(grid), ctypes.c_void_p(st.cuda_stream))
    else:
        rc = P.probe_crc_wave_times(d.data_ptr(), 65536, n >> 16, out.data_ptr(), tb[k].data_ptr(),
                                    ticket.data_ptr(), 32, 0, 0, cus, ctypes.c_void_p(st.cuda_stream))
    assert rc == 0, (kind, rc)


def stats(kind, k):
    if kind == "long":
        t = tl[k].cpu().numpy().reshape(-1, 8).astype(np.int64)
        t = t[t[:, 3] > 0]
        start, body_end, end, xcc = t[:, 0], t[:, 2], t[:, 3], t[:, 5] & 7
    else:
        t = tb[k].cpu().numpy().reshape(-1, 6).astype(np.int64)
        t = t[t[:, 1] > 0]
        start, body_end, end, xcc = t[:, 0], t[:, 1], t[:, 1], t[:, 3] & 7
    b = start.min()
    rel = (body_end - b) / 100.0
    extra = {"start_p50_us": float(np.median(start - b)) / 100.0, "start_max_us": float((start - b).max()) / 100.0}
    if kind == "long":  # table build + basis words: wave start -> first chunk
        extra["prologue_p50_us"] = float(np.median(t[:, 1] - start)) / 100.0
    return {**extra, "span_us": (end.max() - b) / 100.0, "end_p50_us": float(np.median(rel)),
            "end_p90_us": float(np.percentile(rel, 90)), "end_max_us": float(rel.max()),
            "tail_after_body_us": (end.max() - body_end.max()) / 100.0,
            "xcc_end_med_us": [float(np.median(rel[xcc == x])) for x in range(8)]}


res = {kind: [] for kind in ("long", "batch")}
for r in range(ROUNDS):
    for kind in (("long", "batch") if r % 2 == 0 else ("batch", "long")):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(N)]
        for k in range(N):
            ev[k][0].record(st)
            run(kind, k)
            ev[k][1].record(st)
        torch.cuda.synchronize()
        for k in range(N // 2, N):
            s = stats(kind, k)
            s["event_us"] = ev[k][0].elapsed_time(ev[k][1]) * 1e3
            res[kind].append(s)
for kind, rows in res.items():
    agg = {key: round(float(np.median([r[key] for r in rows])), 2) for key in rows[0] if key != "xcc_end_med_us"}
    agg["xcc_end_med_us"] = [round(float(np.median([r["xcc_end_med_us"][x] for r in rows])), 1) for x in range(8)]
    print(json.dumps({"variant": kind, "n": n, **agg}), flush=True)
