#!/usr/bin/env python3
"""Where does a long-buffer launch spend its time? (bench-only probe)

long_stamped_kernel (libphoton_probes.so) is the product's
crc32c_long_kernel<G, 4> (the same long_run) with per-wave s_memrealtime
stamps at the start, after the LDS table prologue, after the wave's chunks
and after the cross-workgroup reduce. VARIANTS = lanes/rounds, cut as the
product cuts it for that shape (long_plan.h). For one buffer at base+1 (test_checksum.cpp:125-168)
of each size, LAUNCHES back-to-back launches with HIP events; for the last
launches: event time, the span of the stamps (first start -> last end),
start skew, median prologue, median / max body, the reduce tail, per-XCC
median end, in-kernel clock. The CRC must equal the product's
(photon_crc32c_extend_device). One JSON line per size."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from photonlibos_amd import checksum as ck  # noqa: E402

P = ctypes.CDLL(os.environ.get("PHOTON_CRC_PROBES") or os.path.join(REPO, "photonlibos_amd", "lib", "libphoton_probes.so"))
vp, u64, u32, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
P.probe_long_stamped.argtypes = [vp, u64, u32, vp, vp, vp, ci, ci, ci, u64, vp, vp]
P.probe_long_stamped.restype = ci

N = int(os.environ.get("LAUNCHES", "30"))
SIZES = [int(x) << 20 for x in os.environ.get("SIZES_MIB", "64,256,1024").split(",")]
VARIANTS = [tuple(int(v) for v in x.split("/")) for x in os.environ.get("VARIANTS", "64/1,64/2,32/1,32/2").split(",")]
# CHUNKS_KIB: instead of SIZES, one buffer per forced chunk size c, sized so
# the shape's lane-group slots each get exactly `rounds` chunks:
# n = (slots - 1) * c + 4095 at base+1 (chunk 0 = the 4095-byte head).
CHUNKS = [int(float(x) * 1024) for x in os.environ.get("CHUNKS_KIB", "").split(",") if x]
st = torch.cuda.current_stream()
cus = torch.cuda.get_device_properties(0).multi_processor_count
big = max(SIZES) if not CHUNKS else max(16 * cus * (64 // l) * r * c for l, r in VARIANTS for c in CHUNKS) + 8192
d = torch.empty(big + 4096, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(d, big + 4096, big + 4096, 1, 0x5EED0B00, stream=st)
out = torch.zeros(1, dtype=torch.int32, device="cuda")
want = torch.zeros(1, dtype=torch.int32, device="cuda")
state = torch.zeros(1024, dtype=torch.int32, device="cuda")
TICK = 1e-2  # s_memrealtime: 100 MHz -> 0.01 us

grid = ctypes.c_int(0)
runs = ([(n, l, r, 0) for n in SIZES for l, r in VARIANTS] if not CHUNKS else
        [((16 * cus * (64 // l) * r - 1) * c + 4095, l, r, c) for c in CHUNKS for l, r in VARIANTS])
ROUNDS = int(os.environ.get("ROUNDS", "1"))  # interleaved rounds (A/B in one process), order alternating
nw = cus * 16
ts = [torch.zeros(8 * nw, dtype=torch.int64, device="cuda") for _ in range(N)]
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(N)]
base = d.data_ptr() + 1
rows = {i: [] for i in range(len(runs))}
same = {}
for rnd in range(ROUNDS):
  for i in (range(len(runs)) if rnd % 2 == 0 else reversed(range(len(runs)))):
    n, lanes, rounds, force = runs[i]
    for k in range(N):
        ev[k][0].record(st)
        rc = P.probe_long_stamped(base, n, 7, out.data_ptr(), state.data_ptr(), ts[k].data_ptr(), cus,
                                  lanes, rounds, force, ctypes.byref(grid), ctypes.c_void_p(st.cuda_stream))
        ev[k][1].record(st)
        assert rc == 0, (rc, runs[i])
    torch.cuda.synchronize()
    got = int(out.item())
    ck.extend_device(base, n, 7, want, stream=st)
    torch.cuda.synchronize()
    same[i] = same.get(i, True) and got == int(want.item())
    for k in range(N // 2, N):
        t = ts[k].cpu().numpy().reshape(-1, 8).astype(np.int64)
        t = t[t[:, 3] > 0]
        t0, ttab, tbody, t1 = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
        xcc = t[:, 5] & 7
        clk = np.median((t[:, 7] - t[:, 6]) / np.maximum(t1 - t0, 1) * 100.0)
        begin = t0.min()
        rows[i].append({
            "event_us": ev[k][0].elapsed_time(ev[k][1]) * 1e3,
            "span_us": (t1.max() - begin) * TICK,
            "start_skew_us": (t0.max() - begin) * TICK,
            "prologue_us_med": float(np.median(ttab - t0)) * TICK,
            "body_us_med": float(np.median(tbody - ttab)) * TICK,
            "body_us_max": float((tbody - ttab).max()) * TICK,
            "body_end_spread_us": (tbody.max() - tbody.min()) * TICK,
            "reduce_tail_us": (t1.max() - tbody.max()) * TICK,
            "xcc_end_med_us": [round(float(np.median(tbody[xcc == x] - begin)) * TICK, 2) for x in range(8)],
            "clock_mhz_med": float(clk),
        })
for i, (n, lanes, rounds, force) in enumerate(runs):
    r_ = rows[i]
    agg = {key: round(float(np.median([r[key] for r in r_])), 2) for key in r_[0] if key != "xcc_end_med_us"}
    agg["xcc_end_med_us"] = [round(float(np.median([r["xcc_end_med_us"][x] for r in r_])), 2) for x in range(8)]
    print(json.dumps({"n": n, "lanes": lanes, "rounds": rounds, "chunk_forced": force, "launches": N * ROUNDS,
                      "same_crc": same[i], "GBps_event": round(n / agg["event_us"] / 1e3, 1),
                      "GBps_body_med": round(n / agg["body_us_med"] / 1e3, 1),
                      "frac_event": round(n / agg["event_us"] / 8e6, 4), **agg}), flush=True)
