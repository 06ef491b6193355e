#!/usr/bin/env python3
"""Where does a long-buffer launch spend its time? (bench-only probe)

long_stamped_kernel (libphoton_probes.so) is the product's
crc32c_long_kernel<64, 4> with per-wave s_memrealtime stamps at the start,
after the LDS table prologue, after the wave's chunks and after the
cross-workgroup reduce. For one buffer at base+1 (test_checksum.cpp:125-168)
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
P.probe_long_stamped.argtypes = [vp, u64, u32, u64, vp, vp, vp, ci, vp]
P.probe_long_stamped.restype = ci

N = int(os.environ.get("LAUNCHES", "30"))
SIZES = [int(x) << 20 for x in os.environ.get("SIZES_MIB", "64,256,1024").split(",")]
st = torch.cuda.current_stream()
cus = torch.cuda.get_device_properties(0).multi_processor_count
big = max(SIZES)
d = torch.empty(big + 4096, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(d, big + 4096, big + 4096, 1, 0x5EED0B00, stream=st)
out = torch.zeros(1, dtype=torch.int32, device="cuda")
want = torch.zeros(1, dtype=torch.int32, device="cuda")
state = torch.zeros(1024, dtype=torch.int32, device="cuda")
TICK = 1e-2  # s_memrealtime: 100 MHz -> 0.01 us

for n in SIZES:
    chunk = max(16384, ((n + 16 * cus - 1) // (16 * cus) + 4095) & ~4095)  # long_plan, 64 lanes, 1 round
    nch = (n + chunk - 1) // chunk
    nw = min(cus, (nch + 15) // 16) * 16
    ts = [torch.zeros(8 * nw, dtype=torch.int64, device="cuda") for _ in range(N)]
    base = d.data_ptr() + 1
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(N)]
    for k in range(N):
        ev[k][0].record(st)
        rc = P.probe_long_stamped(base, n, 7, chunk, out.data_ptr(), state.data_ptr(), ts[k].data_ptr(), cus,
                                  ctypes.c_void_p(st.cuda_stream))
        ev[k][1].record(st)
        assert rc == 0, rc
    torch.cuda.synchronize()
    ck.extend_device(base, n, 7, want, stream=st)
    torch.cuda.synchronize()
    same = int(out.item()) == int(want.item())
    rows = []
    for k in range(N // 2, N):
        t = ts[k].cpu().numpy().reshape(-1, 8).astype(np.int64)
        t = t[t[:, 3] > 0]
        t0, ttab, tbody, t1 = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
        xcc = t[:, 5] & 7
        clk = np.median((t[:, 7] - t[:, 6]) / np.maximum(t1 - t0, 1) * 100.0)
        begin = t0.min()
        rows.append({
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
    agg = {key: round(float(np.median([r[key] for r in rows])), 2) for key in rows[0] if key != "xcc_end_med_us"}
    agg["xcc_end_med_us"] = [round(float(np.median([r["xcc_end_med_us"][x] for r in rows])), 2) for x in range(8)]
    print(json.dumps({"n": n, "chunk": chunk, "chunks": nch, "waves": nw, "launches": N, "same_crc": same,
                      "GBps_event": round(n / agg["event_us"] / 1e3, 1), **agg}), flush=True)
