#!/usr/bin/env python3
"""Does giving the odd XCDs less work shorten a C2 launch? (bench-only probe.)
crc_wave_times_kernel (the product's batch body + stamps, probes.hip) over
the C2 batch (64 Ki x 64 KiB, 32 lanes): MODE 0 = the product's static
split; MODE 5:E = even XCDs take ntask/2 * (1 + E/1000) wave tasks, odd XCDs
the rest. Interleaved rounds in one process, after a 3 s warm-up so the
clock has settled; per variant the median launch (HIP events), the per-XCC
median of wave end times and the last wave end. Same CRCs checked."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from photonlibos_amd import checksum as ck  # noqa: E402

P = ctypes.CDLL(os.path.join(REPO, "photonlibos_amd", "lib", "libphoton_probes.so"))
vp, u64, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
P.probe_crc_wave_times.argtypes = [vp, u64, u64, vp, vp, vp, ci, ci, ci, ci, vp]
P.probe_crc_wave_times.restype = ci

st = torch.cuda.current_stream()
cus = torch.cuda.get_device_properties(0).multi_processor_count
n, cnt = 65536, 65536
VARIANTS = os.environ.get("VARIANTS", "0,5:0,5:20,5:40,5:60,5:90").split(",")
N = int(os.environ.get("LAUNCHES", "10"))
ROUNDS = int(os.environ.get("ROUNDS", "6"))
buf = torch.empty(n * cnt, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(buf, n, n, cnt, 0x5EED0001, stream=st)
outs = {v: torch.zeros(cnt, dtype=torch.int32, device="cuda") for v in VARIANTS}
ticket = torch.zeros(256, dtype=torch.int32, device="cuda")
ts = [torch.zeros(6 * cus * 16, dtype=torch.int64, device="cuda") for _ in range(N)]


def run(v, k):
    mode, e = (int(x) for x in v.split(":")) if ":" in v else (int(v), 0)
    rc = P.probe_crc_wave_times(buf.data_ptr(), n, cnt, outs[v].data_ptr(), ts[k].data_ptr(), ticket.data_ptr(), 32,
                                mode, e, cus, ctypes.c_void_p(st.cuda_stream))
    assert rc == 0, (v, rc)


t_end = time.time() + 3.0
while time.time() < t_end:  # settle the clock
    for k in range(10):
        run("0", k)
    torch.cuda.synchronize()

res = {v: {"ms": [], "xcc": [], "last": []} for v in VARIANTS}
for r in range(ROUNDS):
    for v in (VARIANTS if r % 2 == 0 else VARIANTS[::-1]):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(N + 1)]
        ev[0].record(st)
        for k in range(N):
            run(v, k)
            ev[k + 1].record(st)
        torch.cuda.synchronize()
        for k in range(N):
            res[v]["ms"].append(ev[k].elapsed_time(ev[k + 1]))
            t = ts[k].cpu().numpy().reshape(-1, 6).astype(np.int64)
            t = t[t[:, 1] > 0]
            b = t[:, 0].min()
            x = t[:, 3] & 7
            end = (t[:, 1] - b) / 100.0
            res[v]["xcc"].append([float(np.max(end[x == i])) if (x == i).any() else 0.0 for i in range(8)])
            res[v]["last"].append(float(end.max()))
ref = outs[VARIANTS[0]]
for v in VARIANTS:
    r = res[v]
    print(json.dumps({"variant": v, "launch_ms_median": round(float(np.median(r["ms"])), 4),
                      "frac_median": round(n * cnt / (float(np.median(r["ms"])) * 1e-3) / 8e12, 4),
                      "last_wave_end_us": round(float(np.median(r["last"])), 1),
                      "xcc_last_end_us": [round(float(np.median([a[i] for a in r["xcc"]])), 1) for i in range(8)],
                      "same_crc": bool(torch.equal(outs[v], ref))}), flush=True)
