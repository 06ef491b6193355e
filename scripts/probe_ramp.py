#!/usr/bin/env python3
"""Start-up ramp of the C2 launch time: clock or kernel? (bench-only probe)

In a fresh process: fill the C2 batch (the bench's data generation), then
back-to-back launches of crc_wave_times_kernel (libphoton_probes.so: the
product's generic strided CRC32C kernel, G = 32, plus per-wave s_memtime /
s_memrealtime stamps) with HIP events around each launch. Per launch: event
ms, in-kernel shader clock (median over waves of d(s_memtime) / d(s_memrealtime)
x 100 MHz, MI355X_MICROARCH.md "DVFS give-back" item 6), wave-span, and the
median wave busy time in shader CYCLES (constant if the kernel does the same
work and only the clock moves). Then, after an idle pause, the same for the
product kernel itself (events only) and again for the probe.
Prints one JSON line per phase; CRCs are checked equal to the product's.

--kernel read | rows (the control): the same fresh-process
sequence with a READ-ONLY body carrying the same stamps -- `read`: the
product's read_stream_kernel (grid-stride, cus*8 x 256 threads), `rows`: the
CRC kernel's own lane-group row pattern (32 lanes x 4 rows, 512-byte rows,
persistent 1024-thread workgroups) with the CRC replaced by an XOR. If a
read-only body holds a higher clock than the CRC body over launches 5-25,
the CRC body's issue density costs the driver-run points."""
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

P = ctypes.CDLL(os.environ.get("PHOTON_CRC_PROBES") or os.path.join(REPO, "photonlibos_amd", "lib", "libphoton_probes.so"))
vp, u64, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
P.probe_crc_wave_times.argtypes = [vp, u64, u64, vp, vp, vp, ci, ci, ci, ci, vp]
P.probe_crc_wave_times.restype = ci
P.probe_read_stream_stamped.argtypes = [vp, u64, vp, vp, ci, vp]
P.probe_read_stream_stamped.restype = ci
P.probe_group_rows_stamped.argtypes = [vp, u64, u64, u64, vp, vp, ci, vp]
P.probe_group_rows_stamped.restype = ci
KERNEL = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "crc"
assert KERNEL in ("crc", "read", "rows"), KERNEL

N = int(os.environ.get("LAUNCHES", "40"))
st = torch.cuda.current_stream()
cus = torch.cuda.get_device_properties(0).multi_processor_count
nw = cus * 32 if KERNEL == "read" else cus * 16  # waves per launch (read: cus*8 blocks of 4 waves)
n, cnt = 65536, 65536
buf = torch.empty(n * cnt, dtype=torch.uint8, device="cuda")
ts = [torch.zeros(6 * nw, dtype=torch.int64, device="cuda") for _ in range(N)]
ticket = torch.zeros(256, dtype=torch.int32, device="cuda")
out = torch.zeros(cnt, dtype=torch.int32, device="cuda")
want = torch.zeros(cnt, dtype=torch.int32, device="cuda")


sink = torch.zeros(cus * 8 * 256 if KERNEL == "read" else cus * 1024, dtype=torch.int32, device="cuda")


def launch(k):
    if KERNEL == "read":
        return P.probe_read_stream_stamped(buf.data_ptr(), n * cnt, sink.data_ptr(), ts[k].data_ptr(), cus * 8,
                                           st.cuda_stream)
    if KERNEL == "rows":
        return P.probe_group_rows_stamped(buf.data_ptr(), n, n // 512, cnt, sink.data_ptr(), ts[k].data_ptr(), cus,
                                          st.cuda_stream)
    return P.probe_crc_wave_times(buf.data_ptr(), n, cnt, out.data_ptr(), ts[k].data_ptr(), ticket.data_ptr(),
                                  32, 0, 0, cus, st.cuda_stream)


def probe_phase(name):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(N)]
    for k in range(N):
        ev[k][0].record(st)
        rc = launch(k)
        assert rc == 0, rc
        ev[k][1].record(st)
    torch.cuda.synchronize()
    rows = []
    for k in range(N):
        v = ts[k].cpu().numpy().reshape(-1, 6).astype(np.int64)
        v = v[v[:, 1] > 0]
        dt = (v[:, 1] - v[:, 0]).astype(np.float64)
        dc = (v[:, 5] - v[:, 4]).astype(np.float64)
        rows.append({"ms": round(ev[k][0].elapsed_time(ev[k][1]), 4),
                     "clock_ghz": round(float(np.median(dc / dt)) * 0.1, 3),
                     "span_us": round(float(v[:, 1].max() - v[:, 0].min()) / 100.0, 1),
                     "wave_kcycles_median": round(float(np.median(dc)) / 1e3, 1)})
    print(json.dumps({"phase": name, "kernel": KERNEL, "launches": rows}), flush=True)
    return out.clone()


def product_phase(name):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(N)]
    for k in range(N):
        ev[k][0].record(st)
        ck.batch_strided(buf, n, n, cnt, out, stream=st)
        ev[k][1].record(st)
    torch.cuda.synchronize()
    print(json.dumps({"phase": name, "ms": [round(a.elapsed_time(b), 4) for a, b in ev]}), flush=True)


ck.fill_splitmix(buf, n, n, cnt, 0x5EED0001, stream=st)  # as bench.py: data generation, then launches
if KERNEL != "crc":
    probe_phase(f"fresh process, right after the fill: read-only control ({KERNEL}) + stamps")
    time.sleep(2.0)
    probe_phase(f"after 2 s idle: read-only control ({KERNEL}) + stamps")
    sys.exit(0)
first = probe_phase("fresh process, right after the fill: probe kernel (product kernel + stamps)")
ck.batch_strided(buf, n, n, cnt, want, stream=st)
torch.cuda.synchronize()
assert torch.equal(first, want), "probe CRCs differ from the product's"
time.sleep(2.0)
product_phase("after 2 s idle: product kernel")
time.sleep(2.0)
assert torch.equal(probe_phase("after 2 s idle: probe kernel"), want)
