#!/usr/bin/env python3
"""Does the persistent grid's static task split leave a tail? (bench-only probe)

Runs probe_crc_wave_times (libphoton_probes.so: the product's generic strided
CRC32C kernel with per-wave s_memrealtime stamps) on the C2 and C3 shapes with
static hand-out (= the product), all-ticket hand-out and static-then-tickets,
alternating variants over rounds. Prints per variant: kernel ms (median of
rounds, HIP events), GB/s, and for each launch the spread of wave end times
and the idle share = sum over waves of (last end - wave end) / (waves * span).
CRCs are checked equal to the product's batch call on the same buffers."""
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
P.probe_crc_wave_times.argtypes = [vp, u64, u64, vp, vp, vp, ci, ci, ci, ci, vp]
P.probe_crc_wave_times.restype = ci

st = torch.cuda.current_stream()
s = st.cuda_stream
cus = torch.cuda.get_device_properties(0).multi_processor_count
nw = cus * 16
t = torch.zeros(6 * nw, dtype=torch.int64, device="cuda")
ticket = torch.zeros(256, dtype=torch.int32, device="cuda")
rounds = int(os.environ.get("ROUNDS", "6"))


def launch(buf, n, cnt, out, g, mode, sr):
    rc = P.probe_crc_wave_times(buf.data_ptr(), n, cnt, out.data_ptr(), t.data_ptr(), ticket.data_ptr(),
                                g, mode, sr, cus, s)
    assert rc == 0, rc


def spread():
    v = t.cpu().numpy().reshape(-1, 6).astype(np.int64)
    v = v[v[:, 1] > 0]
    span = v[:, 1].max() - v[:, 0].min()
    idle = (v[:, 1].max() - v[:, 1]).sum() / (len(v) * span)
    return {"span_us": span / 100.0, "end_spread_us": (v[:, 1].max() - v[:, 1].min()) / 100.0,
            "start_spread_us": (v[:, 0].max() - v[:, 0].min()) / 100.0,
            "end_p10_us": float(np.percentile(v[:, 1].max() - v[:, 1], 90)) / 100.0, "idle_share": float(idle)}


def structure():
    """Where the slow waves sit (last launch): mean busy time (end - start, us)
    per XCC, per shader engine, per SIMD and per wave slot; and the spread of
    per-CU means."""
    v = t.cpu().numpy().reshape(-1, 6).astype(np.int64)
    v = v[v[:, 1] > 0]
    busy = (v[:, 1] - v[:, 0]) / 100.0
    hw, xcc = v[:, 2], v[:, 3] & 0xF
    simd, cu, se = (hw >> 4) & 3, (hw >> 8) & 0xF, (hw >> 13) & 7

    def by(key):
        return {int(k): round(float(busy[key == k].mean()), 1) for k in np.unique(key)}
    cu_key = xcc * 1024 + se * 64 + cu
    cu_means = np.array([busy[cu_key == k].mean() for k in np.unique(cu_key)])
    return {"busy_by_xcc": by(xcc), "busy_by_se": by(se), "busy_by_simd": by(simd),
            "cu_mean_min_max_us": [round(float(cu_means.min()), 1), round(float(cu_means.max()), 1)],
            "n_cus": int(len(cu_means)),
            "wave_busy_min_p50_max_us": [round(float(np.percentile(busy, p)), 1) for p in (0, 50, 100)]}


for name, n, cnt, g, static_opts in (("c2", 65536, 65536, 32, (6,)), ("c3", 4096, 1 << 20, 8, (28,))):
    buf = torch.empty(n * cnt, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(buf, n, n, cnt, 0x5EED0001)
    want = torch.zeros(cnt, dtype=torch.int32, device="cuda")
    ck.batch_strided(buf, n, n, cnt, want)
    out = torch.zeros(cnt, dtype=torch.int32, device="cuda")
    variants = [("static", 0, 0), ("static_rotated", 4, 0)] + [(f"static{r}+xcc_tickets", 3, r) for r in static_opts]
    res = {v[0]: {"ms": [], "spread": []} for v in variants}
    for rnd in range(rounds):
        order = variants if rnd % 2 == 0 else variants[::-1]
        for vname, mode, sr in order:
            for _ in range(3):
                launch(buf, n, cnt, out, g, mode, sr)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            a.record(st)
            for _ in range(reps):
                launch(buf, n, cnt, out, g, mode, sr)
            b.record(st)
            b.synchronize()
            res[vname]["ms"].append(a.elapsed_time(b) / reps)
            res[vname]["spread"].append(spread())
            if vname in ("static", "static_rotated") and rnd == 0:
                print(json.dumps({"config": name, "variant": vname, "structure": structure()}), flush=True)
            assert torch.equal(out, want), f"{name} {vname}: CRC mismatch"
            out.zero_()
    for vname, r in res.items():
        ms = float(np.median(r["ms"]))
        sp = {k: round(float(np.median([x[k] for x in r["spread"]])), 4) for k in r["spread"][0]}
        print(json.dumps({"config": name, "variant": vname, "ms": round(ms, 4),
                          "GBps": round(n * cnt / ms / 1e6, 1), "frac": round(n * cnt / ms / 1e6 / 8000, 4),
                          **sp}), flush=True)
    del buf
    torch.cuda.empty_cache()
