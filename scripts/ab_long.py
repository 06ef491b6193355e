#!/usr/bin/env python3
"""A/B of one long buffer (photon_crc32c_extend_device) across library builds
and long-kernel shapes in ONE process, interleaved rounds with alternating
order (DVFS moves the clock between processes and with launch history, so
only interleaved runs compare; cdna_hip_programming.md §5.4 rule 24).
Bench-only.

  LIBS      name=path,... of libphoton_checksum.so builds (default: new = in-tree)
  VARIANTS  name:lanes/rounds,... (0/0 = automatic); probe:lanes/rounds/chunk_kib[/abl]
            (the stamped probe build of the same long_run, libphoton_probes.so,
            with that chunk size forced; 0 = the plan's); "c64" (CRC-64/ECMA,
            photon_crc64ecma_extend_device, automatic shape) and "b64k64" (the
            CRC-64 batch kernel over the same bytes as 64 KiB pieces); "batch64k" (the
            strided batch kernel over the same bytes as 64 KiB pieces from an
            aligned base) and "read" (the read-only grid-stride stream)
  SIZES_MIB buffer sizes (at base+1, test_checksum.cpp:125-168)
  MID       1 (default) / 0: photon_crc_set_mid_kernel in every build (0: the
            long kernel for spans of up to 32 MiB too)
  LAUNCHES  back-to-back launches per variant per round, ROUNDS rounds (after
            WARM untimed interleaved rounds: under rocprofv3 every kernel then
            starts past the fill's DVFS dip, so the kernels' stats compare)
Prints one JSON line per (size, variant): mean / median ms over all launches,
frac of 8 TB/s; every variant's CRC must equal the first's."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from photonlibos_amd import checksum as ck  # noqa: E402

vp, u64, u32, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
libs = {}
for item in os.environ.get("LIBS", "new=" + os.path.join(REPO, "photonlibos_amd/lib/libphoton_checksum.so")).split(","):
    name, path = item.split("=", 1)
    lib = ctypes.CDLL(path if os.path.isabs(path) else os.path.join(REPO, path), mode=ctypes.RTLD_LOCAL)
    lib.photon_crc32c_extend_device.argtypes = [vp, u64, u32, vp, vp]
    lib.photon_crc32c_extend_device.restype = ci
    lib.photon_crc_set_long_shape.argtypes = [ci, ci]
    lib.photon_crc_set_long_shape.restype = ci
    if hasattr(lib, "photon_crc_set_mid_kernel"):  # MID=0: spans <= 32 MiB on the long kernel too
        lib.photon_crc_set_mid_kernel(int(os.environ.get("MID", "1")))
    libs[name] = lib
VARIANTS = os.environ.get("VARIANTS", "new:0/0,batch64k,read").split(",")
OFF = int(os.environ.get("OFF", "1"))  # buffer start offset from a 2 MiB-aligned allocation
P = ctypes.CDLL(os.path.join(REPO, "photonlibos_amd", "lib", "libphoton_probes.so"))
P.probe_long_stamped.argtypes = [vp, u64, u32, vp, vp, vp, ci, ci, ci, u64, vp, vp]
P.probe_long_stamped.restype = ci
cus = torch.cuda.get_device_properties(0).multi_processor_count
SIZES = [int(x) << 20 for x in os.environ.get("SIZES_MIB", "1024").split(",")]
N = int(os.environ.get("LAUNCHES", "10"))
ROUNDS = int(os.environ.get("ROUNDS", "6"))

st = torch.cuda.current_stream()
big = max(SIZES)
d = torch.empty(big + 4096, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(d, big + 4096, big + 4096, 1, 0x5EED0B00, stream=st)
out = torch.zeros(N, dtype=torch.int32, device="cuda")
out64 = torch.zeros(N, dtype=torch.int64, device="cuda")
pstate = torch.zeros(1024, dtype=torch.int32, device="cuda")
pstamps = torch.zeros(8 * 16 * cus, dtype=torch.int64, device="cuda")
pgrid = ctypes.c_int(0)
sink = torch.zeros(1 << 22, dtype=torch.int32, device="cuda")


def make(v, n):
    # "variant@OFFSET": that buffer start offset for this variant (default OFF;
    # batch64k: its pieces start at the offset, default 0)
    off = OFF
    if "@" in v:
        v, o = v.split("@")
        off = int(o)
    elif v in ("batch64k", "batchfold", "b64k64"):
        off = 0
    if v == "c64" or v.startswith("c64:"):  # c64[:lanes/rounds]
        lanes, rounds = (int(x) for x in v.split(":")[1].split("/")) if ":" in v else (0, 0)
        lib = next(iter(libs.values()))

        def fc64(k):
            lib.photon_crc_set_long_shape(lanes, rounds)
            ck.extend64_device(d.data_ptr() + off, n, out64[k:k + 1], seed=7, stream=st)
        return fc64
    if v.startswith("c64="):  # c64=<library path>[#lanes/rounds]: another build's CRC-64 extend_device
        # (same kernel names in two loaded builds: only builds with the same
        # kernel argument layout compare reliably)
        path = v.split("=", 1)[1]
        shape64 = (0, 0)
        if "#" in path:
            path, sh = path.split("#")
            shape64 = tuple(int(x) for x in sh.split("/"))
        l64 = ctypes.CDLL(path if os.path.isabs(path) else os.path.join(REPO, path), mode=ctypes.RTLD_LOCAL)
        l64.photon_crc64ecma_extend_device.argtypes = [vp, u64, ctypes.c_uint64, vp, vp]
        l64.photon_crc64ecma_extend_device.restype = ci
        l64.photon_crc_set_long_shape.argtypes = [ci, ci]
        l64.photon_crc_set_long_shape.restype = ci

        def f64(k):
            l64.photon_crc_set_long_shape(*shape64)
            rc = l64.photon_crc64ecma_extend_device(d.data_ptr() + off, n, 7, out64.data_ptr() + 8 * k,
                                                    ctypes.c_void_p(st.cuda_stream))
            assert rc == 0, (v, rc)
        return f64
    if v == "b64k64":
        pieces64 = torch.zeros(n >> 16, dtype=torch.int64, device="cuda")
        return lambda k: ck.batch64_strided(d.data_ptr() + off, 65536, 65536, (n - off) >> 16, pieces64, stream=st)
    if v == "read":
        return lambda k: ck.read_stream(d.data_ptr(), n, sink, sink.numel(), stream=st)
    if v in ("batch64k", "batchfold"):
        pieces = torch.zeros(n >> 16, dtype=torch.int32, device="cuda")
        cnt = (n - off) >> 16
        if v == "batch64k":
            return lambda k: ck.batch_strided(d.data_ptr() + off, 65536, 65536, cnt, pieces, stream=st)

        def bf(k):  # the pieces' CRCs folded by a second launch (combine_series)
            ck.batch_strided(d.data_ptr() + off, 65536, 65536, cnt, pieces, stream=st)
            ck.combine_series_device(pieces, 65536, cnt, out[k:k + 1], stream=st)
        return bf
    name, shape = v.split(":")
    if name in ("probe", "probe+ev"):
        # probe+ev: the same launch followed by a (timing-disabled) event
        # record on the stream, as the product's scratch lease does per call
        xev = torch.cuda.Event(enable_timing=False) if name == "probe+ev" else None
        parts = [int(x) for x in shape.split("/")]
        lanes, rounds, ckib = parts[:3]
        rounds |= (parts[3] if len(parts) > 3 else 0) << 8  # long_run ablation bits

        def fp(k):
            rc = P.probe_long_stamped(d.data_ptr() + off, n, 7, out.data_ptr() + 4 * k, pstate.data_ptr(),
                                      pstamps.data_ptr(), cus, lanes, rounds, ckib * 1024, ctypes.byref(pgrid),
                                      ctypes.c_void_p(st.cuda_stream))
            assert rc == 0, (v, rc)
            if xev is not None:
                xev.record(st)
        return fp
    lanes, rounds = (int(x) for x in shape.split("/"))
    lib = libs[name]

    def f(k):
        lib.photon_crc_set_long_shape(lanes, rounds)
        rc = lib.photon_crc32c_extend_device(d.data_ptr() + off, n, 7, out.data_ptr() + 4 * k,
                                             ctypes.c_void_p(st.cuda_stream))
        assert rc == 0, (v, rc)
    return f


WARM = int(os.environ.get("WARM", "0"))  # untimed interleaved rounds first (past the fill's DVFS dip)
for n in SIZES:
    fns = {v: make(v, n) for v in VARIANTS}
    for r in range(WARM):
        for v in (VARIANTS if r % 2 == 0 else VARIANTS[::-1]):
            for k in range(N):
                fns[v](k)
        torch.cuda.synchronize()
    times = {v: [] for v in VARIANTS}
    crcs = {}
    c64 = {}
    for r in range(ROUNDS):
        for v in (VARIANTS if r % 2 == 0 else VARIANTS[::-1]):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(N)]
            for k in range(N):
                ev[k][0].record(st)
                fns[v](k)
                ev[k][1].record(st)
            torch.cuda.synchronize()
            times[v] += [a.elapsed_time(b) for a, b in ev]
            if ":" in v and "@" not in v and not v.startswith("c64"):
                crcs.setdefault(v, set()).update(int(x) & 0xFFFFFFFF for x in out.cpu().numpy())
            if v.startswith("c64"):
                c64.setdefault(v, set()).update(int(x) & 0xFFFFFFFFFFFFFFFF for x in out64.cpu().numpy())
    for lib in libs.values():
        lib.photon_crc_set_long_shape(0, 0)
    ref = None
    for v in VARIANTS:
        t = np.array(times[v])
        row = {"n": n, "variant": v, "ms_mean": round(float(t.mean()), 4), "ms_median": round(float(np.median(t)), 4),
               "frac": round(n / float(t.mean()) / 8e9, 4), "launches": len(t)}
        if v in c64:
            row["same_crc"] = len(c64[v]) == 1 and c64[v] == next(iter(c64.values()))
        if v in crcs:
            ref = crcs[v] if ref is None else ref
            row["same_crc"] = len(crcs[v]) == 1 and crcs[v] == ref
        print(json.dumps(row), flush=True)
