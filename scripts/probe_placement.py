"""Does the payload's placement change a batch kernel's rate? (bench-only)

One process, one library: the C3-shape batch (1 Mi x 4 KiB, CRC-64 full-row
kernel by default, KIND=crc32 for CRC-32C) over several 4 GiB copies of the
same bytes at different device addresses, alternating blocks of launches so
that every copy sees the same power state. Prints one JSON line per copy:
base address modulo 2 MiB / 1 GiB and the median launch rate.

  ALLOCS=torch,hip,contig BLOCKS=6 PER=60 KIND=crc64|crc32 SHAPE=c3|c2|c5|c5_chain PRE_GIB=0 python scripts/probe_placement.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from photonlibos_amd import checksum as ck  # noqa: E402

GIB = 1 << 30
SHAPE = os.environ.get("SHAPE", "c3")
# c5 / c5_chain: 64 Ki messages x 8 scattered 8 KiB segments (bench.py's C5
# layout: a random permutation of the pool's slots), CRC-32C only
N, CNT = {"c2": (65536, 1 << 16), "c5": (8192, 1 << 19), "c5_chain": (8192, 1 << 19)}.get(SHAPE, (4096, 1 << 20))
NSEG = 8
BLOCKS = int(os.environ.get("BLOCKS", "6"))
PER = int(os.environ.get("PER", "60"))
KIND = os.environ.get("KIND", "crc64")
SKEW = int(os.environ.get("SKEW_KIB", "0")) << 10  # copy k starts k * SKEW past a 2 MiB boundary
PRE = int(os.environ.get("PRE_GIB", "0"))  # GiB allocated (and held) before the first copy
# how each copy is allocated: torch (caching allocator), hip (hipMalloc through
# the library's runtime, photon_crc_device_alloc), contig (hipExtMallocWithFlags
# hipDeviceMallocContiguous in that runtime)
ALLOCS = os.environ.get("ALLOCS", "torch,torch,torch").split(",")
COPIES = len(ALLOCS)
# engine settings compared on every copy, in the same process: VARIANTS is a
# comma list of specs, each '+'-joined tokens: lN (lanes per buffer), rN
# (generic-kernel rows per step), fMrN (CRC-64 full-row mode M, N rows), gN
# (workgroups of the persistent grid), d
# (the product default); LANES=8,16 is short for VARIANTS=l8,l16
LANES = os.environ.get("VARIANTS") or ",".join("l" + x for x in os.environ.get("LANES", "0").split(","))
LANES = LANES.split(",")


def apply(spec):
    ck.set_lanes_per_buffer(0)
    ck.set_generic_rows(-1)
    ck.set_full_rows64(3, 2)
    ck.lib().photon_crc_set_batch_grid(0)
    ck.set_msg_mode(0)
    ck.set_msg_rows(2)
    for t in spec.split("+"):
        if t.startswith("l"):
            ck.set_lanes_per_buffer(int(t[1:]))
        elif t.startswith("f"):
            m, r = t[1:].split("r")
            ck.set_full_rows64(int(m), int(r))
        elif t.startswith("r"):
            ck.set_generic_rows(int(t[1:]))
        elif t.startswith("g"):
            ck.lib().photon_crc_set_batch_grid(int(t[1:]))
        elif t.startswith("m"):  # mM: message form (0 auto, 1 one kernel, 2 segments + fold)
            ck.set_msg_mode(int(t[1:]))
        elif t.startswith("u"):  # uN: rows per step of the one-kernel message form
            ck.set_msg_rows(int(t[1:]))

st = torch.cuda.Stream()
bufs, outs, keep, msgs = [], [], [], []
if PRE:
    keep.append(torch.empty(PRE << 30, dtype=torch.uint8, device="cuda"))
hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime the library is linked to (already loaded)


class Dev:
    def __init__(self, p):
        self.p = p

    def data_ptr(self):
        return self.p


for k, how in enumerate(ALLOCS):
    size = N * CNT + (4 << 20)
    if how == "torch":
        raw = torch.empty(size, dtype=torch.uint8, device="cuda")
        base = raw.data_ptr()
    else:
        p = ctypes.c_void_p()
        if how == "hip":
            rc = ck.lib().photon_crc_device_alloc(ctypes.byref(p), ctypes.c_uint64(size))
        else:
            rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(size), ctypes.c_uint(4))
        assert rc == 0 and p.value, (how, rc)
        raw, base = p, p.value
    off = (-base) % (2 << 20) + k * SKEW
    view = Dev(base + off)
    ck.fill_splitmix(view, N, N, CNT, 0x5EED0003, stream=st)
    keep.append(raw)
    bufs.append(view)
    outs.append(torch.zeros(CNT, dtype=torch.int64 if KIND == "crc64" else torch.int32, device="cuda"))
    if SHAPE.startswith("c5"):
        perm = np.random.default_rng(0x5EED0005).permutation(CNT).astype(np.uint64)
        iov = np.empty((CNT, 2), np.uint64)
        iov[:, 0] = np.uint64(view.data_ptr()) + perm * np.uint64(N)
        iov[:, 1] = N
        msgs.append((torch.from_numpy(iov.view(np.int64)).cuda(),
                     torch.zeros(CNT // NSEG, dtype=torch.int32, device="cuda"),
                     torch.zeros(CNT, dtype=torch.int32, device="cuda") if SHAPE == "c5" else None))
torch.cuda.synchronize()


start = torch.from_numpy(np.arange(0, CNT + 1, NSEG, dtype=np.uint64).view(np.int64)).cuda()


def launch(k):
    if SHAPE.startswith("c5"):
        iov, mout, sout = msgs[k]
        ck.batch_msg_n(iov, start, CNT // NSEG, CNT, sout, mout, stream=st)
    elif KIND == "crc64":
        ck.batch64_strided(bufs[k], N, N, CNT, outs[k], stream=st)
    else:
        ck.batch_strided(bufs[k], N, N, CNT, outs[k], stream=st)


for k in range(COPIES):  # warm
    for _ in range(10):
        launch(k)
st.synchronize()
times = {(k, g): [] for k in range(COPIES) for g in LANES}
same = True
for b in range(BLOCKS):
    for k in range(COPIES):
        for g in LANES:
            apply(g)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(PER + 1)]
            with torch.cuda.stream(st):
                ev[0].record(st)
                for i in range(PER):
                    launch(k)
                    ev[i + 1].record(st)
            st.synchronize()
            times[(k, g)] += [ev[i].elapsed_time(ev[i + 1]) for i in range(PER)]
            if SHAPE.startswith("c5"):
                same = same and bool(torch.equal(msgs[k][1], msgs[0][1]))
            else:
                same = same and bool(torch.equal(outs[k], outs[0]))
apply("d")
for (k, g), tl in times.items():
    how = ALLOCS[k]
    ms = float(np.median(tl))
    print(json.dumps({"kind": KIND, "shape": SHAPE, "pre_gib": PRE, "copy": k, "alloc": how,
                      "variant": g, "base_mod_2MiB": bufs[k].data_ptr() % (2 << 20),
                      "base_mod_1GiB": bufs[k].data_ptr() % GIB, "base_hex": hex(bufs[k].data_ptr()),
                      "median_ms": round(ms, 4), "frac_of_8TBps": round(N * CNT / (ms * 1e-3) / 8e12, 4),
                      "same_crcs_everywhere": same}), flush=True)
