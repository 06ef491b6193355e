"""BASELINE configs at their FULL sizes, every CRC checked bit-exactly against
the pinned oracle (VERDICT r2 "next" #1).

The device payload is generated on the GPU (the bench's splitmix streams and
C5 permutation), run through the C-ABI exactly as bench.py runs it, copied to
the host once, and the oracle's C restatement (oracle/crc_oracle.c,
slicing-by-8 = crc.cpp:77-117) checks every buffer / segment / message on a
thread pool. At these counts every wave of the persistent grid (256 CUs x 16
waves) runs its full number of rounds -- C2: 2 buffers per wave task, 8
rounds; C3: 4 per task, 64 rounds; C5: 8 messages per task, 2 rounds (the
count the held-back segment stores are built around); C4 shard: 1 per task,
8 rounds -- which the reduced-count tests in test_gpu_parity.py do not reach.

Reference shapes: common/checksum/test/test_checksum.cpp:231-266 (properties),
rpc/serialize.h:244-251 (Crc32Hasher: chained crc32c_extend per message)."""
import os

import numpy as np
import pytest

from photonlibos_amd import checksum as ck

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

SEED_BASE = 0x5EED0001  # bench.py shard_seed_base(0, count)


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    assert ck.device_count() >= 1
    yield torch
    torch.cuda.empty_cache()


@pytest.fixture(autouse=True)
def _reset():
    yield
    ck.set_lanes_per_buffer(0)
    ck.set_msg_mode(0)


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def _strided(torch, d, nbytes, count, seed=0):
    out = torch.zeros(count, dtype=torch.int32, device="cuda")
    ck.batch_strided(d, nbytes, nbytes, count, out, seed=seed)
    torch.cuda.synchronize()
    return _u32(out)


def _first_mismatch(got, want):
    bad = np.flatnonzero(got != want)
    return None if bad.size == 0 else (int(bad[0]), int(bad.size))


@pytest.mark.parametrize("cfg", ["c2", "c3"])
def test_full_strided_every_crc(torch_dev, oracle, cfg):
    # C2: 65,536 x 64 KiB (lanes 32, 4 rows/step); C3: 1,048,576 x 4 KiB
    # (lanes 16, 2 rows/step): all 4 GiB, every CRC vs the oracle, with seed
    # 0 (crc32c) and an all-ones seed (crc32c_extend, crc32c.h:30-33).
    torch = torch_dev
    nbytes, count = (65536, 65536) if cfg == "c2" else (4096, 1 << 20)
    d = torch.empty(nbytes * count, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, nbytes, nbytes, count, SEED_BASE)
    host = d.cpu().numpy()
    for seed in (0, 0xFFFFFFFF):
        got = _strided(torch, d, nbytes, count, seed)
        want = oracle.crc32c_strided(host, nbytes, nbytes, count, seed)
        assert _first_mismatch(got, want) is None, (cfg, seed, _first_mismatch(got, want))
    del d, host


def test_full_c3_crc64_every_crc(torch_dev, oracle):
    # CRC-64/ECMA (row f2) on the C3 shape at full size: the product's
    # path (crc64_full_kernel<8,2,true> since round 6: 4-8 KiB uniform
    # batches take 8 lanes) and the 16-lane one (lanes override; the
    # default before round 6), every CRC of both against the oracle.
    torch = torch_dev
    nbytes, count = 4096, 1 << 20
    d = torch.empty(nbytes * count, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, nbytes, nbytes, count, SEED_BASE)
    want = oracle.crc64ecma_strided(d.cpu().numpy(), nbytes, nbytes, count)
    assert ck.lanes_for(nbytes) in (8, 16)
    for lanes in (0, 16):
        ck.set_lanes_per_buffer(lanes)
        try:
            out = torch.zeros(count, dtype=torch.int64, device="cuda")
            ck.batch64_strided(d, nbytes, nbytes, count, out)
            torch.cuda.synchronize()
        finally:
            ck.set_lanes_per_buffer(0)
        got = out.cpu().numpy().view(np.uint64)
        assert _first_mismatch(got, want) is None, (lanes, _first_mismatch(got, want))


def test_full_c5_every_segment_and_message(torch_dev, oracle):
    # C5 as bench.py builds it: 65,536 messages x 8 segments of 8 KiB at the
    # permuted slots of a 524,288-slot pool, per-message seeds. Checked: every
    # segment CRC and every message CRC of the default one-kernel form with
    # segment CRCs (crc32c_batch_kernel<8,2,2>), every message CRC of the
    # chained form (<8,2,1>, no segment CRCs) and of the two-kernel form.
    torch = torch_dev
    n, nmsg, nseg = 8192, 65536, 8
    slots = nmsg * nseg
    d = torch.empty(n * slots, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, n, n, slots, SEED_BASE)
    perm = np.random.default_rng(0x5EED0005).permutation(slots).astype(np.uint64)
    iov = np.empty((slots, 2), np.uint64)
    iov[:, 0] = np.uint64(d.data_ptr()) + perm * np.uint64(n)
    iov[:, 1] = n
    start = np.arange(0, slots + 1, nseg, dtype=np.uint64)
    seeds = (np.arange(nmsg, dtype=np.uint64) * np.uint64(2654435761) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    d_iov = torch.from_numpy(iov.view(np.int64).copy()).cuda()
    d_start = torch.from_numpy(start.view(np.int64).copy()).cuda()
    d_seeds = torch.from_numpy(seeds.view(np.int32).copy()).cuda()

    host = d.cpu().numpy()
    hiov = iov.copy()
    hiov[:, 0] = np.uint64(host.ctypes.data) + perm * np.uint64(n)
    want_seg = oracle.crc32c_iov(hiov)
    want_msg = oracle.msg_chain(hiov, start, seeds)

    seg_out = torch.zeros(slots, dtype=torch.int32, device="cuda")
    out = torch.zeros(nmsg, dtype=torch.int32, device="cuda")
    ck.batch_msg_n(d_iov, d_start, nmsg, slots, seg_out, out, seeds=d_seeds)  # default: <8,2,2>
    torch.cuda.synchronize()
    assert _first_mismatch(_u32(seg_out), want_seg) is None, ("segments", _first_mismatch(_u32(seg_out), want_seg))
    assert _first_mismatch(_u32(out), want_msg) is None, ("messages", _first_mismatch(_u32(out), want_msg))

    chained = torch.zeros(nmsg, dtype=torch.int32, device="cuda")
    ck.batch_msg_n(d_iov, d_start, nmsg, slots, None, chained, seeds=d_seeds)  # <8,2,1>
    torch.cuda.synchronize()
    assert _first_mismatch(_u32(chained), want_msg) is None, ("chained", _first_mismatch(_u32(chained), want_msg))

    ck.set_msg_mode(2)  # segment kernel + fold kernel
    two = torch.zeros(nmsg, dtype=torch.int32, device="cuda")
    seg2 = torch.zeros(slots, dtype=torch.int32, device="cuda")
    ck.batch_msg_n(d_iov, d_start, nmsg, slots, seg2, two, seeds=d_seeds)
    torch.cuda.synchronize()
    assert np.array_equal(_u32(seg2), want_seg) and np.array_equal(_u32(two), want_msg)
    del d, host


def test_full_c4_shard_every_crc(torch_dev, oracle):
    # The C4 shard one GPU runs at 8 GPUs: 32,768 x 1 MiB = 32 GiB (rank 0's
    # global ids). Two engine shapes (64 lanes, the default, and 32 lanes) agree
    # on every CRC, and every CRC equals the oracle (checked in 4 GiB host
    # chunks to bound host memory).
    torch = torch_dev
    nbytes, count = 1 << 20, 32768
    d = torch.empty(nbytes * count, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, nbytes, nbytes, count, SEED_BASE)
    a = _strided(torch, d, nbytes, count)
    assert ck.lanes_for(nbytes) == 64
    ck.set_lanes_per_buffer(32)
    b = _strided(torch, d, nbytes, count)
    ck.set_lanes_per_buffer(0)
    assert _first_mismatch(a, b) is None, _first_mismatch(a, b)
    per = 4096
    for lo in range(0, count, per):
        host = d[lo * nbytes:(lo + per) * nbytes].cpu().numpy()
        want = oracle.crc32c_strided(host, nbytes, nbytes, per)
        assert _first_mismatch(a[lo:lo + per], want) is None, (lo, _first_mismatch(a[lo:lo + per], want))
    del d


# ------------------------------------------------- one long buffer (row f3)
# photon_crc32c_extend_device / photon_crc64ecma_extend_device: one launch,
# chunks of the buffer one per wavefront, XOR-combined by workgroup atomics.
# The reference's own perf shape (test_checksum.cpp:125-168: one 128 KiB and
# one 1 GiB buffer at buf+1) and every edge of the chunk plan.

def _extend(torch, d, off, n, seed, crc64=False):
    if crc64:
        out = torch.zeros(1, dtype=torch.int64, device="cuda")
        ck.extend64_device(d.data_ptr() + off, n, out, seed=seed)
        torch.cuda.synchronize()
        return int(out.cpu().numpy().view(np.uint64)[0])
    out = torch.zeros(1, dtype=torch.int32, device="cuda")
    ck.extend_device(d.data_ptr() + off, n, seed, out)
    torch.cuda.synchronize()
    return int(_u32(out)[0])


@pytest.mark.parametrize("n", [128 << 10, 1 << 30])
def test_extend_device_reference_perf_shape(torch_dev, oracle, n):
    torch = torch_dev
    d = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, n + 64, n + 64, 1, 0x5EED0600)
    host = d.cpu().numpy()[1:1 + n]
    for seed in (0, 0xFFFFFFFF):
        assert _extend(torch, d, 1, n, seed) == oracle.crc32c(host, seed), (n, seed)
    if n <= (128 << 10):
        assert _extend(torch, d, 1, n, 7, True) == oracle.crc64ecma(host, 7)
    del d


@pytest.mark.parametrize("mid", [True, False])
def test_extend_device_plan_edges(torch_dev, oracle, mid):
    # Chunk-plan edges: one chunk, the one-workgroup limit (256 KiB, 16
    # chunks) and one byte past it, T at multiples of 16 waves +- 1, the
    # 16-KiB-chunk limit of a full grid (64 MiB) +- a few bytes, odd sizes;
    # offsets 0, 1, 15; seeds; CRC-32C and CRC-64. Each call also leaves its
    # accumulator state zeroed for the next one (repeated calls agree). With
    # the mid kernel on (the default) spans up to 16 MiB take the mid layout;
    # off, every span over 256 KiB takes the long kernel.
    torch = torch_dev
    ck.set_mid_kernel(mid)
    try:
        _plan_edges(torch, oracle)
    finally:
        ck.set_mid_kernel(True)


def _plan_edges(torch, oracle):
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    big = 16 * cus * (16 << 10)
    sizes = [0, 1, 15, 64, 4095, 4096, 4097, 65536 + 3, (256 << 10) - 1, 256 << 10, (256 << 10) + 1,
             (256 << 10) + 16385, 17 * (16 << 10), 33 * (16 << 10) + 5, big - 1, big, big + 7, 3 * big + 12345]
    d = torch.empty(max(sizes) + 64, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, d.numel(), d.numel(), 1, 0x5EED0700)
    host = d.cpu().numpy()
    for k, n in enumerate(sizes):
        off = (0, 1, 15)[k % 3]
        seed = (k * 0x9E3779B1) & 0xFFFFFFFF
        want = oracle.crc32c(host[off:off + n], seed)
        assert _extend(torch, d, off, n, seed) == want, (n, off)
        assert _extend(torch, d, off, n, seed) == want, ("repeat", n, off)
        if n <= (1 << 20):
            s64 = seed * 0x100000001
            assert _extend(torch, d, off, n, s64, True) == oracle.crc64ecma(host[off:off + n], s64), (n, off)
    n = big + 7  # CRC-64 on a full grid of chunks
    assert _extend(torch, d, 3, n, 5, True) == oracle.crc64ecma(host[3:3 + n], 5)
    del d


def test_extend_device_concurrent_streams(torch_dev, oracle):
    # Eight streams each run long-buffer calls at once: every call leases its
    # own accumulator (scratch_alloc(zeroed)), results stay exact.
    torch = torch_dev
    n = (40 << 20) + 11
    d = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, n + 64, n + 64, 1, 0x5EED0800)
    host = d.cpu().numpy()
    streams = [torch.cuda.Stream() for _ in range(8)]
    outs = [torch.zeros(4, dtype=torch.int32, device="cuda") for _ in streams]
    torch.cuda.synchronize()
    for r in range(4):
        for k, (s, o) in enumerate(zip(streams, outs)):
            ck.extend_device(d.data_ptr() + k, n - 8 * k, r + k, o[r:r + 1], stream=s)
    torch.cuda.synchronize()
    for k, o in enumerate(outs):
        got = _u32(o)
        for r in range(4):
            assert int(got[r]) == oracle.crc32c(host[k:k + n - 8 * k], r + k), (k, r)
    del d


def test_extend_device_small_path_edges(torch_dev, oracle):
    """The one-workgroup latency kernel (crc32c_small_kernel: block span <=
    256 KiB, tables copied from the device image): every length 0..259 at
    every start offset 0..15 with a seed (seeds over fewer than 4 data bytes,
    heads and tails in one block), random lengths, and the span limit
    itself: 256 KiB spans at offsets 0 and 15 (the last small case / the
    first long one), all against the oracle."""
    torch = torch_dev
    n_max = (256 << 10) + 64
    d = torch.empty(n_max + 64, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, d.numel(), d.numel(), 1, 0x5EED0D00)
    host = d.cpu().numpy()
    base = (-d.data_ptr()) % 16  # offset of a 16-byte-aligned address
    out = torch.zeros(260 * 16, dtype=torch.int32, device="cuda")
    cases = []
    for n in range(260):
        for off in range(16):
            cases.append((base + off, n, (n * 0x9E3779B1 + off) & 0xFFFFFFFF))
    rng = np.random.default_rng(0x5EED0D01)
    for _ in range(200):
        n = int(rng.integers(260, 256 << 10))
        cases.append((base + int(rng.integers(0, 16)), n, int(rng.integers(0, 1 << 32))))
    span = 256 << 10
    cases += [(base, span, 1), (base + 15, span - 15, 2), (base + 15, span - 14, 3), (base, span + 1, 4),
              (base + 1, span - 4, 5), (base + 12, span - 16, 6)]
    for k0 in range(0, len(cases), out.numel()):
        part = cases[k0:k0 + out.numel()]
        for k, (off, n, seed) in enumerate(part):
            ck.extend_device(d.data_ptr() + off, n, seed, out[k:k + 1])
        torch.cuda.synchronize()
        got = _u32(out)
        for k, (off, n, seed) in enumerate(part):
            assert int(got[k]) == oracle.crc32c(host[off:off + n], seed), (off - base, n, seed)


def test_extend64_device_small_path_edges(torch_dev, oracle):
    """crc64_small_kernel (CRC-64/ECMA, block span <= 256 KiB): every length
    0..139 at every start offset 0..15 with a 64-bit seed (inits over fewer
    than 8 data bytes, heads and tails in one block), random lengths, and the
    span limit at offsets 0 and 15, all against the oracle."""
    torch = torch_dev
    n_max = (256 << 10) + 64
    d = torch.empty(n_max + 64, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, d.numel(), d.numel(), 1, 0x5EED0D64)
    host = d.cpu().numpy()
    base = (-d.data_ptr()) % 16
    out = torch.zeros(140 * 16, dtype=torch.int64, device="cuda")
    cases = []
    for n in range(140):
        for off in range(16):
            cases.append((base + off, n, (n * 0x9E3779B97F4A7C15 + off) & 0xFFFFFFFFFFFFFFFF))
    rng = np.random.default_rng(0x5EED0D65)
    for _ in range(150):
        n = int(rng.integers(140, 256 << 10))
        cases.append((base + int(rng.integers(0, 16)), n, int(rng.integers(0, 1 << 63)) * 2 + 1))
    span = 256 << 10
    cases += [(base, span, 1), (base + 15, span - 15, 2), (base + 15, span - 14, 3), (base, span + 1, 4),
              (base + 1, 128 << 10, 5), (base + 12, span - 16, 6)]
    for k0 in range(0, len(cases), out.numel()):
        part = cases[k0:k0 + out.numel()]
        for k, (off, n, seed) in enumerate(part):
            ck.extend64_device(d.data_ptr() + off, n, out[k:k + 1], seed=seed)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint64)
        for k, (off, n, seed) in enumerate(part):
            assert int(got[k]) == oracle.crc64ecma(host[off:off + n], seed), (off - base, n, hex(seed))


MID_LANES = 512 * 256  # crc32c_kernels.h kMidWg * 256


@pytest.mark.parametrize("crc64", [False, True])
def test_extend_device_mid_path_edges(torch_dev, oracle, crc64):
    """The mid layout (crc32c_small_kernel / crc64_small_kernel over 512
    workgroups, spans over 256 KiB up to 16 MiB): one byte
    over the small limit, every row count at its boundaries (+-1 block, at
    offsets 0, 1, 15), the span limit and one byte past it (the long kernel),
    random sizes and seeds; calls queued back to back on one stream (one
    reduce state), all against the oracle."""
    torch = torch_dev
    row = MID_LANES * 16
    rows_max = 8  # crc32c_kernels.h kMidRows: the long kernel past 16 MiB
    cap = rows_max * row + 64
    d = torch.empty(cap, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, cap, cap, 1, 0x5EED0E00 + crc64)
    host = d.cpu().numpy()
    base = (-d.data_ptr()) % 16
    cover = 8 if crc64 else 4
    cases = [(base + 1, (256 << 10), 1), (base, (256 << 10) + 1, 2), (base + 15, row - 15, 3),
             (base, rows_max * row, 4), (base + 1, rows_max * row - 1, 5), (base + 3, rows_max * row - 2, 6),
             (base, rows_max * row + 1, 7), (base + 9, 3 * row + 12345, 8)]
    for k in range(1, rows_max):
        for off, dn in ((0, 0), (1, 1), (15, -15), (0, 16), (7, -16 - 7)):
            cases.append((base + off, k * row + dn, k * 0x9E3779B1 + off))
    rng = np.random.default_rng(0x5EED0E01 + crc64)
    for _ in range(24):
        cases.append((base + int(rng.integers(0, 16)), int(rng.integers(256 << 10, rows_max * row - 16)),
                      int(rng.integers(0, 1 << 62))))
    cases = [(o, n, s) for o, n, s in cases if o + max(n, cover) <= cap - 16]
    if crc64:
        out = torch.zeros(len(cases), dtype=torch.int64, device="cuda")
        for k, (off, n, seed) in enumerate(cases):
            ck.extend64_device(d.data_ptr() + off, n, out[k:k + 1], seed=seed)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint64)
        for k, (off, n, seed) in enumerate(cases):
            assert int(got[k]) == oracle.crc64ecma(host[off:off + n], seed), (off - base, n, hex(seed))
    else:
        out = torch.zeros(len(cases), dtype=torch.int32, device="cuda")
        for k, (off, n, seed) in enumerate(cases):
            ck.extend_device(d.data_ptr() + off, n, seed & 0xFFFFFFFF, out[k:k + 1])
        torch.cuda.synchronize()
        got = _u32(out)
        for k, (off, n, seed) in enumerate(cases):
            assert int(got[k]) == oracle.crc32c(host[off:off + n], seed & 0xFFFFFFFF), (off - base, n, seed)
    del d


def test_extend_device_thousand_back_to_back_launches(torch_dev, oracle):
    """the fence-free cross-workgroup reduce (long_reduce)
    reused by 1,000 back-to-back full-grid launches on ONE stream (one state:
    ticket + per-workgroup slots), consecutive launches over DIFFERENT data
    (8 buffers of 64-72 MiB at odd offsets, cycled, with a new seed each
    launch), so a slot read before its store landed, or a stale slot of the
    previous launch, gives a wrong CRC. Every result is checked against the
    oracle: CRC(buffer j, seed) = crc32c_combine(seed, CRC(buffer j, 0), n_j)
    (linearity, crc.cpp:393-405), the 8 base CRCs computed on the host."""
    torch = torch_dev
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    nbuf, launches = 8, 1000
    lens = [(64 << 20) + j * (1 << 20) + 4099 * j + 1 for j in range(nbuf)]
    offs = [1 + 7 * j for j in range(nbuf)]
    bufs = []
    for j in range(nbuf):
        b = torch.empty(lens[j] + 64, dtype=torch.uint8, device="cuda")
        ck.fill_splitmix(b, b.numel(), b.numel(), 1, 0x5EED0B00 + j)
        bufs.append(b)
    base = [oracle.crc32c(bufs[j].cpu().numpy()[offs[j]:offs[j] + lens[j]], 0) for j in range(nbuf)]
    rng = np.random.default_rng(0x5EED0B10)
    seeds = [int(x) for x in rng.integers(1, 1 << 32, launches, dtype=np.uint64)]
    out = torch.zeros(launches, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    torch.cuda.synchronize()
    for k in range(launches):
        j = k % nbuf
        ck.extend_device(bufs[j].data_ptr() + offs[j], lens[j], seeds[k], out[k:k + 1], stream=st)
    torch.cuda.synchronize()
    got = _u32(out)
    # every launch filled the grid (the 16 KiB chunk floor: >= 16 waves x cus chunks)
    assert min(lens) >= 16 * cus * (16 << 10)
    for k in range(launches):
        j = k % nbuf
        assert int(got[k]) == oracle.combine(seeds[k], base[j], lens[j]), (k, j)
    del bufs


@pytest.mark.parametrize("mid", [True, False])
def test_extend_device_graph_capture(torch_dev, oracle, mid):
    """every extend_device call captures into a HIP graph -- a
    one-workgroup call, a multi-workgroup small-kernel call (128 KiB) and a
    full-grid long-kernel call (1 MiB) -- each multi-workgroup launch with a
    reduce state owned by the graph (reset mode), so the graph replays exactly
    any number of times over new data; the stream runs long calls on its own
    state again after the capture, and destroying the graph hands the states
    back for the next capture."""
    torch = torch_dev
    ck.set_mid_kernel(mid)  # the 1 MiB span: the mid layout's 256 workgroups, or the long kernel
    try:
        _graph_capture(torch, oracle)
    finally:
        ck.set_mid_kernel(True)


def _graph_capture(torch, oracle):
    d = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, d.numel(), d.numel(), 1, 0x5EED0C00)
    spans = ((3, 3000), (3, 128 << 10), (3, (1 << 20) - 64))
    for rep in range(2):  # the second capture reuses the states the first graph handed back
        out = torch.zeros(3, dtype=torch.int32, device="cuda")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            st = torch.cuda.current_stream()
            for k, (off, n) in enumerate(spans):
                ck.extend_device(d.data_ptr() + off, n, 9 + k, out[k:k + 1], stream=st)
        for seed_fill in (0x5EED0C01, 0x5EED0C02, 0x5EED0C01):  # new data, same graph, replayed thrice
            ck.fill_splitmix(d, d.numel(), d.numel(), 1, seed_fill + rep)
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            host = d.cpu().numpy()
            for k, (off, n) in enumerate(spans):
                assert int(_u32(out)[k]) == oracle.crc32c(host[off:off + n], 9 + k), (rep, k)
        del g
    out = torch.zeros(1, dtype=torch.int32, device="cuda")
    ck.extend_device(d.data_ptr() + 3, (1 << 20) - 64, 9, out)
    torch.cuda.synchronize()
    assert int(_u32(out)[0]) == oracle.crc32c(d.cpu().numpy()[3:3 + (1 << 20) - 64], 9)
    # CRC-64 (crc64_small_kernel and crc64_long_kernel): the same rule
    out64 = torch.zeros(3, dtype=torch.int64, device="cuda")
    g64 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g64):
        st = torch.cuda.current_stream()
        for k, (off, n) in enumerate(spans):
            ck.extend64_device(d.data_ptr() + off + 2, n, out64[k:k + 1], seed=11 + k, stream=st)
    for seed_fill in (0x5EED0C03, 0x5EED0C04):
        ck.fill_splitmix(d, d.numel(), d.numel(), 1, seed_fill)
        torch.cuda.synchronize()
        g64.replay()
        torch.cuda.synchronize()
        host = d.cpu().numpy()
        got = out64.cpu().numpy().view(np.uint64)
        for k, (off, n) in enumerate(spans):
            assert int(got[k]) == oracle.crc64ecma(host[off + 2:off + 2 + n], 11 + k), k


def test_two_live_graphs_replay_concurrently(torch_dev, oracle):
    """a captured multi-workgroup launch owns a reduce state through
    a graph user object, handed back when the graph is destroyed; torch
    destroys the hipGraph_t right after instantiation, so the executable graph
    must keep its own reference. Two graphs stay alive -- the second captured
    after the first's hipGraph_t is gone -- and replay at the same time on two
    streams, many times, over spans that take many workgroups (small 128 KiB,
    mid / long 1 MiB): a shared state would mix their tickets and slots and
    give wrong CRCs."""
    torch = torch_dev
    bufs = [torch.empty(1 << 20, dtype=torch.uint8, device="cuda") for _ in range(2)]
    for i, b in enumerate(bufs):
        ck.fill_splitmix(b, b.numel(), b.numel(), 1, 0x6A0 + i)
    torch.cuda.synchronize()
    spans = ((3, 128 << 10), (3, (1 << 20) - 64), (1, 200000))
    outs = [torch.zeros(len(spans), dtype=torch.int32, device="cuda") for _ in range(2)]
    graphs = []
    for i in range(2):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            st = torch.cuda.current_stream()
            for k, (off, n) in enumerate(spans):
                ck.extend_device(bufs[i].data_ptr() + off, n, 40 + k, outs[i][k:k + 1], stream=st)
        graphs.append(g)
    hosts = [b.cpu().numpy() for b in bufs]
    want = [[oracle.crc32c(h[off:off + n], 40 + k) for k, (off, n) in enumerate(spans)] for h in hosts]
    streams = [torch.cuda.Stream() for _ in range(2)]
    torch.cuda.synchronize()
    for rep in range(150):
        for i in range(2):
            outs[i].zero_()
        torch.cuda.synchronize()
        for i in range(2):
            with torch.cuda.stream(streams[i]):
                graphs[i].replay()
        torch.cuda.synchronize()
        for i in range(2):
            got = [int(x) for x in _u32(outs[i])]
            assert got == want[i], (rep, i, got, want[i])


def test_first_small_call_inside_capture(torch_dev):
    """the small kernels' table images are built lazily on
    a device's first small call; when that first call is made while the
    caller's stream is being captured, the build runs in relaxed capture mode
    and the capture stays valid. Needs a fresh process (the images are per
    process)."""
    import subprocess
    import sys
    code = r"""
import sys, numpy as np, torch
sys.path.insert(0, %r)
from photonlibos_amd import checksum as ck
from tests import _oracle as oracle
d = torch.empty(1 << 18, dtype=torch.uint8, device="cuda")
ck.fill_splitmix(d, d.numel(), d.numel(), 1, 0x5EED0D00)
out = torch.zeros(2, dtype=torch.int32, device="cuda")
out64 = torch.zeros(1, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    st = torch.cuda.current_stream()
    ck.extend_device(d.data_ptr() + 1, 5000, 3, out[0:1], stream=st)
    ck.extend_device(d.data_ptr() + 1, 100000, 4, out[1:2], stream=st)
    ck.extend64_device(d.data_ptr() + 1, 5000, out64, seed=5, stream=st)
g.replay()
torch.cuda.synchronize()
h = d.cpu().numpy()
got = out.cpu().numpy().view(np.uint32)
assert int(got[0]) == oracle.crc32c(h[1:5001], 3)
assert int(got[1]) == oracle.crc32c(h[1:100001], 4)
assert int(out64.cpu().numpy().view(np.uint64)[0]) == oracle.crc64ecma(h[1:5001], 5)
print("ok")
""" % (REPO,)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.stdout[-2000:], r.stderr[-4000:])


@pytest.mark.parametrize("shape", [(0, 0), (64, 1), (64, 2), (32, 1), (32, 2), (32, 3)])
def test_extend_device_aligned_grid_edges(torch_dev, oracle, shape):
    # The chunk grid is anchored at the first 4 KiB boundary at or after the
    # data start (long_plan.h): chunk 0 = the head (0 bytes when the data is
    # 4 KiB-aligned, < 64 bytes on the byte-serial path, up to 4095), the last
    # chunk cut at the end (1 byte up to a whole chunk), the whole buffer in
    # chunk 0 when it ends before the boundary. Every lane/round shape
    # (photon_crc_set_long_shape; (0, 0) = automatic), CRC-32C and CRC-64.
    torch = torch_dev
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    lanes, rounds = shape
    ck.set_long_shape(lanes, rounds)
    ck.set_mid_kernel(False)  # the long kernel's plan for every span over 256 KiB
    try:
        full = 16 * cus * (64 // (lanes or 64)) * (rounds or 1)  # lane-group slots of a full grid
        n_full = 16384 * full  # the 16 KiB chunk floor of a full grid (64 MiB at 64 x 1)
        d = torch.empty(n_full + 4 * 4096, dtype=torch.uint8, device="cuda")
        ck.fill_splitmix(d, d.numel(), d.numel(), 1, 0x5EED0900 + lanes + rounds)
        host = d.cpu().numpy()
        al = (-d.data_ptr()) % 4096  # offset of the first 4 KiB boundary
        cases = [(al, n_full), (al + 1, n_full), (al + 4095, n_full + 1),
                 (al + 4096 - 10, 300 << 10), (al + 4096 - 100, (300 << 10) + 1),
                 (al + 4096 - 5, 4), (al + 4096 - 5, 5), (al + 4096 - 5, 6), (al + 7, 4096 - 7),
                 (al + 3, (256 << 10) + 4093), (al + 2, n_full - (16 << 10) + 1), (al + 5, 40 << 20)]
        assert max(off + n for off, n in cases) <= d.numel()
        for k, (off, n) in enumerate(cases):
            seed = (k * 0x9E3779B1 + 1) & 0xFFFFFFFF
            want = oracle.crc32c(host[off:off + n], seed)
            assert _extend(torch, d, off, n, seed) == want, (shape, off - al, n)
            if k == 0 or n < (1 << 20):
                s64 = seed * 0x100000001
                assert _extend(torch, d, off, n, s64, True) == oracle.crc64ecma(host[off:off + n], s64), \
                    (shape, off - al, n)
        del d
    finally:
        ck.set_long_shape(0, 0)
        ck.set_mid_kernel(True)


def test_extend_spans_one_buffer_over_devices(torch_dev, oracle):
    # photon_crc32c_extend_spans / photon_crc64ecma_extend_spans: ONE logical
    # buffer cut into spans, each span on a device (round-robin over the
    # visible devices; all on device 0 on a one-GPU box), the span CRCs folded
    # on the host (crc.cpp:393-405). Spans: empty, 1 byte, unaligned, one over
    # the one-workgroup limit, a full-grid one; seeds 0 and all-ones.
    torch = torch_dev
    ndev = torch.cuda.device_count()
    lens = [0, 1, 4095, 12345, (256 << 10) + 3, 0, 7, 9 << 20, 64]
    host = np.random.default_rng(0x5EED0A00).integers(0, 256, sum(lens) + 64, dtype=np.uint8)
    keep, spans, pos = [], [], 0
    for k, n in enumerate(lens):
        dev = k % ndev
        t = torch.from_numpy(host[pos:pos + n + 16].copy()).to(f"cuda:{dev}")
        keep.append(t)
        spans.append((dev, t.data_ptr() + (k % 3), n))  # unaligned span starts
        host[pos:pos + n] = host[pos + (k % 3):pos + (k % 3) + n].copy()
        pos += n
    data = host[:pos]
    for seed in (0, 0xFFFFFFFF, 0x1234567):
        assert ck.extend_spans(spans, seed) == oracle.crc32c(data, seed), seed
        s64 = seed * 0x100000001
        assert ck.extend64_spans(spans, s64) == oracle.crc64ecma(data, s64), seed
    assert ck.extend_spans([], 5) == 5  # no bytes: the seed
    with pytest.raises(ck.CrcError):
        ck.extend_spans([(0, 0, 16)], 0)  # null span with bytes
