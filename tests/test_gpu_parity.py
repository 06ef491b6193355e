"""Parity of the MI355X CRC32C engine (libphoton_checksum.so, HIP/gfx950)
against the reference's own outputs and the pinned oracle. Bit-exact: CRC is
integer GF(2) work, there is no tolerance.

All calls go through the C-ABI (photonlibos_amd.checksum -> ctypes ->
photon_crc32c_*); torch only provides device memory."""
import random

import numpy as np
import pytest

from photonlibos_amd import checksum as ck
from photonlibos_amd import datagen

pytestmark = pytest.mark.gpu

ALPHA = np.frombuffer((b"abcdefghijklmnopqrstuvwxyz" * 400)[:8192], np.uint8)


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    assert ck.device_count() >= 1
    return torch


@pytest.fixture(autouse=True)
def _reset_lanes():
    yield
    ck.set_lanes_per_buffer(0)
    ck.set_generic_rows(-1)
    ck.set_msg_mode(0)


# Message batch forms: 0 automatic, 1 one fused kernel (a lane group per
# message), 2 segment kernel + fold kernel.
MSG_MODES = [0, 1, 2]


# Batch kernel variants: rows per step of the generic kernel (-1 = by
# lane-group size, the product default). The fused and streaming kernels of
# earlier rounds measured slower and were deleted.
VARIANTS = [-1, 2, 4, 8]


def to_dev(torch, arr):
    return torch.from_numpy(np.array(arr, copy=True)).cuda()


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def run_iov(torch, dbuf, offs, lens, seeds=None, seed0=0):
    n = len(offs)
    iov = np.zeros((n, 2), np.uint64)
    iov[:, 0] = np.uint64(dbuf.data_ptr()) + np.asarray(offs, np.uint64)
    iov[:, 1] = np.asarray(lens, np.uint64)
    d_iov = to_dev(torch, iov.view(np.int64))
    d_seeds = to_dev(torch, np.asarray(seeds, np.uint32).view(np.int32)) if seeds is not None else None
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    ck.batch_iov(d_iov, n, out, seed=seed0, seeds=d_seeds)
    torch.cuda.synchronize()
    return u32(out)


def run_strided(torch, dbuf, stride, nbytes, count, seeds=None, seed0=0, base_off=0):
    out = torch.zeros(count, dtype=torch.int32, device="cuda")
    d_seeds = to_dev(torch, np.asarray(seeds, np.uint32).view(np.int32)) if seeds is not None else None
    ck.batch_strided(dbuf.data_ptr() + base_off, stride, nbytes, count, out, seed=seed0, seeds=d_seeds)
    torch.cuda.synchronize()
    return u32(out)


def test_golden_512(torch_dev, golden_in):
    # checksum.in known answers (test_checksum.cpp:50-63), lengths 1..512.
    d = to_dev(torch_dev, ALPHA)
    got = run_iov(torch_dev, d, [0] * 512, list(range(1, 513)))
    assert list(got) == golden_in["crc32c"]


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("g", [0, 4, 64])
def test_alphabet_lengths_0_4096(torch_dev, ref_vectors, g, variant):
    ck.set_generic_rows(variant)
    ck.set_lanes_per_buffer(g)
    d = to_dev(torch_dev, ALPHA)
    got = run_iov(torch_dev, d, [0] * 4097, list(range(4097)))
    assert list(got) == ref_vectors["alphabet_crc32c"]


@pytest.mark.parametrize("variant", VARIANTS)
def test_reference_random_vectors(torch_dev, ref_vectors, variant):
    # Outputs of the reference's own crc.cpp on seeded data, with misaligned
    # starts (1..15) and non-zero seeds, lengths 1 .. 1 MiB.
    rv = ref_vectors
    pos, offs, chunks = 0, [], []
    for n, off in zip(rv["rand_len"], rv["rand_off"]):
        pos = (pos + 15) // 16 * 16 + off
        offs.append(pos)
        pos += n
    host = np.zeros(pos + 64, np.uint8)
    for o, n, st in zip(offs, rv["rand_len"], rv["rand_stream"]):
        host[o:o + n] = datagen.stream_bytes(st, n)
    d = to_dev(torch_dev, host)
    ck.set_generic_rows(variant)
    for g in (0, 4, 8, 16, 32, 64):
        ck.set_lanes_per_buffer(g)
        got = run_iov(torch_dev, d, offs, rv["rand_len"], seeds=rv["rand_seed"])
        assert list(got) == rv["rand_crc32c"], g


@pytest.mark.parametrize("variant", VARIANTS)
def test_every_length_and_alignment(torch_dev, oracle, variant):
    ck.set_generic_rows(variant)
    host = datagen.stream_bytes(0x1234, 1 << 16)
    d = to_dev(torch_dev, host)
    rnd = random.Random(1)
    offs, lens, seeds = [], [], []
    for n in list(range(0, 300)) + [rnd.randrange(300, 20000) for _ in range(300)]:
        for off in range(16):
            offs.append(off + 16 * rnd.randrange(100))
            lens.append(n)
            seeds.append(rnd.getrandbits(32) if n % 3 else 0)
    got = run_iov(torch_dev, d, offs, lens, seeds=seeds)
    want = [oracle.crc32c(host[o:o + n], s) for o, n, s in zip(offs, lens, seeds)]
    assert list(got) == want


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("g", [4, 8, 16, 32, 64])
@pytest.mark.parametrize("nbytes,stride", [(64, 64), (100, 112), (1000, 1000), (4096, 4096), (8192, 8192),
                                           (65536, 65536), (65536 + 7, 65536 + 16), (300000, 300001)])
def test_strided_all_lane_groups(torch_dev, oracle, g, nbytes, stride, variant):
    ck.set_generic_rows(variant)
    ck.set_lanes_per_buffer(g)
    count = max(3, min(97, (8 << 20) // stride))
    host = datagen.stream_bytes(g * 1000 + nbytes, stride * count + 64)
    d = to_dev(torch_dev, host)
    for base_off in (0, 5):
        seeds = [(i * 0x9E3779B1) & 0xFFFFFFFF for i in range(count)]
        got = run_strided(torch_dev, d, stride, nbytes, count, seeds=seeds, base_off=base_off)
        want = [oracle.crc32c(host[base_off + i * stride: base_off + i * stride + nbytes], seeds[i])
                for i in range(count)]
        assert list(got) == want, (g, nbytes, stride, base_off)


def test_device_fill_matches_datagen(torch_dev):
    d = torch_dev.zeros(5 * 1000 + 3, dtype=torch_dev.uint8, device="cuda")
    ck.fill_splitmix(d, 1000, 997, 5, 0xABC)
    torch_dev.cuda.synchronize()
    h = d.cpu().numpy()
    for i in range(5):
        assert np.array_equal(h[i * 1000:i * 1000 + 997], datagen.stream_bytes(0xABC + i, 997))
        assert not h[i * 1000 + 997:(i + 1) * 1000].any()


@pytest.mark.parametrize("nbytes,count", [(65536, 1024), (4096, 8192), (1 << 20, 48), (8192, 2048)])
def test_config_shapes_every_buffer(torch_dev, oracle, nbytes, count):
    # BASELINE configs C2/C3/C4/C5-segment shapes at reduced counts: every CRC checked.
    d = torch_dev.empty(nbytes * count, dtype=torch_dev.uint8, device="cuda")
    ck.fill_splitmix(d, nbytes, nbytes, count, 0x5EED0001)
    got = run_strided(torch_dev, d, nbytes, nbytes, count)
    want = [oracle.crc32c(datagen.stream_bytes(0x5EED0001 + i, nbytes)) for i in range(count)]
    assert list(got) == want


def test_full_c2_4gib(torch_dev, oracle):
    # C2 at full size: 64 Ki x 64 KiB device-resident. Size-independent checks:
    # two engine configurations agree on every buffer, a sample matches the
    # oracle, and the result is deterministic.
    nbytes, count = 65536, 65536
    d = torch_dev.empty(nbytes * count, dtype=torch_dev.uint8, device="cuda")
    ck.fill_splitmix(d, nbytes, nbytes, count, 0x5EED0001)
    a = run_strided(torch_dev, d, nbytes, nbytes, count)
    ck.set_lanes_per_buffer(16)
    b = run_strided(torch_dev, d, nbytes, nbytes, count)
    ck.set_lanes_per_buffer(0)
    ck.set_generic_rows(2)  # another rows-per-step shape
    c = run_strided(torch_dev, d, nbytes, nbytes, count)
    ck.set_generic_rows(8)
    e = run_strided(torch_dev, d, nbytes, nbytes, count)
    ck.set_generic_rows(-1)
    assert np.array_equal(a, b) and np.array_equal(a, c) and np.array_equal(a, e)
    rnd = random.Random(2)
    for i in [0, 1, count - 1] + [rnd.randrange(count) for _ in range(61)]:
        assert a[i] == oracle.crc32c(datagen.stream_bytes(0x5EED0001 + i, nbytes)), i
    del d
    torch_dev.cuda.empty_cache()


def _pool_messages(nmsg, nseg, seglen, seed):
    # C5 layout: message m's segment j lives at pool slot perm[m*nseg + j].
    perm = list(range(nmsg * nseg))
    random.Random(seed).shuffle(perm)
    return perm


@pytest.mark.parametrize("mode", MSG_MODES)
@pytest.mark.parametrize("nmsg,nseg,seglen", [(512, 8, 8192), (64, 28, 4096)])
def test_msg_scatter_gather(torch_dev, oracle, nmsg, nseg, seglen, mode):
    ck.set_msg_mode(mode)
    slots = nmsg * nseg
    d = torch_dev.empty(slots * seglen, dtype=torch_dev.uint8, device="cuda")
    ck.fill_splitmix(d, seglen, seglen, slots, 0x5EED0005)
    perm = _pool_messages(nmsg, nseg, seglen, 0x5EED0005)
    base = d.data_ptr()
    iov = np.array([[base + perm[k] * seglen, seglen] for k in range(slots)], np.uint64)
    start = np.arange(0, slots + 1, nseg, dtype=np.uint64)
    seeds = np.array([(m * 2654435761) & 0xFFFFFFFF for m in range(nmsg)], np.uint32)
    d_iov = to_dev(torch_dev, iov.view(np.int64))
    d_start = to_dev(torch_dev, start.view(np.int64))
    d_seeds = to_dev(torch_dev, seeds.view(np.int32))
    seg_out = torch_dev.zeros(slots, dtype=torch_dev.int32, device="cuda")
    out = torch_dev.zeros(nmsg, dtype=torch_dev.int32, device="cuda")
    ck.batch_msg(d_iov, d_start, nmsg, seg_out, out, seeds=d_seeds)
    torch_dev.cuda.synchronize()
    got, segs = u32(out), u32(seg_out)
    slot_data = [datagen.stream_bytes(0x5EED0005 + s, seglen) for s in range(slots)]
    for k in range(slots):
        assert segs[k] == oracle.crc32c(slot_data[perm[k]])
    for m in range(nmsg):
        parts = [slot_data[perm[m * nseg + j]] for j in range(nseg)]
        assert got[m] == oracle.extend_chain(parts, int(seeds[m])), m
    # the fully asynchronous form (host supplies the segment count) agrees
    out2 = torch_dev.zeros(nmsg, dtype=torch_dev.int32, device="cuda")
    ck.batch_msg_n(d_iov, d_start, nmsg, slots, seg_out, out2, seeds=d_seeds)
    torch_dev.cuda.synchronize()
    assert np.array_equal(u32(out2), got)


@pytest.mark.parametrize("mode", MSG_MODES)
@pytest.mark.parametrize("g", [0, 4, 64])
def test_msg_ragged_segments(torch_dev, oracle, mode, g):
    # Generic iovectors: odd lengths, odd addresses, empty segments, empty messages.
    ck.set_msg_mode(mode)
    ck.set_lanes_per_buffer(g)
    rnd = random.Random(3)
    host = datagen.stream_bytes(77, 1 << 20)
    d = to_dev(torch_dev, host)
    iov, start, want_segs = [], [0], []
    msgs = []
    for m in range(300):
        k = rnd.choice([0, 1, 2, 5, 28])
        parts = []
        for _ in range(k):
            n = rnd.choice([0, 1, 3, 17, 64, 100, 4095, 8192, 10000])
            o = rnd.randrange(len(host) - n)
            iov.append([d.data_ptr() + o, n])
            parts.append(host[o:o + n])
        start.append(len(iov))
        msgs.append(parts)
    seeds = np.array([rnd.getrandbits(32) for _ in msgs], np.uint32)
    d_iov = to_dev(torch_dev, np.array(iov, np.uint64).view(np.int64))
    d_start = to_dev(torch_dev, np.array(start, np.uint64).view(np.int64))
    seg_out = torch_dev.zeros(max(len(iov), 1), dtype=torch_dev.int32, device="cuda")
    out = torch_dev.zeros(len(msgs), dtype=torch_dev.int32, device="cuda")
    ck.batch_msg(d_iov, d_start, len(msgs), seg_out, out, seeds=to_dev(torch_dev, seeds.view(np.int32)))
    out_ns = torch_dev.zeros(len(msgs), dtype=torch_dev.int32, device="cuda")
    ck.batch_msg(d_iov, d_start, len(msgs), None, out_ns, seeds=to_dev(torch_dev, seeds.view(np.int32)))
    torch_dev.cuda.synchronize()
    got = u32(out)
    assert np.array_equal(u32(out_ns), got)
    for m, parts in enumerate(msgs):
        assert got[m] == oracle.extend_chain(parts, int(seeds[m])), m


def test_combine_batch(torch_dev, ref_vectors):
    rv = ref_vectors
    c1 = to_dev(torch_dev, np.array(rv["comb_crc1"], np.uint32).view(np.int32))
    c2 = to_dev(torch_dev, np.array(rv["comb_crc2"], np.uint32).view(np.int32))
    l2 = to_dev(torch_dev, np.array(rv["comb_len2"], np.uint32).view(np.int32))
    out = torch_dev.zeros(len(rv["comb_sw"]), dtype=torch_dev.int32, device="cuda")
    ck.combine_batch(c1, c2, l2, len(rv["comb_sw"]), out)
    torch_dev.cuda.synchronize()
    assert list(u32(out)) == rv["comb_sw"]


def test_series_shape(torch_dev, ref_vectors):
    # crc32c_series over a device buffer == strided batch with stride == part_size.
    rv = ref_vectors
    host = datagen.stream_bytes(0x5EEDA000, 1 << 20)
    d = to_dev(torch_dev, host)
    pos = 0
    for ps, npart in zip(rv["series_part"], rv["series_n"]):
        want = rv["series_sw"][pos:pos + npart]
        pos += npart
        assert list(run_strided(torch_dev, d, ps, ps, npart)) == want, ps


def test_single_bit_flips_detected(torch_dev, oracle):
    # Failure detection: any single-bit corruption changes the CRC, and the change
    # equals crc(error pattern) (linearity) -- exercised on device.
    n = 65536
    host = datagen.stream_bytes(99, n)
    rnd = random.Random(4)
    bufs = [host.copy()]
    flips = []
    for _ in range(63):
        b = host.copy()
        bit = rnd.randrange(n * 8)
        b[bit // 8] ^= 1 << (bit % 8)
        bufs.append(b)
        flips.append(bit)
    d = to_dev(torch_dev, np.concatenate(bufs))
    got = run_strided(torch_dev, d, n, n, len(bufs))
    assert got[0] == oracle.crc32c(host)
    for k, bit in enumerate(flips, 1):
        e = np.zeros(n, np.uint8)
        e[bit // 8] = 1 << (bit % 8)
        assert got[k] != got[0]
        assert got[k] ^ got[0] == oracle.crc32c(e)


def test_host_batch_pipeline(torch_dev, oracle):
    # Host-resident (pinned) batch through the chunked H2D + kernel + D2H pipeline,
    # more buffers than one staging chunk holds, odd stride, per-buffer seeds.
    nbytes, stride, count = 65536 + 8, 65536 + 24, 5000
    host = torch_dev.empty(stride * count, dtype=torch_dev.uint8, pin_memory=True)
    host.numpy()[:] = np.resize(datagen.stream_bytes(0xB0B, 1 << 20), stride * count)
    seeds = torch_dev.from_numpy(np.arange(count, dtype=np.uint32).view(np.int32)).pin_memory()
    out = torch_dev.zeros(count, dtype=torch_dev.int32, pin_memory=True)
    ck.host_batch_strided(host, stride, nbytes, count, out, seeds=seeds)
    got = out.numpy().view(np.uint32)
    h = host.numpy()
    for i in list(range(0, count, 97)) + [count - 1]:
        assert got[i] == oracle.crc32c(h[i * stride:i * stride + nbytes], i), i
    # The same batch sharded over this process's devices (all; then one)
    # gives the same CRCs (every device visible here takes a slice).
    for ndev in (0, 1):
        out2 = torch_dev.zeros(count, dtype=torch_dev.int32, pin_memory=True)
        ck.host_batch_strided_multi(host, stride, nbytes, count, out2, seeds=seeds, ndev=ndev)
        assert np.array_equal(out2.numpy(), out.numpy()), ndev


def test_host_batches_zero_length(torch_dev):
    # nbytes == 0 with count > 0 is legal (crc32c_extend over
    # 0 bytes returns the seed, crc.cpp:114-117) and once divided by zero in the
    # host pipeline. Every host batch returns the seeds (or seed0).
    count = 37
    host = torch_dev.zeros(64, dtype=torch_dev.uint8, pin_memory=True)
    seeds = np.arange(1, count + 1, dtype=np.uint32) * np.uint32(0x9E3779B1)
    d_seeds = torch_dev.from_numpy(seeds.view(np.int32).copy()).pin_memory()
    for fn in (lambda o, **kw: ck.host_batch_strided(host, 0, 0, count, o, **kw),
               lambda o, **kw: ck.host_batch_strided_multi(host, 0, 0, count, o, **kw)):
        out = torch_dev.zeros(count, dtype=torch_dev.int32, pin_memory=True)
        fn(out, seeds=d_seeds)
        assert np.array_equal(out.numpy().view(np.uint32), seeds)
        out = torch_dev.zeros(count, dtype=torch_dev.int32, pin_memory=True)
        fn(out, seed=0xCAFEF00D)
        assert set(out.numpy().view(np.uint32).tolist()) == {0xCAFEF00D}
    seeds64 = np.arange(1, count + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    d_seeds64 = torch_dev.from_numpy(seeds64.view(np.int64).copy()).pin_memory()
    out64 = torch_dev.zeros(count, dtype=torch_dev.int64, pin_memory=True)
    ck.host_batch64_strided(host, 0, 0, count, out64, seeds=d_seeds64)
    assert np.array_equal(out64.numpy().view(np.uint64), seeds64)


def test_device_shards(torch_dev, oracle):
    # photon_crc32c_batch_strided_shards: two shards (halves, different seeds)
    # enqueued on the device(s); equal to one batch per half.
    nbytes, count = 4096, 1000
    d = torch_dev.empty(nbytes * count, dtype=torch_dev.uint8, device="cuda")
    ck.fill_splitmix(d, nbytes, nbytes, count, 0x5EED0001)
    out = torch_dev.zeros(count, dtype=torch_dev.int32, device="cuda")
    half = count // 2
    ck.batch_strided_shards([
        dict(device=0, d_base=d.data_ptr(), stride=nbytes, nbytes=nbytes, count=half, seed0=0,
             d_out=out.data_ptr()),
        dict(device=0, d_base=d.data_ptr() + half * nbytes, stride=nbytes, nbytes=nbytes, count=count - half,
             seed0=0xABCDEF01, d_out=out.data_ptr() + 4 * half),
    ])
    torch_dev.cuda.synchronize()
    got = u32(out)
    for i in (0, 1, half - 1, half, count - 1):
        want = oracle.crc32c(datagen.stream_bytes(0x5EED0001 + i, nbytes), 0 if i < half else 0xABCDEF01)
        assert got[i] == want, i


def test_msg_many_messages_fused_vs_two_kernels(torch_dev, oracle):
    # Enough messages for the automatic one-kernel form (>= 4096 waves of
    # groups): ragged messages of 0..6 segments at random offsets; the fused
    # and two-kernel forms agree on every message and segment, a sample
    # matches the oracle.
    rnd = random.Random(11)
    host = datagen.stream_bytes(0x11, 1 << 20)
    d = to_dev(torch_dev, host)
    nmsg = 40000
    iov, start, msgs = [], [0], []
    for m in range(nmsg):
        parts = []
        for _ in range(rnd.choice([0, 1, 3, 6])):
            n = rnd.choice([0, 5, 64, 200, 1500, 3000])
            o = rnd.randrange(len(host) - n)
            iov.append([d.data_ptr() + o, n])
            parts.append((o, n))
        start.append(len(iov))
        msgs.append(parts)
    seeds = np.array([rnd.getrandbits(32) for _ in range(nmsg)], np.uint32)
    d_iov = to_dev(torch_dev, np.array(iov, np.uint64).view(np.int64))
    d_start = to_dev(torch_dev, np.array(start, np.uint64).view(np.int64))
    d_seeds = to_dev(torch_dev, seeds.view(np.int32))
    res = {}
    for mode in (1, 2, 0):
        ck.set_msg_mode(mode)
        seg_out = torch_dev.zeros(len(iov), dtype=torch_dev.int32, device="cuda")
        out = torch_dev.zeros(nmsg, dtype=torch_dev.int32, device="cuda")
        ck.batch_msg_n(d_iov, d_start, nmsg, len(iov), seg_out, out, seeds=d_seeds)
        # without per-segment CRCs (the seed-chained form when fused)
        out_ns = torch_dev.zeros(nmsg, dtype=torch_dev.int32, device="cuda")
        ck.batch_msg_n(d_iov, d_start, nmsg, len(iov), None, out_ns, seeds=d_seeds)
        torch_dev.cuda.synchronize()
        res[mode] = (u32(out).copy(), u32(seg_out).copy())
        assert np.array_equal(u32(out_ns), res[mode][0]), mode
    assert np.array_equal(res[1][0], res[2][0]) and np.array_equal(res[1][1], res[2][1])
    assert np.array_equal(res[0][0], res[1][0])
    for m in list(range(0, nmsg, 97)) + [nmsg - 1]:
        parts = [host[o:o + n] for o, n in msgs[m]]
        assert res[1][0][m] == oracle.extend_chain(parts, int(seeds[m])), m
