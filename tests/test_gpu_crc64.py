"""CRC-64/ECMA device batches (photon_crc64ecma_batch_*) against the
reference's golden data (checksum.crc64), its own crc64ecma_sw outputs
(ref_vectors.json) and the pinned oracle. Bit-exact."""
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
    assert torch.cuda.is_available()
    return torch


@pytest.fixture(autouse=True)
def _reset():
    yield
    ck.set_lanes_per_buffer(0)


def run_iov64(torch, d, offs, lens, seeds=None):
    n = len(offs)
    iov = np.zeros((n, 2), np.uint64)
    iov[:, 0] = np.uint64(d.data_ptr()) + np.asarray(offs, np.uint64)
    iov[:, 1] = np.asarray(lens, np.uint64)
    d_iov = torch.from_numpy(iov.view(np.int64)).cuda()
    d_seeds = torch.from_numpy(np.asarray(seeds, np.uint64).view(np.int64)).cuda() if seeds is not None else None
    out = torch.zeros(n, dtype=torch.int64, device="cuda")
    ck.batch64_iov(d_iov, n, out, seeds=d_seeds)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint64)


def test_golden_checksum_crc64(torch_dev, golden_in):
    d = torch_dev.from_numpy(ALPHA.copy()).cuda()
    got = run_iov64(torch_dev, d, [0] * 512, list(range(1, 513)))
    assert [int(x) for x in got] == golden_in["crc64ecma"]


@pytest.mark.parametrize("g", [0, 4, 16, 64])
def test_alphabet_and_reference_vectors(torch_dev, ref_vectors, g):
    ck.set_lanes_per_buffer(g)
    rv = ref_vectors
    d = torch_dev.from_numpy(ALPHA.copy()).cuda()
    got = run_iov64(torch_dev, d, [0] * 4097, list(range(4097)))
    assert [int(x) for x in got] == rv["crc64_alphabet"]
    pos, offs = 0, []
    for n in rv["crc64_len"]:
        pos = (pos + 15) // 16 * 16 + 3
        offs.append(pos)
        pos += n
    host = np.zeros(pos + 64, np.uint8)
    for o, n, st in zip(offs, rv["crc64_len"], rv["crc64_stream"]):
        host[o:o + n] = datagen.stream_bytes(st, n)
    d = torch_dev.from_numpy(host).cuda()
    got = run_iov64(torch_dev, d, offs, rv["crc64_len"], seeds=rv["crc64_seed"])
    assert [int(x) for x in got] == rv["crc64_sw"]


def test_every_length_alignment_seed(torch_dev, oracle):
    host = datagen.stream_bytes(0x64, 1 << 16)
    d = torch_dev.from_numpy(host).cuda()
    rnd = random.Random(5)
    offs, lens, seeds = [], [], []
    for n in list(range(0, 200)) + [rnd.randrange(200, 30000) for _ in range(100)]:
        for off in (0, 1, 5, 8, 13, 15):
            offs.append(off + 16 * rnd.randrange(100))
            lens.append(n)
            seeds.append(rnd.getrandbits(64) if n % 2 else 0)
    got = run_iov64(torch_dev, d, offs, lens, seeds=seeds)
    want = [oracle.crc64ecma(host[o:o + n], s) for o, n, s in zip(offs, lens, seeds)]
    assert [int(x) for x in got] == want


@pytest.mark.parametrize("g", [4, 8, 16, 32, 64])
def test_strided(torch_dev, oracle, g):
    ck.set_lanes_per_buffer(g)
    for nbytes, stride, count in ((65536, 65536, 40), (4096, 4096, 300), (5000, 5008, 50)):
        d = torch_dev.empty(stride * count, dtype=torch_dev.uint8, device="cuda")
        ck.fill_splitmix(d, stride, nbytes, count, 0x640 + nbytes)
        out = torch_dev.zeros(count, dtype=torch_dev.int64, device="cuda")
        ck.batch64_strided(d, stride, nbytes, count, out, seed=0x1234)
        torch_dev.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint64)
        for i in range(count):
            assert int(got[i]) == oracle.crc64ecma(datagen.stream_bytes(0x640 + nbytes + i, nbytes), 0x1234), i


@pytest.mark.parametrize("g", [4, 8, 16, 32, 64])
def test_lane_groups_uniform_batches(torch_dev, oracle, g):
    # The batch kernel at every lane-group size on uniform batches (the shapes
    # the retired streaming kernel used to take), with seed0, per-buffer seeds
    # and no seed; counts that do not fill whole wave tuples.
    ck.set_lanes_per_buffer(g)
    try:
        for nbytes, count in ((16 * 64 * 8, 37), (65536, 301), (4096, 1001)):
            d = torch_dev.empty(nbytes * count, dtype=torch_dev.uint8, device="cuda")
            ck.fill_splitmix(d, nbytes, nbytes, count, 0x6400 + nbytes)
            seeds = [(0x9E3779B97F4A7C15 * (i + 1)) & 0xFFFFFFFFFFFFFFFF for i in range(count)]
            d_seeds = torch_dev.from_numpy(np.asarray(seeds, np.uint64).view(np.int64)).cuda()
            for kw, sd in ((dict(), lambda i: 0), (dict(seed=0xFEDCBA9876543210), lambda i: 0xFEDCBA9876543210),
                           (dict(seeds=d_seeds), lambda i: seeds[i])):
                out = torch_dev.zeros(count, dtype=torch_dev.int64, device="cuda")
                ck.batch64_strided(d, nbytes, nbytes, count, out, **kw)
                torch_dev.cuda.synchronize()
                got = out.cpu().numpy().view(np.uint64)
                for i in list(range(0, count, max(1, count // 25))) + [count - 1]:
                    want = oracle.crc64ecma(datagen.stream_bytes(0x6400 + nbytes + i, nbytes), sd(i))
                    assert int(got[i]) == want, (g, nbytes, i)
    finally:
        ck.set_lanes_per_buffer(0)


def test_full_c2_crc64(torch_dev, oracle):
    # C2 shape at full size: two lane-group sizes agree on all 65,536 CRCs; a
    # sample is checked against the oracle.
    n, cnt = 65536, 65536
    d = torch_dev.empty(n * cnt, dtype=torch_dev.uint8, device="cuda")
    ck.fill_splitmix(d, n, n, cnt, 0x5EED0001)
    a = torch_dev.zeros(cnt, dtype=torch_dev.int64, device="cuda")
    b = torch_dev.zeros(cnt, dtype=torch_dev.int64, device="cuda")
    ck.batch64_strided(d, n, n, cnt, a)  # default: 32 lanes per buffer
    ck.set_lanes_per_buffer(64)
    try:
        ck.batch64_strided(d, n, n, cnt, b)
    finally:
        ck.set_lanes_per_buffer(0)
    torch_dev.cuda.synchronize()
    assert torch_dev.equal(a, b)
    got = a.cpu().numpy().view(np.uint64)
    for i in range(0, cnt, 4099):
        assert int(got[i]) == oracle.crc64ecma(d[i * n:(i + 1) * n].cpu().numpy())


def test_combine64_batch_reference_triples(torch_dev, ref_vectors):
    # photon_crc64ecma_combine_batch vs the reference's own crc64ecma_combine_sw
    # outputs (ref_vectors.json c64_*), shortcuts included.
    rv = ref_vectors
    n = len(rv["c64_crc1"])
    t = lambda a, dt: torch_dev.from_numpy(np.asarray(a, dt).view(  # noqa: E731
        np.int64 if dt == np.uint64 else np.int32)).cuda()
    out = torch_dev.zeros(n, dtype=torch_dev.int64, device="cuda")
    ck.combine64_batch(t(rv["c64_crc1"], np.uint64), t(rv["c64_crc2"], np.uint64), t(rv["c64_len2"], np.uint32),
                       n, out)
    torch_dev.cuda.synchronize()
    assert [int(v) for v in out.cpu().numpy().view(np.uint64)] == rv["c64_comb_sw"]


def test_msg64_scatter_gather(torch_dev, oracle):
    # Messages of ragged, misaligned, empty segments (and empty messages):
    # photon_crc64ecma_batch_msg_n == crc64ecma_extend chained over the segments.
    rnd = random.Random(64)
    host = datagen.stream_bytes(0x64, 1 << 20)
    d = torch_dev.from_numpy(host.copy()).cuda()
    iov, start, segs = [], [0], []
    for m in range(300):
        k = rnd.choice([0, 1, 2, 3, 8, 28])
        for _ in range(k):
            n = rnd.choice([0, 1, 7, 63, 64, 100, 4096, 8192, 20000])
            o = rnd.randrange(0, (1 << 20) - n)
            iov.append((d.data_ptr() + o, n))
            segs.append((o, n))
        start.append(len(iov))
    nseg, nmsg = len(iov), len(start) - 1
    seeds = [rnd.getrandbits(64) if m % 3 else 0 for m in range(nmsg)]
    d_iov = torch_dev.from_numpy(np.asarray(iov, np.uint64).view(np.int64)).cuda()
    d_start = torch_dev.from_numpy(np.asarray(start, np.uint64).view(np.int64)).cuda()
    d_seeds = torch_dev.from_numpy(np.asarray(seeds, np.uint64).view(np.int64)).cuda()
    seg_out = torch_dev.zeros(max(nseg, 1), dtype=torch_dev.int64, device="cuda")
    out = torch_dev.zeros(nmsg, dtype=torch_dev.int64, device="cuda")
    ck.batch64_msg_n(d_iov, d_start, nmsg, nseg, seg_out, out, seeds=d_seeds)
    torch_dev.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint64)
    for m in range(nmsg):
        acc = seeds[m]
        for o, n in segs[start[m]:start[m + 1]]:
            acc = oracle.crc64ecma(host[o:o + n], acc)
        assert int(got[m]) == acc, m


@pytest.mark.parametrize("nbytes", [0, 1, 4095, 16384, 16389, 1 << 20, (1 << 20) + 3, (64 << 20) + 7])
def test_extend64_device_single_buffer(torch_dev, oracle, nbytes):
    # photon_crc64ecma_extend_device: one long buffer split into pieces,
    # checksummed in parallel and folded; unaligned start, seeds 0 and not.
    d = torch_dev.empty(nbytes + 32, dtype=torch_dev.uint8, device="cuda")
    ck.fill_splitmix(d, nbytes + 32, nbytes + 32, 1, 0x6465)
    host = d.cpu().numpy()
    out = torch_dev.zeros(1, dtype=torch_dev.int64, device="cuda")
    for seed in (0, 0x0123456789ABCDEF):
        ck.extend64_device(d.data_ptr() + 5, nbytes, out, seed=seed)
        torch_dev.cuda.synchronize()
        assert int(out.cpu().numpy().view(np.uint64)[0]) == oracle.crc64ecma(host[5:5 + nbytes], seed), seed


def test_host_batch64_pipeline(torch_dev, oracle):
    # CRC-64 host-memory pipeline: pinned host batch, odd stride, seeds.
    nbytes, stride, count = 65536 + 8, 65536 + 24, 4500
    host = torch_dev.empty(stride * count, dtype=torch_dev.uint8, pin_memory=True)
    host.numpy()[:] = np.resize(datagen.stream_bytes(0xC64, 1 << 20), stride * count)
    seeds = torch_dev.from_numpy((np.arange(count, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)).view(
        np.int64)).pin_memory()
    out = torch_dev.zeros(count, dtype=torch_dev.int64, pin_memory=True)
    ck.host_batch64_strided(host, stride, nbytes, count, out, seeds=seeds)
    got = out.numpy().view(np.uint64)
    h = host.numpy()
    sd = seeds.numpy().view(np.uint64)
    for i in list(range(0, count, 211)) + [count - 1]:
        assert int(got[i]) == oracle.crc64ecma(h[i * stride:i * stride + nbytes], int(sd[i])), i


def test_trim64_batch_reference_vectors(torch_dev, ref_vectors, oracle):
    # photon_crc64ecma_trim_batch vs the reference's crc64ecma_trim_sw outputs
    # (ref_vectors t64_*; same buffer as tests/test_crc64_dropin.py), plus the
    # error path and the shortcuts.
    rv = ref_vectors
    buf = datagen.stream_bytes(0x5EEDB064, 5100)
    x = rv["t64_all"][0]
    cases = []
    for l1, l3 in zip(rv["t64_l1"], rv["t64_l3"]):
        c1 = oracle.crc64ecma(buf[:l1])
        c3 = oracle.crc64ecma(buf[5100 - l3:]) if l3 else 0
        cases.append(((x, 5100), (c1, l1), (c3, l3)))
    want = list(rv["t64_sw"])
    cases += [((123, 10), (1, 6), (2, 6)),          # EINVAL: 0 and counted
              ((0xDEAD, 100), (0, 0), (0, 0)),       # nothing to trim
              ((0xDEAD, 100), (0, 40), (0x12, 60))]  # prefix.crc == 0 shortcut
    want += [0, ck.crc64ecma_trim((0xDEAD, 100), (0, 0), (0, 0)), ck.crc64ecma_trim((0xDEAD, 100), (0, 40), (0x12, 60))]
    arr = [torch_dev.from_numpy(np.asarray([c[k] for c in cases], np.uint64).view(np.int64)).cuda() for k in range(3)]
    out = torch_dev.zeros(len(cases), dtype=torch_dev.int64, device="cuda")
    nerr = torch_dev.zeros(1, dtype=torch_dev.int32, device="cuda")
    ck.trim64_batch(*arr, len(cases), out, nerr)
    torch_dev.cuda.synchronize()
    assert [int(v) for v in out.cpu().numpy().view(np.uint64)] == want
    assert int(nerr.item()) == 1


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("rows", [2, 4])
@pytest.mark.parametrize("g", [4, 8, 16, 32, 64])
def test_full_row_kernel(torch_dev, oracle, mode, rows, g):
    # crc64_full_kernel (whole-step uniform batches): one and several step
    # pairs per buffer, counts that leave the last wave's groups partly idle
    # (they re-read the last buffer, nothing stored), seed0 entering at the
    # end; every CRC against the oracle. Batches it does not take (seeds per
    # buffer, a ragged length) fall back to the generic kernel.
    ck.set_full_rows64(mode, rows)
    ck.set_lanes_per_buffer(g)
    try:
        for k, count in ((1, 1), (1, 37), (3, 301), (2, 1001)):
            nbytes = 2 * 16 * g * rows * k
            if nbytes * count > (64 << 20):
                count = max(1, (64 << 20) // nbytes)
            d = torch_dev.empty(nbytes * count + 64, dtype=torch_dev.uint8, device="cuda")
            ck.fill_splitmix(d, nbytes, nbytes, count, 0x6500 + nbytes + g)
            host = d.cpu().numpy()
            for seed in (0, 0xFEDCBA9876543210):
                out = torch_dev.full((count + 1,), -1, dtype=torch_dev.int64, device="cuda")
                ck.batch64_strided(d, nbytes, nbytes, count, out, seed=seed)
                torch_dev.cuda.synchronize()
                got = out.cpu().numpy().view(np.uint64)
                want = oracle.crc64ecma_strided(host, nbytes, nbytes, count, seed)
                assert np.array_equal(got[:count], np.asarray(want, np.uint64)), (mode, rows, g, nbytes, count, seed)
                assert int(got[count]) == 0xFFFFFFFFFFFFFFFF  # nothing written past the batch
    finally:
        ck.set_full_rows64(3, 2)
        ck.set_lanes_per_buffer(0)


@pytest.mark.parametrize("nbytes", [4096, 6144, 8192, 12288, 16384, 32768, 8192 + 512])
def test_full_row_auto_shapes(torch_dev, oracle, nbytes):
    # The automatic choice (round 6): uniform 4-8 KiB batches take 8 lanes,
    # the full-row kernel 2 rows per step below 8 KiB and 4 from 8 KiB (a
    # length that is not a multiple of the 4-row step pair -- 8.5 KiB --
    # falls back to the generic kernel); every CRC against the oracle, with
    # and without a seed, nothing written past the batch.
    count = 1537
    d = torch_dev.empty(nbytes * count + 64, dtype=torch_dev.uint8, device="cuda")
    ck.fill_splitmix(d, nbytes, nbytes, count, 0x6A00 + nbytes)
    host = d.cpu().numpy()
    for seed in (0, 0x0123456789ABCDEF):
        out = torch_dev.full((count + 1,), -1, dtype=torch_dev.int64, device="cuda")
        ck.batch64_strided(d, nbytes, nbytes, count, out, seed=seed)
        torch_dev.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint64)
        want = oracle.crc64ecma_strided(host, nbytes, nbytes, count, seed)
        assert np.array_equal(got[:count], np.asarray(want, np.uint64)), (nbytes, seed)
        assert int(got[count]) == 0xFFFFFFFFFFFFFFFF
