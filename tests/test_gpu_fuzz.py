"""Randomised parity: many random shapes through every CRC32C / CRC-64 device
entry point and engine variant, checked bit-exactly against the pinned
oracle (tests/_oracle.py). Seeds are fixed, so a failure reproduces."""
import os
import random

import numpy as np
import pytest

from photonlibos_amd import checksum as ck
from photonlibos_amd import datagen

pytestmark = pytest.mark.gpu

POOL = 4 << 20
# PHOTON_FUZZ_ROUNDS=k multiplies the rounds (longer soak runs, new seeds).
SOAK = max(1, int(os.environ.get("PHOTON_FUZZ_ROUNDS", "1")))


@pytest.fixture(scope="module")
def dev_pool():
    import torch
    assert torch.cuda.is_available()
    host = datagen.stream_bytes(0xF022, POOL)
    return torch, host, torch.from_numpy(host.copy()).cuda()


@pytest.fixture(autouse=True)
def _reset():
    yield
    ck.set_lanes_per_buffer(0)
    ck.set_generic_rows(-1)
    ck.set_msg_mode(0)
    ck.set_msg_rows(2)


ENGINES = [  # (lanes, generic rows): every lane-group size, every rows-per-step shape
    (0, -1), (0, 4), (4, 4), (8, 2), (16, 8), (16, 2), (32, 4), (64, 4), (64, 8),
]


def _lengths(rnd, k):
    out = []
    for _ in range(k):
        r = rnd.random()
        out.append(rnd.randrange(0, 80) if r < 0.3 else rnd.randrange(80, 5000) if r < 0.8
                   else rnd.randrange(5000, 300000))
    return out


@pytest.mark.parametrize("round_", range(4 * SOAK))
def test_fuzz_iov_batches(dev_pool, oracle, round_):
    torch, host, d = dev_pool
    rnd = random.Random(1000 + round_)
    for lanes, rows in ENGINES:
        ck.set_lanes_per_buffer(lanes)
        ck.set_generic_rows(rows)
        lens = _lengths(rnd, 120)
        offs = [rnd.randrange(0, POOL - n) for n in lens]
        seeds = [rnd.getrandbits(32) if rnd.random() < 0.7 else 0 for _ in lens]
        iov = np.zeros((len(lens), 2), np.uint64)
        iov[:, 0] = np.uint64(d.data_ptr()) + np.asarray(offs, np.uint64)
        iov[:, 1] = np.asarray(lens, np.uint64)
        d_iov = torch.from_numpy(iov.view(np.int64)).cuda()
        d_seeds = torch.from_numpy(np.asarray(seeds, np.uint32).view(np.int32)).cuda()
        out = torch.zeros(len(lens), dtype=torch.int32, device="cuda")
        ck.batch_iov(d_iov, len(lens), out, seeds=d_seeds)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        for k, (o, n, s) in enumerate(zip(offs, lens, seeds)):
            assert got[k] == oracle.crc32c(host[o:o + n], s), (lanes, rows, o, n, s)


@pytest.mark.parametrize("round_", range(3 * SOAK))
def test_fuzz_strided_batches(dev_pool, oracle, round_):
    torch, host, d = dev_pool
    rnd = random.Random(2000 + round_)
    for lanes, rows in ENGINES:
        ck.set_lanes_per_buffer(lanes)
        ck.set_generic_rows(rows)
        aligned = rnd.random() < 0.5
        nbytes = rnd.choice([4096, 8192, 65536, 16 * 64 * 4]) if aligned else rnd.randrange(1, 70000)
        stride = nbytes if aligned else nbytes + rnd.randrange(0, 64)
        count = max(1, min(rnd.randrange(1, 300), (POOL - 64) // stride))
        base = 0 if aligned else rnd.randrange(0, 16)
        seed0 = rnd.getrandbits(32)
        out = torch.zeros(count, dtype=torch.int32, device="cuda")
        ck.batch_strided(d.data_ptr() + base, stride, nbytes, count, out, seed=seed0)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        for i in range(count):
            o = base + i * stride
            assert got[i] == oracle.crc32c(host[o:o + nbytes], seed0), (lanes, rows, nbytes, stride, i)


@pytest.mark.parametrize("round_", range(3 * SOAK))
def test_fuzz_messages(dev_pool, oracle, round_):
    torch, host, d = dev_pool
    rnd = random.Random(3000 + round_)
    for mode, mrows in ((0, 2), (1, 2), (1, 4), (2, 2)):
        for lanes in (0, 8, 64):
            ck.set_msg_mode(mode)
            ck.set_msg_rows(mrows)
            ck.set_lanes_per_buffer(lanes)
            nmsg = rnd.randrange(1, 400)
            iov, start, msgs = [], [0], []
            for _ in range(nmsg):
                parts = []
                for n in _lengths(rnd, rnd.choice([0, 1, 2, 5, 12])):
                    n = min(n, 40000)
                    o = rnd.randrange(0, POOL - n)
                    iov.append((d.data_ptr() + o, n))
                    parts.append(host[o:o + n])
                start.append(len(iov))
                msgs.append(parts)
            seeds = [rnd.getrandbits(32) for _ in range(nmsg)]
            d_iov = torch.from_numpy(np.asarray(iov or [(0, 0)], np.uint64).view(np.int64)).cuda()
            d_start = torch.from_numpy(np.asarray(start, np.uint64).view(np.int64)).cuda()
            d_seeds = torch.from_numpy(np.asarray(seeds, np.uint32).view(np.int32)).cuda()
            out = torch.zeros(nmsg, dtype=torch.int32, device="cuda")
            seg = torch.zeros(max(len(iov), 1), dtype=torch.int32, device="cuda") if rnd.random() < 0.5 else None
            ck.batch_msg_n(d_iov, d_start, nmsg, len(iov), seg, out, seeds=d_seeds)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            for m, parts in enumerate(msgs):
                assert got[m] == oracle.extend_chain(parts, seeds[m]), (mode, lanes, m)
            if seg is not None and iov:
                segs = seg.cpu().numpy().view(np.uint32)
                flat = [p for parts in msgs for p in parts]
                for k, part in enumerate(flat):
                    assert segs[k] == oracle.crc32c(part, 0), (mode, lanes, k)


@pytest.mark.parametrize("lanes", [0, 4, 8, 16, 64])
def test_message_segment_crcs_many_rounds(dev_pool, oracle, lanes):
    # Segment CRCs of the one-kernel message form, which holds a lane's
    # segment-CRC stores back (two per lane) until a third arrives or the wave
    # ends: messages of up to 40 segments (several store events per lane and
    # message) and enough messages that every wave runs several rounds.
    torch, host, d = dev_pool
    rnd = random.Random(7000 + lanes)
    ck.set_msg_mode(1)
    ck.set_lanes_per_buffer(lanes)
    iov, start, msgs = [], [0], []
    nmsg = 120000 if lanes in (0, 4, 8) else 3000
    for m in range(nmsg):
        k = rnd.choice([1, 2, 3]) if m % 50 else rnd.randrange(17, 41)
        parts = []
        for _ in range(k):
            n = rnd.randrange(0, 600) if lanes in (0, 4, 8) else rnd.randrange(0, 20000)
            o = rnd.randrange(0, POOL - n)
            iov.append((d.data_ptr() + o, n))
            parts.append((o, n))
        start.append(len(iov))
        msgs.append(parts)
    d_iov = torch.from_numpy(np.asarray(iov, np.uint64).view(np.int64)).cuda()
    d_start = torch.from_numpy(np.asarray(start, np.uint64).view(np.int64)).cuda()
    out = torch.zeros(nmsg, dtype=torch.int32, device="cuda")
    seg = torch.full((len(iov),), -1, dtype=torch.int32, device="cuda")
    ck.batch_msg_n(d_iov, d_start, nmsg, len(iov), seg, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    segs = seg.cpu().numpy().view(np.uint32)
    k = 0
    for m, parts in enumerate(msgs):
        views = [host[o:o + n] for o, n in parts]
        for v in views:
            assert segs[k] == oracle.crc32c(v, 0), (lanes, m, k)
            k += 1
        assert got[m] == oracle.extend_chain(views, 0), (lanes, m)


@pytest.mark.parametrize("round_", range(2 * SOAK))
def test_fuzz_crc64(dev_pool, oracle, round_):
    torch, host, d = dev_pool
    rnd = random.Random(4000 + round_)
    for lanes in (0, 4, 8, 16, 32, 64):
        ck.set_lanes_per_buffer(lanes)
        lens = _lengths(rnd, 80)
        offs = [rnd.randrange(0, POOL - n) for n in lens]
        seeds = [rnd.getrandbits(64) for _ in lens]
        iov = np.zeros((len(lens), 2), np.uint64)
        iov[:, 0] = np.uint64(d.data_ptr()) + np.asarray(offs, np.uint64)
        iov[:, 1] = np.asarray(lens, np.uint64)
        d_iov = torch.from_numpy(iov.view(np.int64)).cuda()
        d_seeds = torch.from_numpy(np.asarray(seeds, np.uint64).view(np.int64)).cuda()
        out = torch.zeros(len(lens), dtype=torch.int64, device="cuda")
        ck.batch64_iov(d_iov, len(lens), out, seeds=d_seeds)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint64)
        for k, (o, n, s) in enumerate(zip(offs, lens, seeds)):
            assert int(got[k]) == oracle.crc64ecma(host[o:o + n], s), (lanes, o, n)


LANES64 = [0, 4, 8, 16, 32, 64]  # lanes per buffer of the CRC-64 batch kernel (0 = automatic)


@pytest.mark.parametrize("round_", range(3 * SOAK))
def test_fuzz_crc64_strided(dev_pool, oracle, round_):
    torch, host, d = dev_pool
    rnd = random.Random(5000 + round_)
    for lanes in LANES64:
        ck.set_lanes_per_buffer(lanes)
        aligned = rnd.random() < 0.6
        nbytes = rnd.choice([4096, 8192, 65536, 16 * 64 * 8]) if aligned else rnd.randrange(1, 70000)
        stride = nbytes if aligned else nbytes + rnd.randrange(0, 64)
        count = max(1, min(rnd.randrange(1, 300), (POOL - 64) // stride))
        base = 0 if aligned else rnd.randrange(0, 16)
        seed0 = rnd.getrandbits(64)
        seeds = [rnd.getrandbits(64) for _ in range(count)] if rnd.random() < 0.4 else None
        d_seeds = torch.from_numpy(np.asarray(seeds, np.uint64).view(np.int64)).cuda() if seeds else None
        out = torch.zeros(count, dtype=torch.int64, device="cuda")
        ck.batch64_strided(d.data_ptr() + base, stride, nbytes, count, out, seed=seed0, seeds=d_seeds)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint64)
        for i in range(count):
            o = base + i * stride
            want = oracle.crc64ecma(host[o:o + nbytes], seeds[i] if seeds else seed0)
            assert int(got[i]) == want, (lanes, nbytes, stride, i)


def _chain64(oracle, parts, seed):
    c = seed
    for p in parts:
        c = oracle.crc64ecma(p, c)
    return c


@pytest.mark.parametrize("round_", range(3 * SOAK))
def test_fuzz_crc64_messages(dev_pool, oracle, round_):
    torch, host, d = dev_pool
    rnd = random.Random(6000 + round_)
    for lanes in (0, 8, 64):
        ck.set_lanes_per_buffer(lanes)
        nmsg = rnd.randrange(1, 300)
        iov, start, msgs = [], [0], []
        for _ in range(nmsg):
            parts = []
            for n in _lengths(rnd, rnd.choice([0, 1, 3, 8])):
                n = min(n, 40000)
                o = rnd.randrange(0, POOL - n)
                iov.append((d.data_ptr() + o, n))
                parts.append(host[o:o + n])
            start.append(len(iov))
            msgs.append(parts)
        seeds = [rnd.getrandbits(64) for _ in range(nmsg)]
        d_iov = torch.from_numpy(np.asarray(iov or [(0, 0)], np.uint64).view(np.int64)).cuda()
        d_start = torch.from_numpy(np.asarray(start, np.uint64).view(np.int64)).cuda()
        d_seeds = torch.from_numpy(np.asarray(seeds, np.uint64).view(np.int64)).cuda()
        out = torch.zeros(nmsg, dtype=torch.int64, device="cuda")
        seg = torch.zeros(max(len(iov), 1), dtype=torch.int64, device="cuda") if rnd.random() < 0.5 else None
        ck.batch64_msg_n(d_iov, d_start, nmsg, len(iov), seg, out, seeds=d_seeds)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint64)
        for m, parts in enumerate(msgs):
            assert int(got[m]) == _chain64(oracle, parts, seeds[m]), (lanes, m)


@pytest.mark.parametrize("round_", range(2 * SOAK))
def test_fuzz_extend_device(dev_pool, oracle, round_):
    # One long buffer (the one-buffer fold path) at random offsets / lengths.
    torch, host, d = dev_pool
    rnd = random.Random(7000 + round_)
    out32 = torch.zeros(1, dtype=torch.int32, device="cuda")
    out64 = torch.zeros(1, dtype=torch.int64, device="cuda")
    for _ in range(6):
        n = rnd.choice([rnd.randrange(0, 5000), rnd.randrange(5000, 1 << 20), rnd.randrange(1 << 20, POOL - 64)])
        o = rnd.randrange(0, POOL - n)
        s32, s64 = rnd.getrandbits(32), rnd.getrandbits(64)
        ck.extend_device(d.data_ptr() + o, n, s32, out32)
        ck.extend64_device(d.data_ptr() + o, n, out64, seed=s64)
        torch.cuda.synchronize()
        assert int(out32.cpu().numpy().view(np.uint32)[0]) == oracle.crc32c(host[o:o + n], s32), (o, n)
        assert int(out64.cpu().numpy().view(np.uint64)[0]) == oracle.crc64ecma(host[o:o + n], s64), (o, n)


@pytest.mark.parametrize("mid", [True, False])
def test_fuzz_extend_device_mixed_spans_one_stream(oracle, mid):
    """Small (33 workgroups), mid (up to 512) and long (up to 256) launches of
    both CRCs queued back to back on ONE stream, so they share its reduce
    state: the two-level tree's group and top counts (closed forms in the
    state's running workgroup count) must stay exact across launches of
    every grid size (crc32c_kernels.h long_reduce_tree). 48 random spans of
    0 B-20 MiB at random offsets and seeds, checked after one sync."""
    import torch
    pool = 24 << 20
    host = datagen.stream_bytes(0xF0E1 + mid, pool)
    d = torch.from_numpy(host.copy()).cuda()
    rnd = random.Random(9100 + mid)
    st = torch.cuda.Stream()
    out32 = torch.zeros(48, dtype=torch.int32, device="cuda")
    out64 = torch.zeros(48, dtype=torch.int64, device="cuda")
    cases = []
    ck.set_mid_kernel(mid)
    try:
        torch.cuda.synchronize()
        for k in range(48):
            n = rnd.choice([rnd.randrange(0, 300000), rnd.randrange(300000, 16 << 20), rnd.randrange(16 << 20, 20 << 20)])
            o = rnd.randrange(0, pool - n)
            s32, s64 = rnd.getrandbits(32), rnd.getrandbits(64)
            ck.extend_device(d.data_ptr() + o, n, s32, out32[k:k + 1], stream=st)
            ck.extend64_device(d.data_ptr() + o, n, out64[k:k + 1], seed=s64, stream=st)
            cases.append((o, n, s32, s64))
        st.synchronize()
    finally:
        ck.set_mid_kernel(True)
    g32 = out32.cpu().numpy().view(np.uint32)
    g64 = out64.cpu().numpy().view(np.uint64)
    for k, (o, n, s32, s64) in enumerate(cases):
        assert int(g32[k]) == oracle.crc32c(host[o:o + n], s32), (k, o, n)
        assert int(g64[k]) == oracle.crc64ecma(host[o:o + n], s64), (k, o, n)
