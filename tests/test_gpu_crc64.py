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


@pytest.mark.parametrize("g", [0, 4, 64])
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
