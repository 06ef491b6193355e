"""CRC-64/ECMA host drop-in (include/photon/common/checksum/crc64ecma.h)
against the reference's golden data (checksum.crc64) and the reference's own
outputs (ref_vectors.json: crc64ecma_sw, combine_sw/hw, trim_sw/hw). CPU only."""
import ctypes
import os

import pytest

from photonlibos_amd import checksum as ck
from photonlibos_amd import datagen

ALPHA = (b"abcdefghijklmnopqrstuvwxyz" * 200)


@pytest.mark.parametrize("f", [ck.crc64ecma_sw, ck.crc64ecma_hw, ck.crc64ecma])
def test_golden_checksum_crc64(f, golden_in):
    for k, want in enumerate(golden_in["crc64ecma"]):
        assert f(ALPHA[: k + 1]) == want, k


@pytest.mark.parametrize("f", [ck.crc64ecma_sw, ck.crc64ecma_hw, ck.crc64ecma])
def test_reference_vectors(f, ref_vectors):
    rv = ref_vectors
    for n, sd, st, want in zip(rv["crc64_len"], rv["crc64_seed"], rv["crc64_stream"], rv["crc64_sw"]):
        assert f(datagen.stream_bytes(st, n).tobytes(), sd) == want, (n, sd)
    for n, want in enumerate(rv["crc64_alphabet"]):
        assert f(ALPHA[:n]) == want


def test_combine(ref_vectors):
    rv = ref_vectors
    for c1, c2, l2, want in zip(rv["c64_crc1"], rv["c64_crc2"], rv["c64_len2"], rv["c64_comb_sw"]):
        assert ck.crc64ecma_combine(c1, c2, l2) == want


def test_combine_identity_and_series():
    buf = datagen.stream_bytes(64, 5100).tobytes()
    x = ck.crc64ecma(buf)
    for l1 in (0, 1, 7, 100, 2550, 5099):
        assert ck.crc64ecma_combine(ck.crc64ecma(buf[:l1]), ck.crc64ecma(buf[l1:]), len(buf) - l1) == x
        assert ck.crc64ecma(buf[l1:], ck.crc64ecma(buf[:l1])) == x  # extend
    parts = ck.crc64ecma_series(buf, 510, 10)
    assert ck.crc64ecma_combine_series(parts, 510) == x


def test_trim(ref_vectors):
    rv = ref_vectors
    buf = datagen.stream_bytes(0x5EEDB064, 5100).tobytes()
    x = rv["t64_all"][0]
    assert ck.crc64ecma(buf) == x
    for l1, l3, want in zip(rv["t64_l1"], rv["t64_l3"], rv["t64_sw"]):
        c1 = ck.crc64ecma(buf[:l1])
        c3 = ck.crc64ecma(buf[5100 - l3:]) if l3 else 0
        assert ck.crc64ecma_trim((x, 5100), (c1, l1), (c3, l3)) == want


def test_trim_error_path():
    fn = ctypes.CDLL(ck.lib()._name, use_errno=True)["_Z17crc64ecma_trim_hw19CRC64ECMA_ComponentS_S_"]
    fn.restype = ctypes.c_uint64
    fn.argtypes = [ctypes.c_uint64] * 6
    ctypes.set_errno(0)
    assert fn(1, 10, 2, 6, 3, 6) == 0 and ctypes.get_errno() == 22


def test_hw_folding_matches_sw():
    # crc64ecma_hw (AVX-512 VPCLMULQDQ folding, 16 states in 4 zmm, on CPUs
    # that have it; PCLMUL folding, 4 interleaved 16-byte states, below 256 B
    # and elsewhere) against the table engine: every length through the fold
    # thresholds of both (64/256-B steps, 64- and 16-B tails), odd offsets, seeds.
    import random
    from photonlibos_amd import datagen
    rnd = random.Random(0xF0D)
    data = datagen.stream_bytes(0xF0D, (1 << 20) + 64).tobytes()
    lengths = list(range(0, 1100)) + [1023, 1024, 4096, 65535, 65536, 65537, 1 << 20]
    for n in lengths:
        for off in (0, 3, 8, 13):
            seed = rnd.getrandbits(64) if n % 2 else 0
            b = data[off:off + n]
            assert ck.crc64ecma_hw(b, seed) == ck.crc64ecma_sw(b, seed), (n, off)


def test_hw_engines_without_avx512():
    # PHOTON_CRC_NO_AVX512 (read once at load) pins the 128-bit PCLMUL engines
    # on any CPU: the same parity for them, in a fresh interpreter.
    import subprocess
    import sys
    code = ("import random\n"
            "from photonlibos_amd import checksum as ck, datagen\n"
            "from tests import _oracle as o\n"
            "d = datagen.stream_bytes(0xA5, 70000).tobytes()\n"
            "r = random.Random(4)\n"
            "for n in list(range(0, 1100)) + [r.randrange(1100, 69000) for _ in range(60)]:\n"
            "    for off in (0, 5):\n"
            "        b = d[off:off + n]\n"
            "        s32, s64 = r.getrandbits(32), r.getrandbits(64)\n"
            "        assert ck.crc32c_hw(b, s32) == o.crc32c(b, s32), n\n"
            "        assert ck.crc64ecma_hw(b, s64) == o.crc64ecma(b, s64), n\n")
    env = dict(os.environ, PHOTON_CRC_NO_AVX512="1")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run([sys.executable, "-c", code], check=True, env=env, cwd=repo, timeout=300)
