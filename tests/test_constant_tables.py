"""The constants the PRODUCT generates (photonlibos_amd/csrc/gf2.h, used by
the host drop-in engines and by every device kernel) against the reference's
own COMPILED tables (crc_tables.cpp:104-107, 147-164, dumped by the reference
build into tests/golden/ref_vectors.json), not just through CRC outputs.
Read through tuning.h's photon_crc_test_tables (host-side values; no GPU)."""
import ctypes

import pytest

from photonlibos_amd._native import lib


def _table(which):
    L = lib()
    f = L.photon_crc_test_tables
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
    out = (ctypes.c_uint32 * 256)()
    n = f(which, out, 256)
    assert n > 0, which
    return list(out)[:n]


def test_host_engine_shift_tables_equal_reference(ref_vectors):
    assert _table(0) == ref_vectors["lshift_table_sw"]        # x^(8*2^i)
    assert _table(1) == ref_vectors["rshift_table_sw"]        # x^-(8*2^i)
    assert _table(2)[4:] == ref_vectors["lshift_table_hw"]    # x^(128*2^i - 33)
    assert _table(3) == ref_vectors["rshift_table_hw"]        # x^-(8*2^i + 33)


def test_device_power_tables_equal_reference(ref_vectors):
    assert _table(4) == ref_vectors["lshift_table_sw"]        # combine / fold kernels
    assert _table(5) == ref_vectors["rshift_table_sw"]        # trim kernel


def test_device_kernel_constants_equal_oracle_powers(oracle, ref_vectors):
    # row shifts x^(8*16*G) of the batch kernels, G = 4..64
    assert _table(6) == [oracle.pow32(128 * g) for g in (4, 8, 16, 32, 64)]
    # lane-combine bases x^(128*2^k): k >= 0 are entries 4.. of x^(8*2^i)
    lsh = ref_vectors["lshift_table_sw"]
    assert _table(7) == [lsh[4 + k] for k in range(6)]
    # finish tables F_d of lane groups <= 8: Q -> P (x^32) and the lane shift x^(128d)
    assert _table(9) == [oracle.pow32(32 + 128 * d) for d in range(8)]


def test_slicing_table_equals_oracle(oracle):
    # crc.cpp:82-97 table[0][n]: 8 shift/XOR steps of the polynomial
    want = [oracle.crc32c_bitwise(bytes([b]), 0) for b in range(256)]
    assert _table(8) == want


def test_bad_table_id():
    out = (ctypes.c_uint32 * 256)()
    assert lib().photon_crc_test_tables(99, out, 256) < 0
