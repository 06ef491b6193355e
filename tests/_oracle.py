"""ctypes binding of oracle/lib/libcrc_oracle.so (oracle/crc_oracle.c).
TEST INFRASTRUCTURE: the checker, never the thing measured or shipped."""
import ctypes
import os

import numpy as np

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_L = ctypes.CDLL(os.path.join(_REPO, "oracle", "lib", "libcrc_oracle.so"), use_errno=True)

_u32, _u64, _sz, _p = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_char_p
for name, res, args in [
    ("or_crc32c_sw", _u32, [_p, _sz, _u32]),
    ("or_crc32c_bitwise", _u32, [_p, _sz, _u32]),
    ("or_clmul_modp32", _u32, [_u32, _u32]),
    ("or_pow32", _u32, [_u64]),
    ("or_ipow32", _u32, [_u64]),
    ("or_crc32c_lshift_hw", _u32, [ctypes.c_uint]),
    ("or_crc32c_rshift_hw", _u32, [ctypes.c_uint]),
    ("or_crc32c_lshift_sw", _u32, [ctypes.c_uint]),
    ("or_crc32c_rshift_sw", _u32, [ctypes.c_uint]),
    ("or_crc32c_combine", _u32, [_u32, _u32, _u32]),
    ("or_crc32c_combine_series", _u32, [ctypes.POINTER(_u32), _u32, _u32]),
    ("or_crc32c_series", None, [_p, _u32, _u32, ctypes.POINTER(_u32)]),
    ("or_crc32c_series_hw", None, [_p, _u32, _u32, ctypes.POINTER(_u32)]),
    ("or_crc32c_trim", _u32, [_u32, _u32, _u32, _u32, _u32, _u32]),
    ("or_crc64ecma_sw", _u64, [_p, _sz, _u64]),
]:
    f = getattr(_L, name)
    f.restype = res
    f.argtypes = args


def _b(data):
    if isinstance(data, np.ndarray):
        return data.tobytes()
    return bytes(data)


def crc32c(data, crc=0):
    b = _b(data)
    return _L.or_crc32c_sw(b, len(b), crc & 0xFFFFFFFF)


def crc32c_bitwise(data, crc=0):
    b = _b(data)
    return _L.or_crc32c_bitwise(b, len(b), crc & 0xFFFFFFFF)


def crc64ecma(data, crc=0):
    b = _b(data)
    return _L.or_crc64ecma_sw(b, len(b), crc)


def combine(c1, c2, len2):
    return _L.or_crc32c_combine(c1, c2, len2)


def combine_series(crcs, part_size):
    arr = (_u32 * max(len(crcs), 1))(*crcs)
    return _L.or_crc32c_combine_series(arr, part_size, len(crcs))


def series(buf, part_size, n_parts, hw_quirk=False):
    b = _b(buf)
    out = (_u32 * max(n_parts, 1))()
    (_L.or_crc32c_series_hw if hw_quirk else _L.or_crc32c_series)(b, part_size, n_parts, out)
    return list(out)[:n_parts]


def trim(all_, prefix, suffix):
    return _L.or_crc32c_trim(all_[0], all_[1], prefix[0], prefix[1], suffix[0], suffix[1])


def errno():
    return ctypes.get_errno()


pow32 = _L.or_pow32
ipow32 = _L.or_ipow32
clmul_modp32 = _L.or_clmul_modp32
lshift_hw = _L.or_crc32c_lshift_hw
rshift_hw = _L.or_crc32c_rshift_hw
lshift_sw = _L.or_crc32c_lshift_sw
rshift_sw = _L.or_crc32c_rshift_sw


def extend_chain(segments, seed=0):
    """Crc32Hasher::extend_hash (rpc/serialize.h:244-247): chained crc32c_extend."""
    c = seed
    for s in segments:
        c = crc32c(s, c)
    return c
