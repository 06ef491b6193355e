"""ctypes binding of oracle/lib/libcrc_oracle.so (oracle/crc_oracle.c).
TEST INFRASTRUCTURE: the checker, never the thing measured or shipped."""
import ctypes
import os

import numpy as np

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_L = ctypes.CDLL(os.path.join(_REPO, "oracle", "lib", "libcrc_oracle.so"), use_errno=True)

_u32, _u64, _sz, _p, _vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_void_p
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
    ("or_crc32c_table", _vp, [ctypes.c_int]),
    ("or_crc32c_strided", None, [_vp, _u64, _u64, _u64, _u32, _vp]),
    ("or_crc64ecma_strided", None, [_vp, _u64, _u64, _u64, _u64, _vp]),
    ("or_crc32c_iov", None, [_vp, _u64, _vp]),
    ("or_crc32c_msg_chain", None, [_vp, _vp, _u64, _vp, _u32, _vp]),
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


def checked_message_object(segments, struct_bytes):
    """CheckedMessage<Crc32Hasher>::add_checksum / validate_checksum as the
    reference runs them on a message OBJECT (rpc/serialize.h:244-275, 425,
    462-463): extend_hash accumulates into m_checksum by reference, and
    m_checksum is the struct's first 4 bytes, so the struct is hashed while
    it holds the running CRC of the payload."""
    acc = extend_chain(segments, 0)
    b = bytearray(_b(struct_bytes))
    b[:4] = acc.to_bytes(4, "little")
    return crc32c(bytes(b), acc)


# ---------------------------------------------------------------- batches
# Full-size parity (tests/test_gpu_fullsize.py): the same oracle functions in
# C loops, fanned out over a thread pool (ctypes releases the GIL). Host
# arrays are passed by address, never copied.

def _threads():
    # the GPU box gives a job 16 CPUs; nproc shows the whole machine there
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def _fan_out(count, fn, threads=None):
    from concurrent.futures import ThreadPoolExecutor
    t = threads or _threads()
    cuts = [count * k // t for k in range(t + 1)]
    with ThreadPoolExecutor(t) as ex:
        list(ex.map(lambda k: fn(cuts[k], cuts[k + 1]), range(t)))


def crc32c_strided(host, stride, nbytes, count, seed=0):
    """CRC32C of `count` buffers at host[i*stride : i*stride+nbytes] (numpy uint8)."""
    assert host.dtype == np.uint8 and host.flags.c_contiguous
    assert count == 0 or (count - 1) * stride + nbytes <= host.size
    _L.or_crc32c_table(0)
    out = np.zeros(count, np.uint32)
    base = host.ctypes.data

    def part(lo, hi):
        if hi > lo:
            _L.or_crc32c_strided(base + lo * stride, stride, nbytes, hi - lo, seed & 0xFFFFFFFF,
                                 out.ctypes.data + 4 * lo)
    _fan_out(count, part)
    return out


def crc64ecma_strided(host, stride, nbytes, count, seed=0):
    assert host.dtype == np.uint8 and host.flags.c_contiguous
    assert count == 0 or (count - 1) * stride + nbytes <= host.size
    crc64ecma(b"")  # builds the table before the threads start
    out = np.zeros(count, np.uint64)
    base = host.ctypes.data

    def part(lo, hi):
        if hi > lo:
            _L.or_crc64ecma_strided(base + lo * stride, stride, nbytes, hi - lo, seed, out.ctypes.data + 8 * lo)
    _fan_out(count, part)
    return out


def crc32c_iov(iov):
    """Seed-0 CRC32C of every {host address, length} row of `iov` (uint64, shape (n, 2))."""
    iov = np.ascontiguousarray(iov, np.uint64)
    _L.or_crc32c_table(0)
    n = iov.shape[0]
    out = np.zeros(n, np.uint32)

    def part(lo, hi):
        if hi > lo:
            _L.or_crc32c_iov(iov.ctypes.data + 16 * lo, hi - lo, out.ctypes.data + 4 * lo)
    _fan_out(n, part)
    return out


def msg_chain(iov, msg_start, seeds=None, seed0=0):
    """extend_chain per message over host iovecs: message m = segments msg_start[m]..msg_start[m+1]-1."""
    iov = np.ascontiguousarray(iov, np.uint64)
    msg_start = np.ascontiguousarray(msg_start, np.uint64)
    seeds = None if seeds is None else np.ascontiguousarray(seeds, np.uint32)
    _L.or_crc32c_table(0)
    nmsg = msg_start.size - 1
    out = np.zeros(nmsg, np.uint32)

    def part(lo, hi):
        if hi > lo:
            _L.or_crc32c_msg_chain(iov.ctypes.data, msg_start.ctypes.data + 8 * lo, hi - lo,
                                   None if seeds is None else seeds.ctypes.data + 4 * lo, seed0 & 0xFFFFFFFF,
                                   out.ctypes.data + 4 * lo)
    _fan_out(nmsg, part)
    return out
