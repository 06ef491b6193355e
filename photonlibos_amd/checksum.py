"""Host-side mirror of PhotonLibOS common/checksum (CRC32C) over the C-ABI
library libphoton_checksum.so.

Two layers, both thin bindings (no arithmetic in Python):

* Drop-in entry points with the reference's names and meaning
  (common/checksum/crc32c.h:20-92): crc32c, crc32c_extend, crc32c_series,
  crc32c_combine, crc32c_combine_series, crc32c_trim (+ the _sw/_hw engines),
  bound to the library's exported C++ symbols and dispatch pointers.
* The batched device engine (include/photon_crc/crc32c_gpu.h):
  batch_strided / batch_iov / batch_msg / combine_batch. Arguments are device
  pointers (ints) or objects exposing .data_ptr() (e.g. torch tensors);
  `stream` is a hipStream_t handle (int) or an object with .cuda_stream.
  Errors raise CrcError; nothing falls back to the CPU.
"""
import ctypes

from ._native import lib

__all__ = [
    "CrcError",
    "crc32c", "crc32c_extend", "crc32c_sw", "crc32c_hw", "crc32c_hw_simple", "crc32c_hw_portable",
    "crc32c_series", "crc32c_series_sw", "crc32c_series_hw",
    "crc32c_combine", "crc32c_combine_sw", "crc32c_combine_hw",
    "crc32c_combine_series", "crc32c_combine_series_sw", "crc32c_combine_series_hw",
    "crc32c_trim", "crc32c_trim_sw", "crc32c_trim_hw", "is_crc32c_hw_available",
    "device_count", "set_lanes_per_buffer", "host_batch_strided", "host_batch_strided_multi", "batch_strided_shards",
    "Shard", "batch_strided", "batch_strided_sync", "batch_iov", "batch_msg",
    "crc64ecma", "crc64ecma_extend", "crc64ecma_sw", "crc64ecma_hw", "crc64ecma_combine", "crc64ecma_series",
    "crc64ecma_combine_series", "crc64ecma_trim",
    "batch64_strided", "batch64_iov", "combine64_batch", "trim64_batch", "batch64_msg_n", "host_batch64_strided", "extend64_device", "extend_spans", "extend64_spans", "Span", "combine_batch", "fill_splitmix", "read_stream", "IOVEC_DTYPE",
]

_CRC_FN = ctypes.CFUNCTYPE(ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32)
_SERIES_FN = ctypes.CFUNCTYPE(None, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                              ctypes.POINTER(ctypes.c_uint32))
_COMB_FN = ctypes.CFUNCTYPE(ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32)
_CSER_FN = ctypes.CFUNCTYPE(ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32, ctypes.c_uint32)
_TRIM_FN = ctypes.CFUNCTYPE(ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64)


class CrcError(RuntimeError):
    def __init__(self, code, what):
        super().__init__(f"photon_crc error {code}: {what}")
        self.code = code


def _auto(name, proto):
    return proto(lib().auto[name].value)


def _buf(data):
    if isinstance(data, str):
        data = data.encode()
    mv = memoryview(data).cast("B")
    if mv.readonly:
        return bytes(mv), len(mv)
    return (ctypes.c_char * len(mv)).from_buffer(mv), len(mv)


# ---------------------------------------------------------------- drop-in API

def crc32c_extend(data, crc):
    """crc32c_extend(data, nbytes, crc) (crc32c.h:30-33, 39-41)."""
    b, n = _buf(data)
    return _auto("crc32c_auto", _CRC_FN)(ctypes.cast(b, ctypes.c_char_p) if not isinstance(b, bytes) else b,
                                         n, crc & 0xFFFFFFFF)


def crc32c(data):
    """crc32c(data, nbytes) == crc32c_extend(data, nbytes, 0) (crc32c.h:35-45)."""
    return crc32c_extend(data, 0)


def _engine(name):
    def f(data, crc=0):
        b, n = _buf(data)
        return lib().cpp[name](ctypes.cast(b, ctypes.c_char_p) if not isinstance(b, bytes) else b, n,
                               crc & 0xFFFFFFFF)
    f.__name__ = name
    f.__doc__ = f"{name}(buffer, nbytes, crc) (crc32c.h:20-22)."
    return f


crc32c_sw = _engine("crc32c_sw")
crc32c_hw = _engine("crc32c_hw")
crc32c_hw_simple = _engine("crc32c_hw_simple")
crc32c_hw_portable = _engine("crc32c_hw_portable")


def _series(fn, buffer, part_size, n_parts):
    b, n = _buf(buffer)
    out = (ctypes.c_uint32 * max(n_parts, 1))()
    fn(ctypes.cast(b, ctypes.c_char_p) if not isinstance(b, bytes) else b, part_size, n_parts, out)
    return list(out)[:n_parts]


def crc32c_series(buffer, part_size, n_parts):
    """crc32c_series (crc32c.h:47-57): CRCs of n_parts consecutive parts."""
    return _series(_auto("crc32c_series_auto", _SERIES_FN), buffer, part_size, n_parts)


def crc32c_series_sw(buffer, part_size, n_parts):
    return _series(lib().cpp["crc32c_series_sw"], buffer, part_size, n_parts)


def crc32c_series_hw(buffer, part_size, n_parts):
    return _series(lib().cpp["crc32c_series_hw"], buffer, part_size, n_parts)


def crc32c_combine(crc1, crc2, len2):
    """crc32c_combine (crc32c.h:59-66): crc(A||B) from crc(A), crc(B), |B|."""
    return _auto("crc32c_combine_auto", _COMB_FN)(crc1, crc2, len2)


def crc32c_combine_sw(crc1, crc2, len2):
    return lib().cpp["crc32c_combine_sw"](crc1, crc2, len2)


def crc32c_combine_hw(crc1, crc2, len2):
    return lib().cpp["crc32c_combine_hw"](crc1, crc2, len2)


def _cseries(fn, crcs, part_size):
    arr = (ctypes.c_uint32 * max(len(crcs), 1))(*crcs)
    return fn(arr, part_size, len(crcs))


def crc32c_combine_series(crcs, part_size):
    """crc32c_combine_series (crc32c.h:68-74); 0 for an empty list."""
    return _cseries(_auto("crc32c_combine_series_auto", _CSER_FN), crcs, part_size)


def crc32c_combine_series_sw(crcs, part_size):
    return _cseries(lib().cpp["crc32c_combine_series_sw"], crcs, part_size)


def crc32c_combine_series_hw(crcs, part_size):
    return _cseries(lib().cpp["crc32c_combine_series_hw"], crcs, part_size)


def _comp(c):
    crc, size = c
    return (crc & 0xFFFFFFFF) | ((size & 0xFFFFFFFF) << 32)


def _trim(fn, all_, prefix, suffix):
    return fn(_comp(all_), _comp(prefix), _comp(suffix))


def crc32c_trim(all_, prefix, suffix):
    """crc32c_trim (crc32c.h:76-87); components are (crc, size) pairs.
    Inconsistent sizes: returns 0 with errno = EINVAL, like the reference."""
    return _trim(_auto("crc32c_trim_auto", _TRIM_FN), all_, prefix, suffix)


def crc32c_trim_sw(all_, prefix, suffix):
    return _trim(lib().cpp["crc32c_trim_sw"], all_, prefix, suffix)


def crc32c_trim_hw(all_, prefix, suffix):
    return _trim(lib().cpp["crc32c_trim_hw"], all_, prefix, suffix)


def is_crc32c_hw_available():
    """crc32c.h:89-92."""
    L = lib()
    return L.auto["crc32c_auto"].value != ctypes.cast(L.cpp["crc32c_sw"], ctypes.c_void_p).value


# ------------------------------------------------------------ CRC-64/ECMA drop-in

_CRC64_FN = ctypes.CFUNCTYPE(ctypes.c_uint64, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64)
_COMB64_FN = ctypes.CFUNCTYPE(ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32)
_TRIM64_FN = ctypes.CFUNCTYPE(ctypes.c_uint64, *([ctypes.c_uint64] * 6))


def _cp(b):
    return ctypes.cast(b, ctypes.c_char_p) if not isinstance(b, bytes) else b


def crc64ecma_extend(data, crc):
    """crc64ecma_extend (crc64ecma.h:23-30): inverted in and out (crc.cpp:119-122)."""
    b, n = _buf(data)
    return _auto("crc64ecma_auto", _CRC64_FN)(_cp(b), n, crc & 0xFFFFFFFFFFFFFFFF)


def crc64ecma(data, crc=0):
    """crc64ecma(buffer, nbytes, crc) (crc64ecma.h:36-38)."""
    return crc64ecma_extend(data, crc)


def crc64ecma_sw(data, crc=0):
    b, n = _buf(data)
    return lib().cpp["crc64ecma_sw"](_cp(b), n, crc & 0xFFFFFFFFFFFFFFFF)


def crc64ecma_hw(data, crc=0):
    b, n = _buf(data)
    return lib().cpp["crc64ecma_hw"](_cp(b), n, crc & 0xFFFFFFFFFFFFFFFF)


def crc64ecma_combine(crc1, crc2, len2):
    """crc64ecma_combine (crc64ecma.h:53-58)."""
    return _auto("crc64ecma_combine_auto", _COMB64_FN)(crc1, crc2, len2)


def crc64ecma_series(buffer, part_size, n_parts):
    b, n = _buf(buffer)
    out = (ctypes.c_uint64 * max(n_parts, 1))()
    lib().cpp["crc64ecma_series_sw"](_cp(b), part_size, n_parts, out)
    return list(out)[:n_parts]


def crc64ecma_combine_series(crcs, part_size):
    arr = (ctypes.c_uint64 * max(len(crcs), 1))(*crcs)
    return lib().cpp["crc64ecma_combine_series_sw"](arr, part_size, len(crcs))


def crc64ecma_trim(all_, prefix, suffix):
    """crc64ecma_trim (crc64ecma.h:68-87); components are (crc, size)."""
    return _auto("crc64ecma_trim_auto", _TRIM64_FN)(all_[0], all_[1], prefix[0], prefix[1], suffix[0], suffix[1])


# ---------------------------------------------------------- batched device API

IOVEC_DTYPE = [("base", "<u8"), ("len", "<u8")]  # == struct iovec / photon_crc_iovec


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    raise TypeError(f"expected a device pointer (int) or an object with data_ptr(), got {type(x)!r}")


def _stream(s):
    if s is None:
        return None
    if isinstance(s, int):
        return s
    return s.cuda_stream


def _check(rc):
    if rc != 0:
        raise CrcError(rc, lib().photon_crc_last_error().decode(errors="replace"))


def device_count():
    """Number of usable gfx950 devices; raises CrcError if there is none."""
    n = lib().photon_crc_device_count()
    if n < 0:
        _check(n)
    return n


def set_lanes_per_buffer(g):
    """Lanes per buffer for the batch kernels (0 = automatic, else 4..64)."""
    _check(lib().photon_crc_set_lanes_per_buffer(g))


def batch_strided(base, stride, nbytes, count, out, seed=0, seeds=None, stream=None):
    """out[i] = crc32c_extend(base + i*stride, nbytes, seeds[i] or seed). Async."""
    _check(lib().photon_crc32c_batch_strided(_ptr(base), stride, nbytes, count, seed & 0xFFFFFFFF, _ptr(seeds),
                                             _ptr(out), _stream(stream)))


def batch_strided_sync(base, stride, nbytes, count, out, seed=0, seeds=None, stream=None):
    _check(lib().photon_crc32c_batch_strided_sync(_ptr(base), stride, nbytes, count, seed & 0xFFFFFFFF,
                                                  _ptr(seeds), _ptr(out), _stream(stream)))


def host_batch_strided(base, stride, nbytes, count, out, seed=0, seeds=None):
    """Host-memory batch through the device (chunked H2D + kernel + D2H). Synchronous.
    base/out/seeds are host pointers (ints) or objects with data_ptr() (pinned tensors)."""
    _check(lib().photon_crc32c_host_batch_strided(_ptr(base), stride, nbytes, count, seed & 0xFFFFFFFF,
                                                  _ptr(seeds), _ptr(out)))


def host_batch_strided_multi(base, stride, nbytes, count, out, seed=0, seeds=None, ndev=0):
    """host_batch_strided sharded over `ndev` devices of this process (0 = all),
    one host thread per device. Synchronous."""
    _check(lib().photon_crc32c_host_batch_strided_multi(_ptr(base), stride, nbytes, count, seed & 0xFFFFFFFF,
                                                        _ptr(seeds), _ptr(out), ndev))


class Shard(ctypes.Structure):
    """photon_crc_shard (include/photon_crc/crc32c_gpu.h)."""
    _fields_ = [("device", ctypes.c_int), ("d_base", ctypes.c_void_p), ("stride", ctypes.c_uint64),
                ("nbytes", ctypes.c_uint64), ("count", ctypes.c_uint64), ("seed0", ctypes.c_uint32),
                ("d_seeds", ctypes.c_void_p), ("d_out", ctypes.c_void_p), ("stream", ctypes.c_void_p)]


def batch_strided_shards(shards):
    """shards: list of dicts with Shard's fields (pointers as ints or .data_ptr()
    objects). Enqueues batch_strided on every shard's device. Async."""
    arr = (Shard * len(shards))()
    for a, s in zip(arr, shards):
        a.device = s.get("device", 0)
        a.d_base = _ptr(s["d_base"])
        a.stride, a.nbytes, a.count = s["stride"], s["nbytes"], s["count"]
        a.seed0 = s.get("seed0", 0) & 0xFFFFFFFF
        a.d_seeds = _ptr(s.get("d_seeds"))
        a.d_out = _ptr(s["d_out"])
        a.stream = _stream(s.get("stream"))
    _check(lib().photon_crc32c_batch_strided_shards(arr, len(shards)))


def batch_iov(iov, count, out, seed=0, seeds=None, stream=None):
    """out[i] = crc32c_extend(iov[i].base, iov[i].len, seed_i). Async."""
    _check(lib().photon_crc32c_batch_iov(_ptr(iov), count, seed & 0xFFFFFFFF, _ptr(seeds), _ptr(out),
                                         _stream(stream)))


def batch_msg(iov, msg_start, nmsg, seg_out, out, seed=0, seeds=None, stream=None):
    """out[m] = chained crc32c_extend over message m's segments. Async."""
    _check(lib().photon_crc32c_batch_msg(_ptr(iov), _ptr(msg_start), nmsg, seed & 0xFFFFFFFF, _ptr(seeds),
                                         _ptr(seg_out), _ptr(out), _stream(stream)))


def batch_msg_n(iov, msg_start, nmsg, nseg, seg_out, out, seed=0, seeds=None, stream=None):
    """batch_msg with the total segment count supplied (fully asynchronous)."""
    _check(lib().photon_crc32c_batch_msg_n(_ptr(iov), _ptr(msg_start), nmsg, nseg, seed & 0xFFFFFFFF, _ptr(seeds),
                                           _ptr(seg_out), _ptr(out), _stream(stream)))


def batch64_strided(base, stride, nbytes, count, out, seed=0, seeds=None, stream=None):
    """out[i] = crc64ecma_extend(base + i*stride, nbytes, seeds[i] or seed) (uint64 out). Async."""
    _check(lib().photon_crc64ecma_batch_strided(_ptr(base), stride, nbytes, count, seed & 0xFFFFFFFFFFFFFFFF,
                                                _ptr(seeds), _ptr(out), _stream(stream)))


def batch64_iov(iov, count, out, seed=0, seeds=None, stream=None):
    """out[i] = crc64ecma_extend(iov[i].base, iov[i].len, seed_i) (uint64 out). Async."""
    _check(lib().photon_crc64ecma_batch_iov(_ptr(iov), count, seed & 0xFFFFFFFFFFFFFFFF, _ptr(seeds), _ptr(out),
                                            _stream(stream)))


def host_batch64_strided(base, stride, nbytes, count, out, seed=0, seeds=None):
    """CRC-64/ECMA host-memory batch (chunked H2D + kernel + D2H). Synchronous."""
    _check(lib().photon_crc64ecma_host_batch_strided(_ptr(base), stride, nbytes, count, seed & 0xFFFFFFFFFFFFFFFF,
                                                     _ptr(seeds), _ptr(out)))


def trim64_batch(all_, prefix, suffix, count, out, nerr=None, stream=None):
    """out[i] = crc64ecma_trim(all_[i], prefix[i], suffix[i]); arrays of 16-byte
    {crc, size} components (device). Async."""
    _check(lib().photon_crc64ecma_trim_batch(_ptr(all_), _ptr(prefix), _ptr(suffix), count, _ptr(out), _ptr(nerr),
                                             _stream(stream)))


def combine64_batch(crc1, crc2, len2, count, out, stream=None):
    """out[i] = crc64ecma_combine(crc1[i], crc2[i], len2[i]) (uint64 crcs, uint32 lengths). Async."""
    _check(lib().photon_crc64ecma_combine_batch(_ptr(crc1), _ptr(crc2), _ptr(len2), count, _ptr(out),
                                                _stream(stream)))


def batch64_msg_n(iov, msg_start, nmsg, nseg, seg_out, out, seed=0, seeds=None, stream=None):
    """out[m] = crc64ecma_extend chained over message m's segments (uint64). Async."""
    _check(lib().photon_crc64ecma_batch_msg_n(_ptr(iov), _ptr(msg_start), nmsg, nseg, seed & 0xFFFFFFFFFFFFFFFF,
                                              _ptr(seeds), _ptr(seg_out), _ptr(out), _stream(stream)))


def extend64_device(data, nbytes, out, seed=0, stream=None):
    """*out = crc64ecma_extend(data, nbytes, seed) for one long device buffer. Async."""
    _check(lib().photon_crc64ecma_extend_device(_ptr(data), nbytes, seed & 0xFFFFFFFFFFFFFFFF, _ptr(out),
                                                _stream(stream)))


def combine_batch(crc1, crc2, len2, count, out, stream=None):
    """out[i] = crc32c_combine(crc1[i], crc2[i], len2[i]). Async."""
    _check(lib().photon_crc32c_combine_batch(_ptr(crc1), _ptr(crc2), _ptr(len2), count, _ptr(out),
                                             _stream(stream)))


def series_device(buffer, part_size, n_parts, out, stream=None):
    """crc32c_series over device memory (crc32c.h:52-57). Async."""
    _check(lib().photon_crc32c_series_device(_ptr(buffer), part_size, n_parts, _ptr(out), _stream(stream)))


def combine_series_device(crcs, part_size, n_parts, result, stream=None):
    """*result = crc32c_combine_series(crcs, part_size, n_parts) on the device (crc32c.h:71-74). Async."""
    _check(lib().photon_crc32c_combine_series_device(_ptr(crcs), part_size, n_parts, _ptr(result),
                                                     _stream(stream)))


def trim_batch(all_, prefix, suffix, count, out, nerr=None, stream=None):
    """out[i] = crc32c_trim(all_[i], prefix[i], suffix[i]); components are {u32 crc, u32 size}
    pairs (crc32c.h:76-87). *nerr counts inconsistent elements (their out is 0). Async."""
    _check(lib().photon_crc32c_trim_batch(_ptr(all_), _ptr(prefix), _ptr(suffix), count, _ptr(out),
                                          _ptr(nerr) if nerr is not None else None, _stream(stream)))


def extend_device(data, nbytes, seed, out, stream=None):
    """*out = crc32c_extend(data, nbytes, seed) for one long device buffer. Async."""
    _check(lib().photon_crc32c_extend_device(_ptr(data), nbytes, seed & 0xFFFFFFFF, _ptr(out), _stream(stream)))


class Span(ctypes.Structure):
    """photon_crc_span (include/photon_crc/crc32c_gpu.h)."""
    _fields_ = [("device", ctypes.c_int), ("d_data", ctypes.c_void_p), ("nbytes", ctypes.c_uint64)]


def _spans(spans):
    arr = (Span * max(1, len(spans)))()
    for a, (dev, ptr, n) in zip(arr, spans):
        a.device, a.d_data, a.nbytes = dev, _ptr(ptr), n
    return arr


def extend_spans(spans, seed=0):
    """crc32c_extend over ONE buffer whose bytes lie on several devices:
    spans = [(device, device_pointer, nbytes), ...] in buffer order. Synchronous."""
    res = ctypes.c_uint32(0)
    _check(lib().photon_crc32c_extend_spans(_spans(spans), len(spans), seed & 0xFFFFFFFF, ctypes.byref(res)))
    return res.value


def extend64_spans(spans, seed=0):
    """crc64ecma_extend over ONE buffer spanning devices (see extend_spans). Synchronous."""
    res = ctypes.c_uint64(0)
    _check(lib().photon_crc64ecma_extend_spans(_spans(spans), len(spans), seed & 0xFFFFFFFFFFFFFFFF,
                                               ctypes.byref(res)))
    return res.value


def set_device_dispatch(on):
    """Route crc32c_auto / crc32c_series_auto / crc32c_combine_series_auto to the
    device for device pointers (photon_crc_set_device_dispatch). Raises
    CrcError(-EIO) if a routed call failed on the device since the last switch
    (it was recomputed on the host: dispatch_fallbacks())."""
    _check(lib().photon_crc_set_device_dispatch(1 if on else 0))


def dispatch_fallbacks():
    """Routed calls whose device work failed and were recomputed on the host."""
    return int(lib().photon_crc_dispatch_fallbacks())


def lanes_for(nbytes):
    """Lanes per buffer the engine picks for buffers of nbytes (tuning.h)."""
    return int(lib().photon_crc_lanes_for(nbytes))


def inject_failures(n):
    """tuning.h failure injection: the next n device entry points called on
    this thread return -EIO before enqueuing anything."""
    lib().photon_crc_test_fail_next(n)


_CRC_PTR_FN = ctypes.CFUNCTYPE(ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32)
_SERIES_PTR_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p)
_CSER_PTR_FN = ctypes.CFUNCTYPE(ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32)


def crc32c_extend_at(addr, nbytes, crc=0):
    """crc32c_extend through the crc32c_auto pointer on a raw address (what a
    C++ caller holding a device pointer would call)."""
    return _auto("crc32c_auto", _CRC_PTR_FN)(addr, nbytes, crc & 0xFFFFFFFF)


_CRC64_PTR_FN = ctypes.CFUNCTYPE(ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64)


def crc64ecma_extend_at(addr, nbytes, crc=0):
    """crc64ecma_extend through the crc64ecma_auto pointer on a raw address."""
    return _auto("crc64ecma_auto", _CRC64_PTR_FN)(addr, nbytes, crc & 0xFFFFFFFFFFFFFFFF)


def crc32c_series_at(addr, part_size, n_parts, out_addr):
    """crc32c_series through crc32c_series_auto on raw addresses."""
    _auto("crc32c_series_auto", _SERIES_PTR_FN)(addr, part_size, n_parts, out_addr)


def crc32c_combine_series_at(addr, part_size, n_parts):
    """crc32c_combine_series through crc32c_combine_series_auto on a raw address."""
    return _auto("crc32c_combine_series_auto", _CSER_PTR_FN)(addr, part_size, n_parts)


def host_register(addr, nbytes):
    """Make host memory [addr, addr+nbytes) device-readable in place."""
    _check(lib().photon_crc_host_register(addr, nbytes))


def host_unregister(addr):
    _check(lib().photon_crc_host_unregister(addr))


def file_strided(fd, offset, stride, nbytes, count, seed=0):
    """CRC32C of `count` records of `nbytes` at offset + i*stride of file descriptor fd
    (pread into pinned chunks + GPU pipeline). Returns a list of ints."""
    out = (ctypes.c_uint32 * max(count, 1))()
    _check(lib().photon_crc32c_file_strided(fd, offset, stride, nbytes, count, seed & 0xFFFFFFFF, out))
    return list(out)[:count]


def set_generic_rows(u):
    """Batch kernel variant: -1 (default) = by lane-group size; 2, 4, 8 = rows
    per step of the generic kernel."""
    _check(lib().photon_crc_set_generic_rows(u))


def set_msg_mode(mode):
    """Message batches: 0 automatic, 1 one fused kernel, 2 segment + fold kernels."""
    _check(lib().photon_crc_set_msg_mode(mode))


def set_long_shape(lanes=0, rounds=0):
    """One long buffer (extend_device / extend64_device): lanes per chunk (0 =
    automatic, 32, 64) and chunks per lane group of the grid (0 = automatic)."""
    _check(lib().photon_crc_set_long_shape(lanes, rounds))


def set_routed_wait(spin_us=40, sleep_ahead=True):
    """Routed drop-in calls: tag-polling window in µs, then a blocking wait;
    sleep_ahead: long calls sleep through their expected time first (tuning)."""
    _check(lib().photon_crc_set_routed_wait(spin_us, 1 if sleep_ahead else 0))


def set_mid_kernel(on=True):
    """Spans over 256 KiB up to 32 MiB: the mid layout (default) or, off, the
    long kernel (tuning; tests of the long kernel's plan)."""
    _check(lib().photon_crc_set_mid_kernel(1 if on else 0))


def set_small_service(idle_us):
    """Routed small crc32c_extend / crc64ecma_extend calls through a resident
    service launch that ends after idle_us without a call; 0 = off, a launch
    per call; default 200 or PHOTON_CRC_SMALL_SERVICE (tuning)."""
    _check(lib().photon_crc_set_small_service(int(idle_us)))


def set_small_service_life(life_us):
    """Life of one service launch (default 2000 us): the bound on how long a
    device-wide wait stalls behind it under steady routed traffic (tuning)."""
    _check(lib().photon_crc_set_small_service_life(int(life_us)))


def set_service_doorbell(bar):
    """The service's doorbell: True = device memory through the PCIe BAR (the
    default, when the host mapping was verified), False = pinned host memory.
    Ends running launches (tuning)."""
    _check(lib().photon_crc_set_service_doorbell(1 if bar else 0))


def small_service_doorbell(kind=0):
    """'bar' or 'pinned': the doorbell the current device's service of `kind`
    (0 CRC-32C, 1 CRC-64) rings; None if that service was never started."""
    r = lib().photon_crc_small_service_doorbell(int(kind))
    if r == -2:  # -ENOENT
        return None
    _check(r if r < 0 else 0)
    return "bar" if r == 1 else "pinned"


def small_service_deferred():
    """Routed small calls that took the launch path because a batch / long
    launch of the library was in flight when they would have started a
    service launch (tests)."""
    return int(lib().photon_crc_small_service_deferred())


def small_service_stats():
    """(served, starts, missed): routed small calls the service served, its
    launches, calls that found it ending (tests)."""
    import ctypes
    v = [ctypes.c_uint64(0) for _ in range(3)]
    _check(lib().photon_crc_small_service_stats(*[ctypes.byref(x) for x in v]))
    return tuple(x.value for x in v)


def set_full_rows64(mode, rows_per_step=2):
    """CRC-64 whole-step uniform batches: 0 generic kernel, 1 full-row kernel,
    2 full-row kernel with cross-buffer prefetch, 3 automatic (the default:
    2 for buffers up to 8 KiB) (tuning)."""
    _check(lib().photon_crc64_set_full_rows(mode, rows_per_step))


def set_msg_rows(u):
    """Rows per step of the one-kernel message form (2 or 4; tuning)."""
    _check(lib().photon_crc_set_msg_rows(u))


def read_stream(base, nbytes, sink, sink_words, stream=None):
    """Bench utility: HBM read-only stream over nbytes (achievable-roofline probe)."""
    _check(lib().photon_crc_util_read_stream(_ptr(base), nbytes, _ptr(sink), sink_words, _stream(stream)))


def fill_splitmix(base, stride, nbytes, count, seed_base, stream=None):
    """Test/bench utility: device buffers = photonlibos_amd.datagen streams."""
    _check(lib().photon_crc_util_fill_splitmix(_ptr(base), stride, nbytes, count, seed_base, _stream(stream)))


def scratch_release():
    """Free the device scratch buffers the library keeps idle (bytes freed)."""
    return int(lib().photon_crc_scratch_release())
