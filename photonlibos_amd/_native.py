"""Locate and load the in-tree native library. Fails loudly when it is missing:
there is no Python or CPU stand-in for the device engine."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PHOTON_CRC_LIB: load another build of the library (A/B of two builds on one box).
LIB_PATH = os.environ.get("PHOTON_CRC_LIB") or os.path.join(_HERE, "lib", "libphoton_checksum.so")

_lib = None


class NativeLibraryMissing(ImportError):
    pass


class PhotonRange(ctypes.Structure):
    """photon_crc_range == IOAlloc::RangeSize {int min, max;} (common/io-alloc.h:33)."""
    _fields_ = [("min", ctypes.c_int), ("max", ctypes.c_int)]


def lib():
    """The loaded libphoton_checksum.so (built by __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(or `make -C photonlibos_amd/csrc`)")
        _lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        _declare(_lib)
    return _lib


def _declare(L):
    u8p, u32, u64, sz, vp = ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p
    u32p = ctypes.POINTER(ctypes.c_uint32)

    def fn(name, res, *args):
        f = getattr(L, name)
        f.restype = res
        f.argtypes = list(args)

    # C-ABI (include/photon_crc/crc32c_gpu.h)
    fn("photon_crc_device_count", ctypes.c_int)
    fn("photon_crc_last_error", ctypes.c_char_p)
    fn("photon_crc_scratch_release", ctypes.c_int64)
    fn("photon_crc_set_lanes_per_buffer", ctypes.c_int, ctypes.c_int)
    fn("photon_crc_set_batch_grid", ctypes.c_int, ctypes.c_int)
    fn("photon_crc32c_batch_strided", ctypes.c_int, vp, u64, u64, u64, u32, vp, vp, vp)
    fn("photon_crc32c_batch_strided_sync", ctypes.c_int, vp, u64, u64, u64, u32, vp, vp, vp)
    fn("photon_crc32c_batch_iov", ctypes.c_int, vp, u64, u32, vp, vp, vp)
    fn("photon_crc32c_host_batch_strided", ctypes.c_int, vp, u64, u64, u64, u32, vp, vp)
    fn("photon_crc32c_host_batch_strided_multi", ctypes.c_int, vp, u64, u64, u64, u32, vp, vp, ctypes.c_int)
    fn("photon_crc32c_batch_strided_shards", ctypes.c_int, vp, ctypes.c_int)
    fn("photon_crc32c_batch_msg", ctypes.c_int, vp, vp, u64, u32, vp, vp, vp, vp)
    fn("photon_crc32c_combine_batch", ctypes.c_int, vp, vp, vp, u64, vp, vp)
    fn("photon_crc64ecma_batch_strided", ctypes.c_int, vp, u64, u64, u64, u64, vp, vp, vp)
    fn("photon_crc64ecma_batch_iov", ctypes.c_int, vp, u64, u64, vp, vp, vp)
    fn("photon_crc64ecma_host_batch_strided", ctypes.c_int, vp, u64, u64, u64, u64, vp, vp)
    fn("photon_crc64ecma_trim_batch", ctypes.c_int, vp, vp, vp, u64, vp, vp, vp)
    fn("photon_crc64ecma_combine_batch", ctypes.c_int, vp, vp, vp, u64, vp, vp)
    fn("photon_crc64ecma_batch_msg_n", ctypes.c_int, vp, vp, u64, u64, u64, vp, vp, vp, vp)
    fn("photon_crc64ecma_extend_device", ctypes.c_int, vp, u64, u64, vp, vp)
    fn("photon_crc_util_fill_splitmix", ctypes.c_int, vp, u64, u64, u64, u64, vp)
    fn("photon_crc_util_read_stream", ctypes.c_int, vp, u64, vp, u64, vp)
    fn("photon_crc_set_generic_rows", ctypes.c_int, ctypes.c_int)
    fn("photon_crc_set_long_shape", ctypes.c_int, ctypes.c_int, ctypes.c_int)
    fn("photon_crc_set_msg_mode", ctypes.c_int, ctypes.c_int)
    fn("photon_crc_set_routed_wait", ctypes.c_int, ctypes.c_int, ctypes.c_int)
    fn("photon_crc_set_small_service", ctypes.c_int, ctypes.c_int)
    fn("photon_crc_set_mid_kernel", ctypes.c_int, ctypes.c_int)
    fn("photon_crc_small_service_stats", ctypes.c_int, vp, vp, vp)
    fn("photon_crc_set_small_service_life", ctypes.c_int, ctypes.c_int)
    fn("photon_crc_set_service_doorbell", ctypes.c_int, ctypes.c_int)
    fn("photon_crc_small_service_doorbell", ctypes.c_int, ctypes.c_int)
    fn("photon_crc_small_service_deferred", u64)
    fn("photon_crc64_set_full_rows", ctypes.c_int, ctypes.c_int, ctypes.c_int)
    fn("photon_crc_host_register", ctypes.c_int, vp, u64)
    fn("photon_crc_stream_create", ctypes.c_int, ctypes.POINTER(vp))
    fn("photon_crc_stream_destroy", ctypes.c_int, vp)
    fn("photon_crc_stream_sync", ctypes.c_int, vp)
    fn("photon_crc_stream_on_complete", ctypes.c_int, vp, vp, vp)
    fn("photon_crc_device_alloc", ctypes.c_int, ctypes.POINTER(vp), u64)
    fn("photon_crc_device_free", ctypes.c_int, vp)
    fn("photon_crc_memcpy_async", ctypes.c_int, vp, vp, u64, vp)
    fn("photon_crc_host_unregister", ctypes.c_int, vp)
    fn("photon_crc32c_file_strided", ctypes.c_int, ctypes.c_int, u64, u64, u64, u64, u32, vp)
    fn("photon_crc_dispatch_fallbacks", u64)
    # tuning / test hooks (include/photon_crc/tuning.h)
    fn("photon_crc_lanes_for", ctypes.c_int, u64)
    fn("photon_crc_test_fail_next", None, ctypes.c_int)
    fn("photon_crc_test_long_plan", ctypes.c_int, u64, u64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
       vp, ctypes.c_int)
    fn("photon_crc32c_series_device", ctypes.c_int, vp, u32, u32, vp, vp)
    fn("photon_crc32c_combine_series_device", ctypes.c_int, vp, u32, u32, vp, vp)
    fn("photon_crc32c_trim_batch", ctypes.c_int, vp, vp, vp, u64, vp, vp, vp)
    fn("photon_crc32c_extend_device", ctypes.c_int, vp, u64, u32, vp, vp)
    fn("photon_crc32c_extend_spans", ctypes.c_int, vp, ctypes.c_int, u32, vp)
    fn("photon_crc64ecma_extend_spans", ctypes.c_int, vp, ctypes.c_int, u64, vp)
    fn("photon_crc_set_device_dispatch", ctypes.c_int, ctypes.c_int)
    fn("photon_crc32c_batch_msg_n", ctypes.c_int, vp, vp, u64, u64, u32, vp, vp, vp, vp)
    # include/photon_crc/checked_batch.h
    fn("photon_crc_pinned_allocate", ctypes.c_int, vp, PhotonRange, ctypes.POINTER(vp))
    fn("photon_crc_pinned_deallocate", ctypes.c_int, vp, vp)
    fn("photon_crc_pinned_stats", ctypes.c_int, ctypes.POINTER(u64), ctypes.POINTER(u64))
    fn("photon_crc_pinned_release", ctypes.c_int64)
    fn("photon_crc_msg_batch_create", vp, u32, u32, u32)
    fn("photon_crc_msg_batch_destroy", None, vp)
    fn("photon_crc_msg_batch_add", ctypes.c_int64, vp, vp, u32, vp, u64, u32)
    fn("photon_crc_msg_batch_submit", ctypes.c_int, vp, vp, vp, vp)
    fn("photon_crc_msg_batch_wait", ctypes.c_int64, vp)
    fn("photon_crc_msg_batch_result", ctypes.c_int, vp, u64, ctypes.POINTER(u32))
    fn("photon_crc_msg_batch_count", u64, vp)
    fn("photon_crc_msg_batch_reset", ctypes.c_int, vp)

    # Drop-in host entry points (include/photon/common/checksum/crc32c.h),
    # C++ linkage: bound by their mangled names.
    cpp = {
        "crc32c_sw": ("_Z9crc32c_swPKhmj", u32, u8p, sz, u32),
        "crc32c_hw": ("_Z9crc32c_hwPKhmj", u32, u8p, sz, u32),
        "crc32c_hw_simple": ("_Z16crc32c_hw_simplePKhmj", u32, u8p, sz, u32),
        "crc32c_hw_portable": ("_Z18crc32c_hw_portablePKhmj", u32, u8p, sz, u32),
        "crc32c_series_sw": ("_Z16crc32c_series_swPKhjjPj", None, u8p, u32, u32, u32p),
        "crc32c_series_hw": ("_Z16crc32c_series_hwPKhjjPj", None, u8p, u32, u32, u32p),
        "crc32c_combine_sw": ("_Z17crc32c_combine_swjjj", u32, u32, u32, u32),
        "crc32c_combine_hw": ("_Z17crc32c_combine_hwjjj", u32, u32, u32, u32),
        "crc32c_combine_series_sw": ("_Z24crc32c_combine_series_swPjjj", u32, u32p, u32, u32),
        "crc32c_combine_series_hw": ("_Z24crc32c_combine_series_hwPjjj", u32, u32p, u32, u32),
        "crc32c_trim_sw": ("_Z14crc32c_trim_sw16CRC32C_ComponentS_S_", u32, u64, u64, u64),
        "crc32c_trim_hw": ("_Z14crc32c_trim_hw16CRC32C_ComponentS_S_", u32, u64, u64, u64),
        # CRC-64/ECMA (crc64ecma.h). CRC64ECMA_Component is 16 bytes: passed as two u64 each.
        "crc64ecma_sw": ("_Z12crc64ecma_swPKhmm", u64, u8p, sz, u64),
        "crc64ecma_hw": ("_Z12crc64ecma_hwPKhmm", u64, u8p, sz, u64),
        "crc64ecma_series_sw": ("_Z19crc64ecma_series_swPKhjjPm", None, u8p, u32, u32, ctypes.POINTER(u64)),
        "crc64ecma_series_hw": ("_Z19crc64ecma_series_hwPKhjjPm", None, u8p, u32, u32, ctypes.POINTER(u64)),
        "crc64ecma_combine_sw": ("_Z20crc64ecma_combine_swmmj", u64, u64, u64, u32),
        "crc64ecma_combine_hw": ("_Z20crc64ecma_combine_hwmmj", u64, u64, u64, u32),
        "crc64ecma_combine_series_sw": ("_Z27crc64ecma_combine_series_swPmjj", u64, ctypes.POINTER(u64), u32, u32),
        "crc64ecma_combine_series_hw": ("_Z27crc64ecma_combine_series_hwPmjj", u64, ctypes.POINTER(u64), u32, u32),
        "crc64ecma_trim_sw": ("_Z17crc64ecma_trim_sw19CRC64ECMA_ComponentS_S_", u64, u64, u64, u64, u64, u64, u64),
        "crc64ecma_trim_hw": ("_Z17crc64ecma_trim_hw19CRC64ECMA_ComponentS_S_", u64, u64, u64, u64, u64, u64, u64),
    }
    L.cpp = {}
    for py, (mangled, res, *args) in cpp.items():
        f = getattr(L, mangled)
        f.restype = res
        f.argtypes = list(args)
        L.cpp[py] = f
    # Dispatch pointers (data symbols).
    L.auto = {}
    for name in ("crc32c_auto", "crc32c_series_auto", "crc32c_combine_auto", "crc32c_combine_series_auto",
                 "crc32c_trim_auto", "crc64ecma_auto", "crc64ecma_series_auto", "crc64ecma_combine_auto",
                 "crc64ecma_combine_series_auto", "crc64ecma_trim_auto"):
        L.auto[name] = ctypes.c_void_p.in_dll(L, name)
