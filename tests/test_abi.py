"""The C-ABI library loads and exports every symbol the public headers
declare; without a GPU the device entry points fail loudly (no compute, no
CPU fallback). CPU only."""
import os
import re
import subprocess

import pytest

from photonlibos_amd import _native
from photonlibos_amd import checksum as ck

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _exported():
    out = subprocess.check_output(["nm", "-D", "--defined-only", _native.LIB_PATH], text=True)
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def _c_abi_functions():
    d = os.path.join(REPO, "include", "photon_crc")
    txt = "".join(open(os.path.join(d, h)).read() for h in sorted(os.listdir(d)) if h.endswith(".h"))
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(photon_crc\w*)\s*\(", txt)))


def test_c_abi_symbols_exported():
    names = _c_abi_functions()
    assert len(names) >= 9
    exp = _exported()
    missing = [n for n in names if n not in exp]
    assert not missing, missing


def test_dropin_symbols_exported():
    # The reference's exported C++ symbols, same mangling.
    want = [
        "_Z9crc32c_swPKhmj", "_Z9crc32c_hwPKhmj", "_Z16crc32c_hw_simplePKhmj", "_Z18crc32c_hw_portablePKhmj",
        "_Z16crc32c_series_swPKhjjPj", "_Z16crc32c_series_hwPKhjjPj", "_Z17crc32c_combine_swjjj",
        "_Z17crc32c_combine_hwjjj", "_Z24crc32c_combine_series_swPjjj", "_Z24crc32c_combine_series_hwPjjj",
        "_Z14crc32c_trim_sw16CRC32C_ComponentS_S_", "_Z14crc32c_trim_hw16CRC32C_ComponentS_S_",
        "crc32c_auto", "crc32c_series_auto", "crc32c_combine_auto", "crc32c_combine_series_auto",
        "crc32c_trim_auto",
    ]
    exp = _exported()
    assert not [w for w in want if w not in exp]


@pytest.mark.parametrize("header", ["crc32c.h", "crc64ecma.h"])
def test_header_declarations_are_exported(header):
    # Every non-inline function and dispatch pointer declared in the drop-in
    # headers is defined by the library.
    txt = open(os.path.join(REPO, "include", "photon", "common", "checksum", header)).read()
    decl = re.findall(r"^(?:uint32_t|uint64_t|void)\s+(crc\w+)\(", txt, flags=re.M)
    ptrs = re.findall(r"^extern \w+ \(\*(crc\w+_auto)\)", txt, flags=re.M)
    assert decl and ptrs
    demangled = subprocess.check_output(["nm", "-DC", "--defined-only", _native.LIB_PATH], text=True)
    for d in decl:
        assert re.search(rf"\b{d}\(", demangled), d
    for pname in ptrs:
        assert re.search(rf"\b{pname}$", demangled, flags=re.M), pname


def test_library_is_gfx950_only():
    # One code object, for gfx950, and no other GPU target (no multi-arch dispatch).
    blob = open(_native.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets
    assert set(re.findall(rb"\bgfx[0-9]{3,4}[a-z]?\b", blob)) == {b"gfx950"}


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="a GPU is present")
def test_device_calls_fail_loudly_without_gpu():
    with pytest.raises(ck.CrcError):
        ck.device_count()
    with pytest.raises(ck.CrcError):
        ck.batch_strided(0x1000, 4096, 4096, 1, 0x2000)
    with pytest.raises(ck.CrcError):
        ck.file_strided(0, 0, 4096, 4096, 1)
    with pytest.raises(ck.CrcError):
        ck.host_batch_strided_multi(0x1000, 4096, 4096, 1, 0x2000)
    import ctypes
    from photonlibos_amd._native import lib
    p = ctypes.c_void_p()
    assert lib().photon_crc_device_alloc(ctypes.byref(p), 4096) < 0
    assert lib().photon_crc_stream_create(ctypes.byref(p)) < 0
    with pytest.raises(ck.CrcError):
        ck.batch_strided_shards([dict(device=0, d_base=0x1000, stride=4096, nbytes=4096, count=1, d_out=0x2000)])
    with pytest.raises(ck.CrcError):
        ck.extend_spans([(0, 0x1000, 4096)], 0)
    with pytest.raises(ck.CrcError):
        ck.extend64_spans([(0, 0x1000, 4096)], 0)
    # no spans: nothing to read, the CRC of the empty buffer is the seed (no device needed)
    assert ck.extend_spans([], 0x1234) == 0x1234
    assert ck.extend64_spans([], 7) == 7


def test_argument_validation():
    with pytest.raises(ck.CrcError) as e:
        ck.set_lanes_per_buffer(3)
    assert e.value.code == -22
    with pytest.raises(ck.CrcError):
        ck.batch_strided(None, 4096, 4096, 4, None)
    # tuning knobs added in round 5 (no GPU needed): ranges are checked
    from photonlibos_amd._native import lib
    assert lib().photon_crc_set_mid_kernel(2) == -22
    assert lib().photon_crc_set_mid_kernel(1) == 0
    assert lib().photon_crc_set_small_service(-1) == -22
    assert lib().photon_crc_set_small_service(2000000) == -22
    # round 6: the service's life, its doorbell, the deferred count
    assert lib().photon_crc_set_small_service_life(99) == -22
    assert lib().photon_crc_set_small_service_life(1000001) == -22
    assert lib().photon_crc_set_small_service_life(2000) == 0
    assert lib().photon_crc_set_service_doorbell(2) == -22
    assert lib().photon_crc_set_service_doorbell(0) == 0
    assert lib().photon_crc_set_service_doorbell(1) == 0
    assert lib().photon_crc_small_service_doorbell(5) == -22
    assert lib().photon_crc_small_service_deferred() >= 0


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="a GPU is present")
def test_checked_batch_fails_loudly_without_gpu():
    from photonlibos_amd.checked import MessageBatch, PinnedAlloc
    with pytest.raises(ck.CrcError):
        MessageBatch(16, 16)
    with pytest.raises(ck.CrcError):
        PinnedAlloc().alloc(4096)
    with pytest.raises(ck.CrcError):  # IOAlloc contract: min > 0, max >= min
        PinnedAlloc().alloc(0)
