"""Producers outside device memory: records of a file
(photon_crc32c_file_strided: pread into pinned chunks + GPU pipeline, O_DIRECT
when the filesystem allows it) and registered host memory read in place by the
message batch. Checked against the pinned oracle; bit-exact."""
import ctypes
import os
import random

import numpy as np
import pytest

from photonlibos_amd import checksum as ck
from photonlibos_amd.checked import MessageBatch
from photonlibos_amd.checksum import CrcError

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available()
    assert ck.device_count() >= 1
    return torch


@pytest.fixture(scope="module")
def data_file(tmp_path_factory):
    rng = np.random.default_rng(0xF11E)
    blob = rng.integers(0, 256, (96 << 20) + 12345, dtype=np.uint8).tobytes()
    p = tmp_path_factory.mktemp("src") / "records.bin"
    p.write_bytes(blob)
    return str(p), blob


@pytest.mark.parametrize("offset,stride,nbytes,count", [
    (0, 4096, 4096, 4096),            # 16 MiB of 4 KiB records
    (777, 65536 + 16, 65536, 1200),   # unaligned start, gaps between records, > one 64 MiB chunk
    (5, 1 << 20, (1 << 20) - 3, 90),  # 1 MiB-ish records across chunk boundaries
    (123, 100, 37, 1000),             # tiny records
])
def test_file_records(torch_dev, oracle, data_file, offset, stride, nbytes, count):
    path, blob = data_file
    fd = os.open(path, os.O_RDONLY)
    try:
        got = ck.file_strided(fd, offset, stride, nbytes, count, seed=0x1234)
    finally:
        os.close(fd)
    idx = list(range(0, count, max(1, count // 60))) + [count - 1]
    for i in idx:
        rec = blob[offset + i * stride: offset + i * stride + nbytes]
        assert got[i] == oracle.crc32c(rec, 0x1234), i


def test_file_o_direct(torch_dev, oracle, data_file):
    path, blob = data_file
    try:
        fd = os.open(path, os.O_RDONLY | os.O_DIRECT)
    except OSError:
        pytest.skip("filesystem does not support O_DIRECT")
    try:
        try:
            got = ck.file_strided(fd, 8192, 65536, 65536, 1000)
        except CrcError as e:
            if e.code == -22:  # EINVAL from the filesystem's O_DIRECT rules
                pytest.skip(f"O_DIRECT pread refused here: {e}")
            raise
    finally:
        os.close(fd)
    for i in (0, 1, 499, 999):
        assert got[i] == oracle.crc32c(blob[8192 + i * 65536: 8192 + (i + 1) * 65536])


def test_file_short_and_bad(torch_dev, data_file):
    path, blob = data_file
    fd = os.open(path, os.O_RDONLY)
    try:
        with pytest.raises(CrcError) as e:  # the last record runs past EOF
            ck.file_strided(fd, len(blob) - 10000, 4096, 4096, 3)
        assert e.value.code == -5
        assert ck.file_strided(fd, 0, 4096, 4096, 0) == []
    finally:
        os.close(fd)
    with pytest.raises(CrcError):
        ck.file_strided(-1, 0, 4096, 4096, 1)


def test_registered_host_memory_in_batch(torch_dev, oracle):
    # Pageable memory is refused by the batch (-EFAULT) until registered.
    buf = np.zeros((8 << 20) + 4096, np.uint8)
    base = (buf.ctypes.data + 4095) & ~4095
    view = np.ctypeslib.as_array((ctypes.c_uint8 * (8 << 20)).from_address(base))
    view[:] = np.random.default_rng(7).integers(0, 256, 8 << 20, dtype=np.uint8)
    segs = [(base + k * 65536 + 3, 65536 - 7) for k in range(0, 128, 2)]
    b = MessageBatch(8, 128)
    with pytest.raises(CrcError):
        b.add(segs[:8])
    ck.host_register(base, 8 << 20)
    try:
        for m in range(8):
            part = segs[m * 8:(m + 1) * 8]
            data = [bytes(view[a - base: a - base + n]) for a, n in part]
            b.add(part, None, oracle.extend_chain(data, 0))
        b.submit()
        assert b.wait() == 0
    finally:
        b.close()
        ck.host_unregister(base)


def test_registered_segment_past_registration_refused(torch_dev):
    """A segment starting inside a photon_crc_host_register range but running
    past its end is refused (-EFAULT) instead of read past the mapping."""
    buf = np.zeros((1 << 20) + 4096, np.uint8)
    base = (buf.ctypes.data + 4095) & ~4095
    ck.host_register(base, 1 << 20)
    try:
        b = MessageBatch(4, 4)
        b.add([(base + 100, (1 << 20) - 100)])  # exactly to the end: fine
        with pytest.raises(CrcError) as e:
            b.add([(base + 100, (1 << 20) - 99)])
        assert e.value.code == -14
        b.close()
    finally:
        ck.host_unregister(base)


def test_concurrent_file_callers(torch_dev, oracle, data_file):
    """Concurrent photon_crc32c_file_strided callers (different records of the
    same file, different fds) each get their own pinned chunk buffers and
    share the persistent reader pool: both results bit-exact."""
    import threading
    path, blob = data_file
    shapes = [(0, 4096, 4096, 8192), (4096 * 3 + 1, 65536, 65000, 700)]
    res = [None, None]
    errs = []

    def run(k):
        off, stride, n, cnt = shapes[k]
        fd = os.open(path, os.O_RDONLY)
        try:
            res[k] = ck.file_strided(fd, off, stride, n, cnt, seed=k)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
        finally:
            os.close(fd)
    for _ in range(3):
        th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
        for k, (off, stride, n, cnt) in enumerate(shapes):
            for i in list(range(0, cnt, max(1, cnt // 40))) + [cnt - 1]:
                assert res[k][i] == oracle.crc32c(blob[off + i * stride: off + i * stride + n], k), (k, i)
