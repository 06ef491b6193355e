"""Batched CheckedMessage<Crc32Hasher> checksums over pinned RPC payloads
(include/photon_crc/checked_batch.h).

Mirrors the reference's receive path: `validate_checksum(iov, body, len)`
(rpc/serialize.h:266-275) saves m_checksum, zeroes it and re-hashes the
payload iovector followed by the message struct. Here many messages are added
to a `MessageBatch` and checked in one GPU submit; the payload memory comes
from the pinned IOAlloc pool (`PinnedAlloc`, common/io-alloc.h:31-85)."""
import ctypes

import numpy as np

from ._native import PhotonRange, lib
from .checksum import CrcError, _check


class PinnedAlloc:
    """IOAlloc over photon_crc_pinned_allocate / _deallocate."""

    def alloc(self, size):
        """IOAlloc::alloc(size) (io-alloc.h:41-49): address of `size` pinned bytes."""
        ptr = ctypes.c_void_p()
        rc = lib().photon_crc_pinned_allocate(None, PhotonRange(size, size), ctypes.byref(ptr))
        if rc <= 0:
            raise CrcError(rc, lib().photon_crc_last_error().decode(errors="replace"))
        return ptr.value

    def dealloc(self, addr):
        _check(lib().photon_crc_pinned_deallocate(None, addr))

    @staticmethod
    def view(addr, size):
        """numpy uint8 view of pinned memory (host side)."""
        return np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(addr))

    @staticmethod
    def stats():
        slab, used = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().photon_crc_pinned_stats(ctypes.byref(slab), ctypes.byref(used)))
        return slab.value, used.value

    @staticmethod
    def release():
        return lib().photon_crc_pinned_release()


TRUSTED = 1
STAGED = 2  # descriptors H2D / verdicts D2H instead of zero-copy staging
DETACHED_BODY = 4  # bodies are separate buffers: payload then body (not the message object)


class MessageBatch:
    """photon_crc_msg_batch: add messages, submit once, read verdicts."""

    def __init__(self, max_messages, max_segments, flags=0):
        self._b = lib().photon_crc_msg_batch_create(max_messages, max_segments, flags)
        if not self._b:
            raise CrcError(-1, lib().photon_crc_last_error().decode(errors="replace"))
        self._iov_cache = None

    def close(self):
        if self._b:
            lib().photon_crc_msg_batch_destroy(self._b)
            self._b = None

    def __del__(self):
        self.close()

    def add(self, segments, body=None, expected=0):
        """segments: [(addr, len)], body: (addr, len) or None. Returns the index."""
        n = len(segments)
        iov = (ctypes.c_uint64 * (2 * max(n, 1)))()
        for k, (a, ln) in enumerate(segments):
            iov[2 * k], iov[2 * k + 1] = a, ln
        baddr, blen = body if body is not None else (None, 0)
        rc = lib().photon_crc_msg_batch_add(self._b, iov, n, baddr, blen, expected & 0xFFFFFFFF)
        if rc < 0:
            raise CrcError(rc, lib().photon_crc_last_error().decode(errors="replace"))
        return rc

    _DONE = ctypes.CFUNCTYPE(None, ctypes.c_void_p)

    def submit(self, stream=None, done=None):
        """One GPU submit of every message added. `done` (optional, no
        arguments) runs on a HIP runtime thread once the verdicts are on the
        host; it must not call HIP, submit, reset or close this batch."""
        cb = self._DONE(lambda _arg: done()) if done is not None else None
        # `cb` (a local) keeps the new trampoline alive through the call. It
        # replaces the one held for the previous submit only once this submit
        # succeeded: the C side refuses (-EBUSY) while the previous callback
        # is queued or running, so after a refusal HIP may still call the old
        # trampoline, and after a success it never will again.
        _check(lib().photon_crc_msg_batch_submit(self._b, stream, ctypes.cast(cb, ctypes.c_void_p) if cb else None,
                                                 None))
        self._cb = cb

    def wait(self):
        rc = lib().photon_crc_msg_batch_wait(self._b)
        if rc < 0:
            raise CrcError(rc, lib().photon_crc_last_error().decode(errors="replace"))
        return rc

    def result(self, i):
        """(valid, crc) of message i."""
        c = ctypes.c_uint32()
        rc = lib().photon_crc_msg_batch_result(self._b, i, ctypes.byref(c))
        if rc < 0:
            raise CrcError(rc, lib().photon_crc_last_error().decode(errors="replace"))
        return bool(rc), c.value

    def __len__(self):
        return lib().photon_crc_msg_batch_count(self._b)

    def reset(self):
        _check(lib().photon_crc_msg_batch_reset(self._b))
