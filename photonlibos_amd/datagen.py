"""Deterministic synthetic payloads (uniform random bytes; never zeros: a raw
CRC of zeros is 0 and hides bugs).

Stream `seed`: 64-bit word k = mix64(seed + (k+1) * 0x9E3779B97F4A7C15)
(splitmix64), stored little-endian. Identical to the device generator
photon_crc_util_fill_splitmix and to oracle/ref/ref_harness.cpp's fill().
"""
import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix64(z):
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def stream_bytes(seed, nbytes):
    """nbytes of splitmix64 stream `seed` as a numpy uint8 array."""
    nw = (nbytes + 7) // 8
    k = np.arange(1, nw + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + k * GOLDEN
    return _mix64(z).astype("<u8").view(np.uint8)[:nbytes].copy()


def buffers(seed_base, count, nbytes):
    """count x nbytes array; row i is stream seed_base + i."""
    out = np.empty((count, nbytes), dtype=np.uint8)
    for i in range(count):
        out[i] = stream_bytes(seed_base + i, nbytes)
    return out
