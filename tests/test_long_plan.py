"""The long-buffer cut and its staged combine, replayed on the CPU (no GPU).

photon_crc_test_long_plan returns the plan and launch constants the library
computes for a buffer (photonlibos_amd/csrc/long_plan.h). These tests replay
what crc32c_long_kernel / crc64_long_kernel do with them -- every slot's CRC
(the head with the seed, empty leading slots, body chunks, the short last
one), the Horner fold per lane group with X^S, the wave stage (X for 32-lane
groups, Z^(15-w)), the workgroup stage (J Y^(grid-1-b), then the last chunk
with factor 1) and the XOR over workgroups -- with the pinned oracle's CRCs
and a GF(2) multiply written here, and compare with the oracle's CRC of the
whole buffer (crc.cpp:393-405 is the identity behind every stage). Small
"devices" (1-3 CUs) keep the slot counts replayable; the algebra does not
depend on the CU count. Also: at the reference's perf shape (1 GiB at buf+1,
test_checksum.cpp:125-168) on 256 CUs every lane group reads the same bytes.
"""
import ctypes

import numpy as np
import pytest

from photonlibos_amd._native import lib

P32, P64 = 0x82F63B78, 0xC96C5795D7870F42


def _mulmod(a, b, width):
    poly = P32 if width == 32 else P64
    r = 0
    for _ in range(width):
        r = (r >> 1) ^ (poly if r & 1 else 0) ^ (a if b & 1 else 0)
        b >>= 1
    return r


def _mul_basis(v, basis):
    r = 0
    i = 0
    while v:
        if v & 1:
            r ^= basis[i]
        v >>= 1
        i += 1
    return r


def _plan(addr, n, cus, lanes=0, rounds=0, crc64=False):
    out = (ctypes.c_uint64 * (9 + 64 + 1 + 16 + 256 + 64))()
    k = lib().photon_crc_test_long_plan(addr, n, cus, lanes, rounds, int(crc64), out, len(out))
    assert k > 0, lib().photon_crc_last_error()
    w = [int(x) for x in out[:k]]
    p = dict(zip(("head", "chunk", "T", "L", "R", "grid", "S", "D", "lanes"), w[:9]))
    rest = w[9:]
    if crc64:
        p["xsb"], p["x"], p["zt"], p["ft"] = rest[:64], rest[64], rest[65:81], rest[81:81 + p["grid"]]
    else:
        p["xsb"], p["xb"], p["zt"], p["ft"] = rest[:32], rest[32:64], rest[64:80], rest[80:80 + p["grid"]]
    return p


def _replay(p, data, seed, oracle, crc64=False, merge_head=True):
    """The kernels' combine over `data` (bytes at the plan's address).
    merge_head (the product, PCRC_LONG_MERGE_HEAD): with a body, the head is
    read as the front of body chunk 0's slot; else it has slot D - 1 (round
    -1 of group S - 1 when D = 0). Both give the CRC."""
    width = 64 if crc64 else 32
    head, chunk, T, L, R, grid, S, D = (p[k] for k in ("head", "chunk", "T", "L", "R", "grid", "S", "D"))
    gpw = 64 // p["lanes"]
    assert R * S - T == D and 0 <= D and S == grid * 16 * gpw and grid <= 256
    assert T == 0 or (T - 1) * chunk + L == len(data) - head
    merged = merge_head and T > 0

    def raw(seg, s):
        if crc64:  # the raw register: starts at ~seed (0 for a body chunk: ~all-ones), not inverted at the end
            return oracle.crc64ecma(seg, s if s is not None else 0xFFFFFFFFFFFFFFFF) ^ 0xFFFFFFFFFFFFFFFF
        return oracle.crc32c(seg, s or 0)

    def slot_crc(v):
        t = v - D
        if merged:
            if t < 0:
                return 0
            if t == 0:  # the head, with the seed, then body chunk 0
                return raw(data[:head + (L if T == 1 else chunk)], seed)
        elif t == -1:  # the head, with the seed (CRC-64: the register starts at ~seed)
            return raw(data[:head], seed)
        elif t < 0:
            return 0
        seg = data[head + t * chunk: head + t * chunk + (L if t == T - 1 else chunk)]
        return raw(seg, None)

    accs, lasts = [], []
    for g in range(S):
        acc = lastc = 0
        for r in range(-1 if (D == 0 and not merged) else 0, R):
            v = g + r * S
            c = slot_crc(v)
            m = _mul_basis(acc, p["xsb"])
            last = v - D == T - 1
            acc = m if last else m ^ c
            lastc = c if last else lastc
        accs.append(acc)
        lasts.append(lastc)
    xb = p["xb"] if not crc64 else [_mulmod(1 << i, p["x"], 64) for i in range(64)]
    total = 0
    for b in range(grid):
        u = e = 0
        for w in range(16):
            g = (16 * b + w) * gpw
            if gpw == 2:
                v = _mul_basis(accs[g], xb) ^ accs[g + 1]
                e ^= lasts[g] ^ lasts[g + 1]
            else:
                v = accs[g]
                e ^= lasts[g]
            u ^= _mulmod(v, p["zt"][w], width)
        total ^= _mulmod(u, p["ft"][b], width) ^ e
    return total ^ 0xFFFFFFFFFFFFFFFF if crc64 else total


SHAPES = [(0, 0), (64, 1), (64, 2), (32, 1), (32, 2), (32, 3)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("cus", [1, 3])
def test_long_plan_replays_to_the_crc(oracle, shape, cus):
    lanes, rounds = shape
    rng = np.random.default_rng(0x5EED0E00 + cus + lanes + rounds)
    buf = rng.integers(0, 256, 4 << 20, dtype=np.uint8).tobytes()
    # sizes over the 256 KiB small-kernel limit, heads 0 / 1 / 4095 / odd,
    # chunk counts that fill the slots exactly (D = 0) and that leave some empty
    cases = [(4096 * 7 + 1, (1 << 20)), (4096 * 7, (1 << 20) + 5), (4096 * 7 + 4095, (300 << 10) + 3),
             (4096 * 7 + 17, 3 << 20), (4096 * 7 + 2048, (2 << 20) - 4096 + 1)]
    for k, (addr_off, n) in enumerate(cases):
        seed = (0x9E3779B1 * (k + 1)) & 0xFFFFFFFF
        p = _plan(addr_off, n, cus, lanes, rounds)
        data = buf[addr_off:addr_off + n]
        assert p["head"] == (-addr_off) % 4096
        for merge in (True, False):
            assert _replay(p, data, seed, oracle, merge_head=merge) == oracle.crc32c(data, seed), \
                (shape, cus, addr_off, n, p["D"], merge)


@pytest.mark.parametrize("shape", [(0, 0), (64, 2), (32, 2)])
def test_long_plan_replays_crc64(oracle, shape):
    lanes, rounds = shape
    rng = np.random.default_rng(0x5EED0E10 + lanes)
    buf = rng.integers(0, 256, 2 << 20, dtype=np.uint8).tobytes()
    # CRC-64 has no small kernel: the plan also covers buffers of a few bytes
    # (the head is all of it, no body chunk) and up to 256 KiB (4 KiB chunks)
    cases = [(4096 * 3 + 1, 1 << 20), (4096 * 3 + 4000, 50), (4096 * 3, 70000), (4096 * 3 + 9, 256 << 10)]
    for k, (addr_off, n) in enumerate(cases):
        seed = (0x9E3779B97F4A7C15 * (k + 1)) & 0xFFFFFFFFFFFFFFFF
        p = _plan(addr_off, n, 2, lanes, rounds, crc64=True)
        data = buf[addr_off:addr_off + n]
        for merge in (True, False):
            assert _replay(p, data, seed, oracle, crc64=True, merge_head=merge) == oracle.crc64ecma(data, seed), \
                (shape, addr_off, n, merge)


def test_reference_perf_shape_is_balanced():
    """1 GiB at buf+1 on 256 CUs (the automatic 32 lanes x 2 rounds): no empty
    slot and head + short last chunk = one chunk, so every lane group reads 2 x
    64 KiB but the two holding chunk 0 (head in front: + 4095 B) and the last
    chunk (- 4095 B); round 4 gave group S - 1 the head as an extra round -1
    (round 3's cut: 130 KiB for most groups, 65 KiB for 250 of them); CRC-64
    takes the same shape."""
    p = _plan(4096 * 100 + 1, 1 << 30, 256)
    assert (p["lanes"], p["R"], p["grid"]) == (32, 2, 256)
    assert p["chunk"] == 64 << 10 and p["D"] == 0 and p["T"] == p["R"] * p["S"]
    assert p["head"] + p["L"] == p["chunk"]  # group S-1: head + (R-1) chunks + the short one = R chunks
    p64 = _plan(4096 * 100 + 1, 1 << 30, 256, crc64=True)
    assert (p64["lanes"], p64["R"]) == (32, 2) and p64["head"] + p64["L"] == p64["chunk"] and p64["D"] == 0


def _mulx(v, width):
    return (v >> 1) ^ ((P32 if width == 32 else P64) if v & 1 else 0)


def _basis_word_lds(c, i, width):
    """basis_word_lds / basis_word64_lds (crc32c_kernels.h, crc64_kernels.h)
    restated over the LDS D tables' contents: slice t, byte v -> (v << 8t) *
    x^width (the D table: one data word absorbed), so slice (nslices - 1) is
    the classic byte table v * x^8."""
    ns = width // 8

    def slice_entry(t, v):
        return _mulmod(v << (8 * t), _xpow(width, width), width)

    k = width - 1 - i
    b, a = k & 7, k >> 3
    y = (c << (8 - b)) & 0xFF
    v = (c >> b) ^ slice_entry(ns - 1, y)
    r = v >> (8 * a)
    for j in range(ns - 1):
        byte = (v >> (8 * j)) & 0xFF if j < a else 0
        r ^= slice_entry((ns + j - a) % ns, byte)
    return r


def _xpow(e, width):
    """x^e mod P in the reflected representation (bit width-1 = x^0)."""
    r = 1 << (width - 1)
    for _ in range(e):
        r = _mulx(r, width)
    return r


@pytest.mark.parametrize("width", [32, 64])
def test_basis_words_from_the_byte_tables(width):
    """The long kernels' basis words (1 << i) * c = c * x^(width-1-i), taken
    from the byte tables in LDS, equal the bit-serial definition for every i."""
    rng = np.random.default_rng(0x5EED0E20 + width)
    for _ in range(8):
        c = int(rng.integers(0, 1 << 62)) | (int(rng.integers(0, 4)) << 62) if width == 64 else int(rng.integers(0, 1 << 32))
        for i in range(width):
            want = c
            for _ in range(width - 1 - i):
                want = _mulx(want, width)
            assert _basis_word_lds(c, i, width) == want, (width, hex(c), i)
            assert want == _mulmod(1 << i, c, width)
