/*
 * crc_oracle.c -- TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
 *
 * A plain-C, deliberately simple restatement of PhotonLibOS's CRC arithmetic
 * in common/checksum, used as the CHECKER for the MI355X path. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - tests/golden/checksum_in.json: the 512 CRC32C and 512 CRC64ECMA known
 *     answers held by the reference's own test data
 *     (common/checksum/test/checksum.in, checksum.crc64; loader
 *     common/checksum/test/test_checksum.cpp:28-45).
 *   - tests/golden/ref_vectors.json: outputs of the reference's own crc.cpp /
 *     crc_tables.cpp, compiled unmodified from /root/reference by
 *     oracle/ref/Makefile and run on seeded inputs (script:
 *     tests/golden/gen_ref_vectors.py).
 *
 * Conventions (reference crc_tables.h:40-41, crc_tables.cpp:63-76):
 *   CRC32C: reflected polynomial 0x82F63B78, init = caller's crc, NO final xor.
 *   Reflected GF(2) representation: ONE = 0x80000000 (x^0), X = 0x40000000.
 *   CRC64ECMA: reflected polynomial 0xC96C5795D7870F42, pre- and post-inverted
 *   (crc.cpp:119-122).
 */
#include <errno.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define OR_CRC32C_POLY 0x82f63b78u
#define OR_CRC64_POLY 0xc96c5795d7870f42ull
#define OR_CRC32C_X_INV 0x05ec76f1u           /* crc_tables.cpp:42 */
#define OR_CRC64_X_INV 0x92d8af2baf0e1e85ull  /* crc_tables.cpp:43 */

/* ---------------------------------------------------------------- GF(2) */

/* (a*b) mod P, reflected; crc_tables.cpp:48-58 and crc.cpp:416-422. */
uint32_t or_clmul_modp32(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 0; i < 32; ++i, b >>= 1)
        r = (r >> 1) ^ ((r & 1) ? OR_CRC32C_POLY : 0) ^ ((b & 1) ? a : 0);
    return r;
}

/* x^n mod P by square-and-multiply; crc_tables.cpp:63-76. */
uint32_t or_pow32(uint64_t n) {
    uint32_t result = 0x80000000u, base = 0x40000000u;
    for (; n; n >>= 1) {
        if (n & 1) result = or_clmul_modp32(result, base);
        base = or_clmul_modp32(base, base);
    }
    return result;
}

/* x^-n mod P; crc_tables.cpp:84-96. */
uint32_t or_ipow32(uint64_t n) {
    uint32_t result = 0x80000000u, base = OR_CRC32C_X_INV;
    for (; n; n >>= 1) {
        if (n & 1) result = or_clmul_modp32(result, base);
        base = or_clmul_modp32(base, base);
    }
    return result;
}

/* Table generators; crc_tables.cpp:104-107. */
uint32_t or_crc32c_lshift_hw(unsigned i) { return or_pow32((128ull << i) - 33); }
uint32_t or_crc32c_rshift_hw(unsigned i) { return or_ipow32((1ull << (i + 3)) + 33); }
uint32_t or_crc32c_lshift_sw(unsigned i) { return or_pow32(1ull << (i + 3)); }
uint32_t or_crc32c_rshift_sw(unsigned i) { return or_ipow32(1ull << (i + 3)); }

/* ------------------------------------------------------------- CRC32C */

/* Bit-serial raw CRC32C: the definition the table engines implement
 * (table construction crc.cpp:83-88 applied one byte at a time). */
uint32_t or_crc32c_bitwise(const uint8_t *p, size_t n, uint32_t crc) {
    for (size_t i = 0; i < n; ++i) {
        crc ^= p[i];
        for (int k = 0; k < 8; ++k)
            crc = (crc >> 1) ^ ((crc & 1) ? OR_CRC32C_POLY : 0);
    }
    return crc;
}

/* Slicing-by-8 tables; TableCRC<uint32_t> at crc.cpp:77-97. */
static uint32_t or_tab32[8][256];
static int or_tab32_ready;

static void or_init_tab32(void) {
    if (or_tab32_ready) return;
    for (int n = 0; n < 256; ++n) {
        uint32_t c = (uint32_t)n;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1) ? OR_CRC32C_POLY : 0);
        or_tab32[0][n] = c;
    }
    for (int n = 0; n < 256; ++n) {
        uint32_t c = or_tab32[0][n];
        for (int k = 1; k < 8; ++k) {
            c = or_tab32[0][c & 0xff] ^ (c >> 8);
            or_tab32[k][n] = c;
        }
    }
    or_tab32_ready = 1;
}

const uint32_t *or_crc32c_table(int k) { or_init_tab32(); return or_tab32[k]; }

/* Slicing-by-8 software CRC32C: crc.cpp:28-54 (head/body/tail walk) with the
 * f1/f8 steps of crc.cpp:99-110. */
uint32_t or_crc32c_sw(const uint8_t *p, size_t n, uint32_t crc) {
    or_init_tab32();
    size_t off = 0;
    size_t mis = (size_t)((uintptr_t)p & 7);
    if (mis) {
        size_t lim = n < 8 - mis ? n : 8 - mis;
        for (; off < lim; ++off) crc = or_tab32[0][(crc ^ p[off]) & 0xff] ^ (crc >> 8);
    }
    for (; off + 8 <= n; off += 8) {
        uint64_t x;
        memcpy(&x, p + off, 8);
        x ^= crc;
        crc = 0;
        for (int i = 0; i < 8; ++i) crc ^= or_tab32[7 - i][(x >> (8 * i)) & 0xff];
    }
    for (; off < n; ++off) crc = or_tab32[0][(crc ^ p[off]) & 0xff] ^ (crc >> 8);
    return crc;
}

/* Batch drivers for the full-size parity tests (tests/test_gpu_fullsize.py):
 * plain loops over or_crc32c_sw, so a caller can fan a 4 GiB batch out over
 * threads (ctypes drops the GIL). Call or_crc32c_table() once first: the
 * lazy table build is not thread-safe. */
void or_crc32c_strided(const uint8_t *base, uint64_t stride, uint64_t nbytes, uint64_t count, uint32_t seed,
                       uint32_t *out) {
    for (uint64_t i = 0; i < count; ++i) out[i] = or_crc32c_sw(base + i * stride, nbytes, seed);
}

/* iov[2k] = host address, iov[2k+1] = length (struct iovec). */
void or_crc32c_iov(const uint64_t *iov, uint64_t count, uint32_t *out) {
    for (uint64_t i = 0; i < count; ++i)
        out[i] = or_crc32c_sw((const uint8_t *)(uintptr_t)iov[2 * i], (size_t)iov[2 * i + 1], 0);
}

/* Crc32Hasher::extend_hash over messages (rpc/serialize.h:244-247): message m
 * chains crc32c_extend over segments msg_start[m] .. msg_start[m+1]-1 from
 * seeds[m] (or seed0 when seeds is NULL). */
void or_crc32c_msg_chain(const uint64_t *iov, const uint64_t *msg_start, uint64_t nmsg, const uint32_t *seeds,
                         uint32_t seed0, uint32_t *out) {
    for (uint64_t m = 0; m < nmsg; ++m) {
        uint32_t c = seeds ? seeds[m] : seed0;
        for (uint64_t s = msg_start[m]; s < msg_start[m + 1]; ++s)
            c = or_crc32c_sw((const uint8_t *)(uintptr_t)iov[2 * s], (size_t)iov[2 * s + 1], c);
        out[m] = c;
    }
}

/* crc_apply_shifts with the software shift tables; crc.cpp:372-380. */
static uint32_t or_apply_lshift_sw(uint32_t crc, uint64_t len) {
    for (; len; len &= len - 1) crc = or_clmul_modp32(crc, or_crc32c_lshift_sw((unsigned)__builtin_ctzll(len)));
    return crc;
}
static uint32_t or_apply_rshift_sw(uint32_t crc, uint64_t len) {
    for (; len; len &= len - 1) crc = or_clmul_modp32(crc, or_crc32c_rshift_sw((unsigned)__builtin_ctzll(len)));
    return crc;
}

/* crc32c_combine_sw; crc.cpp:424-430 (shortcuts at 425-426). */
uint32_t or_crc32c_combine(uint32_t crc1, uint32_t crc2, uint32_t len2) {
    if (!crc1) return crc2;
    if (!len2) return crc1;
    return or_apply_lshift_sw(crc1, len2) ^ crc2;
}

/* crc32c_combine_series_sw; crc.cpp:466-472. */
uint32_t or_crc32c_combine_series(const uint32_t *crc, uint32_t part_size, uint32_t n_parts) {
    if (!n_parts) return 0;
    uint32_t r = crc[0];
    for (uint32_t i = 1; i < n_parts; ++i) r = or_crc32c_combine(r, crc[i], part_size);
    return r;
}

/* crc32c_series_sw; crc.cpp:474-477 (offsets taken in 64 bits here; the
 * reference's 32-bit `i * part_size` wraps past 4 GiB). */
void or_crc32c_series(const uint8_t *buf, uint32_t part_size, uint32_t n_parts, uint32_t *out) {
    for (uint32_t i = 0; i < n_parts; ++i)
        out[i] = or_crc32c_sw(buf + (size_t)i * part_size, part_size, 0);
}

/* crc32c_series_hw's observable quirk (crc.cpp:479-509): parts shorter than
 * 8 bytes are never processed (`if (unlikely(part_main))` at 496), so every
 * part CRC is 0. Longer parts are the plain CRC. */
void or_crc32c_series_hw(const uint8_t *buf, uint32_t part_size, uint32_t n_parts, uint32_t *out) {
    if (part_size < 8) {
        for (uint32_t i = 0; i < n_parts; ++i) out[i] = 0;
        return;
    }
    or_crc32c_series(buf, part_size, n_parts, out);
}

/* do_crc_trim with the software shifts; crc.cpp:442-460. Error path sets
 * errno = EINVAL and returns 0 (crc.cpp:444-445). */
uint32_t or_crc32c_trim(uint32_t all_crc, uint32_t all_size, uint32_t pre_crc, uint32_t pre_size,
                        uint32_t suf_crc, uint32_t suf_size) {
    if (all_size < (uint32_t)(pre_size + suf_size)) {  /* 32-bit sum, as crc.cpp:444 */
        errno = EINVAL;
        return 0;
    }
    if (!pre_size && !suf_size) return all_crc;
    uint32_t crc = all_crc;
    if (pre_size) crc = or_crc32c_combine(pre_crc, crc, all_size - pre_size);
    if (suf_size) crc = or_apply_rshift_sw(crc ^ suf_crc, suf_size);
    return crc;
}

/* ---------------------------------------------------------- CRC64ECMA */

static uint64_t or_tab64[8][256];
static int or_tab64_ready;

static void or_init_tab64(void) {
    if (or_tab64_ready) return;
    for (int n = 0; n < 256; ++n) {
        uint64_t c = (uint64_t)n;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1) ? OR_CRC64_POLY : 0);
        or_tab64[0][n] = c;
    }
    for (int n = 0; n < 256; ++n) {
        uint64_t c = or_tab64[0][n];
        for (int k = 1; k < 8; ++k) {
            c = or_tab64[0][c & 0xff] ^ (c >> 8);
            or_tab64[k][n] = c;
        }
    }
    or_tab64_ready = 1;
}

/* crc64ecma_sw; crc.cpp:119-122 (inverted in and out). */
uint64_t or_crc64ecma_sw(const uint8_t *p, size_t n, uint64_t crc) {
    or_init_tab64();
    uint64_t c = ~crc;
    for (size_t i = 0; i < n; ++i) c = or_tab64[0][(c ^ p[i]) & 0xff] ^ (c >> 8);
    return ~c;
}

/* Batch driver (as or_crc32c_strided; call or_crc64ecma_sw once first). */
void or_crc64ecma_strided(const uint8_t *base, uint64_t stride, uint64_t nbytes, uint64_t count, uint64_t seed,
                          uint64_t *out) {
    for (uint64_t i = 0; i < count; ++i) out[i] = or_crc64ecma_sw(base + i * stride, nbytes, seed);
}

/* (a*b) mod P for the 64-bit table generator; crc_tables.cpp:48-58. */
uint64_t or_clmul_modp64(uint64_t a, uint64_t b) {
    uint64_t r = 0;
    for (int i = 0; i < 64; ++i, b >>= 1)
        r = (r >> 1) ^ ((r & 1) ? OR_CRC64_POLY : 0) ^ ((b & 1) ? a : 0);
    return r;
}

/* x^n mod P (64-bit); crc_tables.cpp:63-76. */
uint64_t or_pow64(uint64_t n) {
    uint64_t result = 1ull << 63, base = 1ull << 62;
    for (; n; n >>= 1) {
        if (n & 1) result = or_clmul_modp64(result, base);
        base = or_clmul_modp64(base, base);
    }
    return result;
}
