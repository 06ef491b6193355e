// gf2.h -- GF(2) arithmetic for raw CRC32C (reflected polynomial 0x82F63B78),
// shared by the host shim and the device kernels.
//
// Representation (reference common/checksum/crc_tables.cpp:63-76): a 32-bit
// reflected value whose bit j is the coefficient of x^(31-j); ONE = 0x80000000,
// X = 0x40000000. A CRC register value c with state-of-message M satisfies
// c = M(x) * x^32 mod P (common/checksum/crc.md:13-20).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define PCRC_HD __host__ __device__ constexpr inline
#else
#define PCRC_HD constexpr inline
#endif

namespace pcrc {

constexpr uint32_t kPoly = 0x82f63b78u;      // crc_tables.h:40
constexpr uint32_t kOne = 0x80000000u;       // x^0
constexpr uint32_t kX = 0x40000000u;         // x^1
constexpr uint32_t kXInv = 0x05ec76f1u;      // x^-1 mod P, crc_tables.cpp:42

// (a * b) mod P. Same recurrence as clmul_modp (crc_tables.cpp:48-58).
PCRC_HD uint32_t mulmod(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 0; i < 32; ++i, b >>= 1) {
        r = (r >> 1) ^ ((0u - (r & 1u)) & kPoly) ^ ((0u - (b & 1u)) & a);
    }
    return r;
}

// x^n mod P (square and multiply), crc_tables.cpp:63-76.
PCRC_HD uint32_t xpow(uint64_t n) {
    uint32_t result = kOne, base = kX;
    for (; n; n >>= 1) {
        if (n & 1) result = mulmod(result, base);
        base = mulmod(base, base);
    }
    return result;
}

// x^-n mod P, crc_tables.cpp:84-96.
PCRC_HD uint32_t xpow_inv(uint64_t n) {
    uint32_t result = kOne, base = kXInv;
    for (; n; n >>= 1) {
        if (n & 1) result = mulmod(result, base);
        base = mulmod(base, base);
    }
    return result;
}

// Shift a CRC by `nbytes` trailing zero bytes: crc * x^(8*nbytes) mod P.
PCRC_HD uint32_t shift_bytes(uint32_t crc, uint64_t nbytes) { return mulmod(crc, xpow(8 * nbytes)); }

// crc32c_combine semantics including the reference's shortcuts
// (crc.cpp:393-405, 424-430): crc1 == 0 -> crc2; len2 == 0 -> crc1.
PCRC_HD uint32_t combine(uint32_t crc1, uint32_t crc2, uint32_t len2) {
    if (!crc1) return crc2;
    if (!len2) return crc1;
    return shift_bytes(crc1, len2) ^ crc2;
}

// Multiplication by a fixed constant K is linear over GF(2): crc * K =
// XOR over set bits i of crc of (1<<i) * K. `basis` holds those 32 products.
PCRC_HD void mul_basis(uint32_t k, uint32_t basis[32]) {
    for (int i = 0; i < 32; ++i) basis[i] = mulmod(1u << i, k);
}

// ------------------------------------------------------------ CRC-64/ECMA
// Same reflected representation at 64 bits (crc_tables.cpp:48-96 with
// T = uint64_t): ONE = 1<<63, X = 1<<62, x^-1 = 0x92d8af2baf0e1e85.
constexpr uint64_t kPoly64 = 0xc96c5795d7870f42ull;
constexpr uint64_t kXInv64 = 0x92d8af2baf0e1e85ull;

PCRC_HD uint64_t mulmod64(uint64_t a, uint64_t b) {
    uint64_t r = 0;
    for (int i = 0; i < 64; ++i, b >>= 1) {
        r = (r >> 1) ^ ((0ull - (r & 1ull)) & kPoly64) ^ ((0ull - (b & 1ull)) & a);
    }
    return r;
}

PCRC_HD uint64_t xpow64(uint64_t n) {
    uint64_t result = 1ull << 63, base = 1ull << 62;
    for (; n; n >>= 1) {
        if (n & 1) result = mulmod64(result, base);
        base = mulmod64(base, base);
    }
    return result;
}

PCRC_HD uint64_t xpow64_inv(uint64_t n) {
    uint64_t result = 1ull << 63, base = kXInv64;
    for (; n; n >>= 1) {
        if (n & 1) result = mulmod64(result, base);
        base = mulmod64(base, base);
    }
    return result;
}

}  // namespace pcrc
