// crc64_cpu.cpp -- host-side drop-in for PhotonLibOS's CRC-64/ECMA-182
// (include/photon/common/checksum/crc64ecma.h; reference crc64ecma.h:20-87,
// crc.cpp:119-122, 511-669): same names, C++ linkage, inversion convention,
// combine/trim semantics (incl. the reference's 32-bit length arguments).
// crc64ecma_sw is slicing-by-8 tables, crc64ecma_hw PCLMUL folding (tables
// without PCLMUL); results identical to the reference's crc64ecma_sw and
// SSE/PCLMUL paths (its AVX-512 path disagrees with them for long inputs,
// SURVEY.md §0.4, and is not reproduced).
#include <photon/common/checksum/crc64ecma.h>

#include <errno.h>
#include <immintrin.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gf2.h"

namespace {

struct Tables64 {
    uint64_t slice[8][256];
    uint64_t lsh[32];  // x^(8*2^i)
    uint64_t rsh[32];  // x^-(8*2^i)
};
Tables64 g_t64;

void build64() {
    for (uint32_t b = 0; b < 256; ++b) {
        uint64_t c = b;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((0ull - (c & 1ull)) & pcrc::kPoly64);
        g_t64.slice[0][b] = c;
    }
    for (int k = 1; k < 8; ++k)
        for (uint32_t b = 0; b < 256; ++b) {
            const uint64_t prev = g_t64.slice[k - 1][b];
            g_t64.slice[k][b] = g_t64.slice[0][prev & 0xff] ^ (prev >> 8);
        }
    for (int i = 0; i < 32; ++i) {
        g_t64.lsh[i] = pcrc::xpow64(8ull << i);
        g_t64.rsh[i] = pcrc::xpow64_inv(8ull << i);
    }
}

// Raw reflected CRC-64 register update (no inversion).
uint64_t engine64(const uint8_t* p, size_t n, uint64_t c) {
    while (n && ((uintptr_t)p & 7)) {
        c = g_t64.slice[0][(c ^ *p++) & 0xff] ^ (c >> 8);
        --n;
    }
    for (; n >= 8; p += 8, n -= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        const uint64_t x = w ^ c;
        c = g_t64.slice[7][x & 0xff] ^ g_t64.slice[6][(x >> 8) & 0xff] ^ g_t64.slice[5][(x >> 16) & 0xff] ^
            g_t64.slice[4][(x >> 24) & 0xff] ^ g_t64.slice[3][(x >> 32) & 0xff] ^
            g_t64.slice[2][(x >> 40) & 0xff] ^ g_t64.slice[1][(x >> 48) & 0xff] ^ g_t64.slice[0][x >> 56];
    }
    for (; n; --n) c = g_t64.slice[0][(c ^ *p++) & 0xff] ^ (c >> 8);
    return c;
}

// crc * x^(+-8*len), one multiply per set bit of len (crc_apply_shifts,
// crc.cpp:372-380; len is uint32_t there).
uint64_t shift64(uint64_t crc, uint32_t len, const uint64_t* tab) {
    for (; len; len &= len - 1) crc = pcrc::mulmod64(crc, tab[__builtin_ctz(len)]);
    return crc;
}

uint64_t combine64(uint64_t crc1, uint64_t crc2, uint32_t len2) {
    // crc.cpp:627-631 / 641-645: only the crc1 == 0 shortcut (no len2 == 0 one).
    if (!crc1) return crc2;
    return crc2 ^ shift64(crc1, len2, g_t64.lsh);
}

uint64_t trim64(CRC64ECMA_Component all, CRC64ECMA_Component prefix, CRC64ECMA_Component suffix) {
    // do_crc_trim (crc.cpp:442-456) with T = CRC64ECMA_Component.
    if (all.size < prefix.size + suffix.size) {
        fprintf(stderr, "crc64ecma_trim: total size (%llu) must be > summed sizes of prefix (%llu) + suffix (%llu)\n",
                (unsigned long long)all.size, (unsigned long long)prefix.size, (unsigned long long)suffix.size);
        errno = EINVAL;
        return 0;
    }
    if (!prefix.size && !suffix.size) return all.crc;
    uint64_t crc = all.crc;
    if (prefix.size) crc = combine64(prefix.crc, crc, (uint32_t)(all.size - prefix.size));
    if (suffix.size) crc = shift64(crc ^ suffix.crc, (uint32_t)suffix.size, g_t64.rsh);
    return crc;
}

// ---------------------------------------------------------- PCLMUL folding
// The hw engine (the reference's crc64ecma_hw is PCLMUL-based too,
// crc.cpp:511-669): fold 16-byte states with carry-less multiplies, finish
// the last state with the table engine.
//
// A 16-byte little-endian block is the reflected 128-bit polynomial
// S = S_hi * x^64 + S_lo with S_hi in the low qword. Moving S forward by d
// bits: S * x^d = S_hi * x^(64+d) + S_lo * x^d, and a carry-less product of
// two reflected 64-bit values is x * (their product) in reflected 128-bit
// form, so the constants are x^(63+d) and x^(d-1) mod P (both reflected, as
// xpow64 returns them). The message so far is congruent to the state modulo
// P, so the register is (S * x^64 mod P) = the table engine run over the 16
// bytes of S from register 0.
struct Fold64 {
    uint64_t k1_lo, k1_hi;  // d = 128: x^191, x^127
    uint64_t k4_lo, k4_hi;  // d = 512: x^575, x^511
};
Fold64 g_fold;
bool g_have_pclmul = false;

__attribute__((target("pclmul,sse4.1"))) inline __m128i fold16(__m128i s, __m128i k) {
    return _mm_xor_si128(_mm_clmulepi64_si128(s, k, 0x00), _mm_clmulepi64_si128(s, k, 0x11));
}

__attribute__((target("pclmul,sse4.1"))) uint64_t engine64_clmul(const uint8_t* p, size_t n, uint64_t c) {
    if (n < 128) return engine64(p, n, c);
    const __m128i k1 = _mm_set_epi64x((long long)g_fold.k1_hi, (long long)g_fold.k1_lo);
    const __m128i k4 = _mm_set_epi64x((long long)g_fold.k4_hi, (long long)g_fold.k4_lo);
    auto ld = [](const uint8_t* q) { return _mm_loadu_si128(reinterpret_cast<const __m128i*>(q)); };
    // Four interleaved states (blocks i, i+4, ...), the register folded into
    // the first 8 message bytes (init linearity).
    __m128i s0 = _mm_xor_si128(ld(p), _mm_cvtsi64_si128((long long)c));
    __m128i s1 = ld(p + 16), s2 = ld(p + 32), s3 = ld(p + 48);
    p += 64;
    n -= 64;
    for (; n >= 64; p += 64, n -= 64) {
        s0 = _mm_xor_si128(fold16(s0, k4), ld(p));
        s1 = _mm_xor_si128(fold16(s1, k4), ld(p + 16));
        s2 = _mm_xor_si128(fold16(s2, k4), ld(p + 32));
        s3 = _mm_xor_si128(fold16(s3, k4), ld(p + 48));
    }
    __m128i s = _mm_xor_si128(fold16(s0, k1), s1);
    s = _mm_xor_si128(fold16(s, k1), s2);
    s = _mm_xor_si128(fold16(s, k1), s3);
    for (; n >= 16; p += 16, n -= 16) s = _mm_xor_si128(fold16(s, k1), ld(p));
    uint8_t tail[16];
    _mm_storeu_si128(reinterpret_cast<__m128i*>(tail), s);
    return engine64(p, n, engine64(tail, 16, 0));
}

void build_fold() {
    g_fold.k1_lo = pcrc::xpow64(191);
    g_fold.k1_hi = pcrc::xpow64(127);
    g_fold.k4_lo = pcrc::xpow64(575);
    g_fold.k4_hi = pcrc::xpow64(511);
    g_have_pclmul = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
}

// AVX-512 VPCLMULQDQ (Zen 4/5 EPYC, Ice Lake and later Xeons): the same
// folding, four 512-bit registers = 16 states, 256 bytes per step
// (crc32c_cpu.cpp has the CRC-32C twin). Constants per move of D bytes:
// {x^(8D+63), x^(8D-1)} mod P in every 128-bit lane.
#define PCRC64_V512 __attribute__((target("avx512f,avx512bw,avx512vl,avx512dq,vpclmulqdq,pclmul,sse4.1")))

struct alignas(64) V512Fold64 {
    uint64_t k256[8], k192[8], k128[8], k64[8], kred[8];
};
V512Fold64 g_v64;
bool g_have_v512 = false;

void fold_pair(uint64_t* k, uint64_t bytes) {
    k[0] = pcrc::xpow64(8 * bytes + 63);
    k[1] = pcrc::xpow64(8 * bytes - 1);
}

void build_v512() {
    for (int l = 0; l < 4; ++l) {
        fold_pair(g_v64.k256 + 2 * l, 256);
        fold_pair(g_v64.k192 + 2 * l, 192);
        fold_pair(g_v64.k128 + 2 * l, 128);
        fold_pair(g_v64.k64 + 2 * l, 64);
    }
    fold_pair(g_v64.kred + 0, 48);
    fold_pair(g_v64.kred + 2, 32);
    fold_pair(g_v64.kred + 4, 16);
    g_v64.kred[6] = g_v64.kred[7] = 0;
    g_have_v512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                  __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512dq") &&
                  __builtin_cpu_supports("vpclmulqdq") && __builtin_cpu_supports("pclmul") &&
                  __builtin_cpu_supports("sse4.1") && !getenv("PHOTON_CRC_NO_AVX512");
}

PCRC64_V512 inline __m512i fold512_64(__m512i a, __m512i k, __m512i d) {
    return _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(a, k, 0x00), _mm512_clmulepi64_epi128(a, k, 0x11), d,
                                     0x96);
}

PCRC64_V512 uint64_t engine64_v512(const uint8_t* p, size_t n, uint64_t c) {
    // n >= 256
    const __m512i k256 = _mm512_load_si512(g_v64.k256);
    __m512i a0 = _mm512_xor_si512(_mm512_loadu_si512(p), _mm512_zextsi128_si512(_mm_cvtsi64_si128((long long)c)));
    __m512i a1 = _mm512_loadu_si512(p + 64);
    __m512i a2 = _mm512_loadu_si512(p + 128);
    __m512i a3 = _mm512_loadu_si512(p + 192);
    p += 256;
    n -= 256;
    for (; n >= 256; p += 256, n -= 256) {
        a0 = fold512_64(a0, k256, _mm512_loadu_si512(p));
        a1 = fold512_64(a1, k256, _mm512_loadu_si512(p + 64));
        a2 = fold512_64(a2, k256, _mm512_loadu_si512(p + 128));
        a3 = fold512_64(a3, k256, _mm512_loadu_si512(p + 192));
    }
    const __m512i k64 = _mm512_load_si512(g_v64.k64);
    __m512i r = fold512_64(a0, _mm512_load_si512(g_v64.k192), a3);
    r = fold512_64(a1, _mm512_load_si512(g_v64.k128), r);
    r = fold512_64(a2, k64, r);
    for (; n >= 64; p += 64, n -= 64) r = fold512_64(r, k64, _mm512_loadu_si512(p));
    const __m512i kr = _mm512_load_si512(g_v64.kred);
    const __m512i t = _mm512_xor_si512(_mm512_clmulepi64_epi128(r, kr, 0x00), _mm512_clmulepi64_epi128(r, kr, 0x11));
    __m128i x = _mm_ternarylogic_epi64(_mm512_castsi512_si128(t), _mm512_extracti64x2_epi64(t, 1),
                                       _mm512_extracti64x2_epi64(t, 2), 0x96);
    x = _mm_xor_si128(x, _mm512_extracti64x2_epi64(r, 3));
    const __m128i k16 = _mm_set_epi64x((long long)g_fold.k1_hi, (long long)g_fold.k1_lo);
    for (; n >= 16; p += 16, n -= 16)
        x = _mm_ternarylogic_epi64(_mm_clmulepi64_si128(x, k16, 0x00), _mm_clmulepi64_si128(x, k16, 0x11),
                                   _mm_loadu_si128(reinterpret_cast<const __m128i*>(p)), 0x96);
    uint8_t tail[16];
    _mm_storeu_si128(reinterpret_cast<__m128i*>(tail), x);
    return engine64(p, n, engine64(tail, 16, 0));
}

uint64_t engine64_hw(const uint8_t* p, size_t n, uint64_t c) {
    if (g_have_v512 && n >= 256) return engine64_v512(p, n, c);
    return g_have_pclmul ? engine64_clmul(p, n, c) : engine64(p, n, c);
}

}  // namespace

uint64_t crc64ecma_sw(const uint8_t* buffer, size_t nbytes, uint64_t crc) { return ~engine64(buffer, nbytes, ~crc); }
uint64_t crc64ecma_hw(const uint8_t* buffer, size_t nbytes, uint64_t crc) { return ~engine64_hw(buffer, nbytes, ~crc); }

void crc64ecma_series_sw(const uint8_t* buffer, uint32_t part_size, uint32_t n_parts, uint64_t* crc_parts) {
    for (uint32_t i = 0; i < n_parts; ++i) crc_parts[i] = crc64ecma_sw(buffer + (size_t)i * part_size, part_size, 0);
}
void crc64ecma_series_hw(const uint8_t* buffer, uint32_t part_size, uint32_t n_parts, uint64_t* crc_parts) {
    for (uint32_t i = 0; i < n_parts; ++i) crc_parts[i] = crc64ecma_hw(buffer + (size_t)i * part_size, part_size, 0);
}

uint64_t crc64ecma_combine_sw(uint64_t crc1, uint64_t crc2, uint32_t len2) { return combine64(crc1, crc2, len2); }
uint64_t crc64ecma_combine_hw(uint64_t crc1, uint64_t crc2, uint32_t len2) { return combine64(crc1, crc2, len2); }

uint64_t crc64ecma_combine_series_sw(uint64_t* crc, uint32_t part_size, uint32_t n_parts) {
    if (!n_parts) return 0;
    uint64_t r = crc[0];
    for (uint32_t i = 1; i < n_parts; ++i) r = combine64(r, crc[i], part_size);
    return r;
}
uint64_t crc64ecma_combine_series_hw(uint64_t* crc, uint32_t part_size, uint32_t n_parts) {
    return crc64ecma_combine_series_sw(crc, part_size, n_parts);
}

uint64_t crc64ecma_trim_sw(CRC64ECMA_Component a, CRC64ECMA_Component p, CRC64ECMA_Component s) { return trim64(a, p, s); }
uint64_t crc64ecma_trim_hw(CRC64ECMA_Component a, CRC64ECMA_Component p, CRC64ECMA_Component s) { return trim64(a, p, s); }

uint64_t (*crc64ecma_auto)(const uint8_t*, size_t, uint64_t) = nullptr;
void (*crc64ecma_series_auto)(const uint8_t*, uint32_t, uint32_t, uint64_t*) = nullptr;
uint64_t (*crc64ecma_combine_auto)(uint64_t, uint64_t, uint32_t) = nullptr;
uint64_t (*crc64ecma_combine_series_auto)(uint64_t*, uint32_t, uint32_t) = nullptr;
uint64_t (*crc64ecma_trim_auto)(CRC64ECMA_Component, CRC64ECMA_Component, CRC64ECMA_Component) = nullptr;

__attribute__((constructor(101))) static void photon_crc64_cpu_init() {
    build64();
    build_fold();
    build_v512();
    crc64ecma_auto = crc64ecma_hw;
    crc64ecma_series_auto = crc64ecma_series_hw;
    crc64ecma_combine_auto = crc64ecma_combine_hw;
    crc64ecma_combine_series_auto = crc64ecma_combine_series_hw;
    crc64ecma_trim_auto = crc64ecma_trim_hw;
}
