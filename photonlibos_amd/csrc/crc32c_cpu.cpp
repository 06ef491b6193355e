// crc32c_cpu.cpp -- host-side drop-in for PhotonLibOS common/checksum
// (CRC32C part): the synchronous per-buffer entry points and dispatch pointers
// declared in include/photon/common/checksum/crc32c.h, with the reference's
// names, C++ linkage, argument meaning, shortcuts and error behaviour.
//
// These are the host engines that Photon callers with small host-memory
// buffers keep using (RPC messages of a few KiB: a GPU launch costs more
// than the CRC). Throughput work goes through the batched device engine
// (crc32c_device.hip, <photon_crc/crc32c_gpu.h>).
//
// Engines:
//   crc32c_sw  -- slicing-by-8 tables (behaviour of crc.cpp:77-117)
//   crc32c_hw  -- SSE4.2 crc32q, three interleaved streams merged with
//                 PCLMULQDQ (behaviour of crc.cpp:303-368)
//   combine / combine_series / trim / series -- crc.cpp:370-509
// The GF(2) constants are generated at load time from gf2.h.
#include <photon/common/checksum/crc32c.h>

#include <errno.h>
#include <immintrin.h>
#include <stdio.h>
#include <string.h>

#include "gf2.h"

namespace {

using pcrc::mulmod;
using pcrc::xpow;
using pcrc::xpow_inv;

struct Tables {
    uint32_t slice[8][256];  // slice[k][b]: byte b followed by k zero bytes
    uint32_t lsh_sw[32];     // x^(8*2^i)
    uint32_t rsh_sw[32];     // x^-(8*2^i)
    uint32_t lsh_hw[32];     // x^(8*2^i - 33): operand of hw_mul (PCLMUL + crc32q = *x^33)
    uint32_t rsh_hw[32];     // x^-(8*2^i + 33)
};

Tables g_tab;

void build_tables() {
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t c = b;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((0u - (c & 1u)) & pcrc::kPoly);
        g_tab.slice[0][b] = c;
    }
    for (int k = 1; k < 8; ++k)
        for (uint32_t b = 0; b < 256; ++b) {
            const uint32_t prev = g_tab.slice[k - 1][b];
            g_tab.slice[k][b] = g_tab.slice[0][prev & 0xff] ^ (prev >> 8);
        }
    for (int i = 0; i < 32; ++i) {
        const uint64_t bits = 8ull << i;
        g_tab.lsh_sw[i] = xpow(bits);
        g_tab.rsh_sw[i] = xpow_inv(bits);
        g_tab.lsh_hw[i] = bits >= 33 ? xpow(bits - 33) : xpow_inv(33 - bits);
        g_tab.rsh_hw[i] = xpow_inv(bits + 33);
    }
}

inline uint32_t sw_byte(uint32_t crc, uint8_t b) { return g_tab.slice[0][(crc ^ b) & 0xff] ^ (crc >> 8); }

inline uint32_t sw_word(uint32_t crc, uint64_t w) {
    const uint64_t x = w ^ crc;
    return g_tab.slice[7][x & 0xff] ^ g_tab.slice[6][(x >> 8) & 0xff] ^ g_tab.slice[5][(x >> 16) & 0xff] ^
           g_tab.slice[4][(x >> 24) & 0xff] ^ g_tab.slice[3][(x >> 32) & 0xff] ^
           g_tab.slice[2][(x >> 40) & 0xff] ^ g_tab.slice[1][(x >> 48) & 0xff] ^ g_tab.slice[0][x >> 56];
}

inline uint64_t load64(const uint8_t* p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}

// ---------------------------------------------------------------- SSE4.2 path
#define PCRC_HW __attribute__((target("sse4.2,pclmul")))

PCRC_HW inline uint32_t hw_byte(uint32_t c, uint8_t b) { return _mm_crc32_u8(c, b); }
PCRC_HW inline uint32_t hw_word(uint32_t c, uint64_t w) { return (uint32_t)_mm_crc32_u64(c, w); }

// a * k * x^33 mod P: the 63-bit carry-less product read as a 64-bit message
// by crc32q is x * (a * k), and the CRC of a message multiplies it by x^32.
PCRC_HW inline uint32_t hw_mul(uint32_t a, uint32_t k) {
    const __m128i p = _mm_clmulepi64_si128(_mm_cvtsi32_si128((int)a), _mm_cvtsi32_si128((int)k), 0x00);
    return (uint32_t)_mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(p));
}

// Three independent crc32q chains over [0,L), [L,2L), [2L,3L), merged as
// crcA * x^(16L) + crcB * x^(8L) + crcC. kA/kB are the hw_mul operands. The
// two carry-less products are XORed into chain C's LAST word instead of being
// reduced on their own (crc32q(c, w ^ t) = crc32q(c, w) ^ crc32q(0, t), and
// crc32q(0, clmul(a, k)) = a * k * x^33): the merge then costs one PCLMUL on
// the critical path, not PCLMUL + crc32q.
template <size_t L>
PCRC_HW inline uint32_t hw_3way(const uint8_t* p, uint32_t crc, uint32_t kA, uint32_t kB) {
    uint32_t a = crc, b = 0, c = 0;
    for (size_t i = 0; i < L - 8; i += 8) {
        a = hw_word(a, load64(p + i));
        b = hw_word(b, load64(p + L + i));
        c = hw_word(c, load64(p + 2 * L + i));
    }
    a = hw_word(a, load64(p + L - 8));
    b = hw_word(b, load64(p + 2 * L - 8));
    const __m128i t = _mm_xor_si128(_mm_clmulepi64_si128(_mm_cvtsi32_si128((int)a), _mm_cvtsi32_si128((int)kA), 0x00),
                                    _mm_clmulepi64_si128(_mm_cvtsi32_si128((int)b), _mm_cvtsi32_si128((int)kB), 0x00));
    return hw_word(c, load64(p + 3 * L - 8) ^ (uint64_t)_mm_cvtsi128_si64(t));
}

struct HwConsts {
    uint32_t k4096a, k4096b, k512a, k512b, k256a, k256b, k128a, k128b, k64a, k64b;
};
HwConsts g_hw;

// SSE4.2 + PCLMUL engine (any x86-64 with those): 3-way crc32q blocks of 12
// KiB while they last, then 1.5 KiB, then one block each of 768, 384 and 192
// bytes -- a 4 KiB buffer takes 4 merges, not 7.
PCRC_HW uint32_t hw_portable_engine(const uint8_t* p, size_t n, uint32_t crc) {
    if (!n) return crc;
    // Align to 8 bytes so the word loop walks aligned words.
    while (n && ((uintptr_t)p & 7)) {
        crc = hw_byte(crc, *p++);
        --n;
    }
    while (n >= 3 * 4096) {
        crc = hw_3way<4096>(p, crc, g_hw.k4096a, g_hw.k4096b);
        p += 3 * 4096;
        n -= 3 * 4096;
    }
    while (n >= 3 * 512) {
        crc = hw_3way<512>(p, crc, g_hw.k512a, g_hw.k512b);
        p += 3 * 512;
        n -= 3 * 512;
    }
    if (n >= 3 * 256) {
        crc = hw_3way<256>(p, crc, g_hw.k256a, g_hw.k256b);
        p += 3 * 256;
        n -= 3 * 256;
    }
    if (n >= 3 * 128) {
        crc = hw_3way<128>(p, crc, g_hw.k128a, g_hw.k128b);
        p += 3 * 128;
        n -= 3 * 128;
    }
    if (n >= 3 * 64) {
        crc = hw_3way<64>(p, crc, g_hw.k64a, g_hw.k64b);
        p += 3 * 64;
        n -= 3 * 64;
    }
    for (; n >= 8; p += 8, n -= 8) crc = hw_word(crc, load64(p));
    for (; n; --n) crc = hw_byte(crc, *p++);
    return crc;
}

// ------------------------------------------------------ AVX-512 VPCLMULQDQ path
// For CPUs with 512-bit carry-less multiply (Zen 4/5 EPYC such as the GPU
// boxes' 9575F, Ice Lake and later Xeons). Folding instead of crc32q chains:
// the buffer is read 64 bytes per register, four registers (256 B) per step,
// and each 128-bit lane S (first 8 bytes H = the higher powers, last 8 bytes L)
// is moved D bytes forward as
//     S * x^(8D) = H * x^(8D+64) + L * x^(8D)   (mod P)
// with two PCLMULs against x^(8D+63) and x^(8D-1) (a carry-less product of
// reflected operands reads as the product times x) and XORed into the data D
// bytes later. What is left at the end is one 128-bit value V whose CRC is
// V(x) * x^32 mod P = two crc32q of its halves; the seed is XORed into the
// first four data bytes (init-value linearity, as the GPU kernels do).
// Same results as every other engine; no table, no reference code.
#define PCRC_V512 __attribute__((target("avx512f,avx512bw,avx512vl,avx512dq,vpclmulqdq,pclmul,sse4.2")))

struct alignas(64) V512Consts {
    uint64_t k256[8];  // every 128-bit lane: {x^(8*256+63), x^(8*256-1)} as 64-bit reflected words
    uint64_t k192[8];
    uint64_t k128[8];
    uint64_t k64[8];
    uint64_t kred[8];  // lanes 0, 1, 2: moves of 48, 32, 16 bytes; lane 3: 0
    uint64_t k16[2];
};
V512Consts g_v;
bool g_has_v512 = false;
constexpr size_t kV512Min = 256;  // shorter buffers take the crc32q engine

void fold_consts(uint64_t* k, uint64_t bytes) {
    // a 32-bit reflected value v (bit i = x^(31-i)) as a 64-bit reflected word: v << 32
    k[0] = (uint64_t)xpow(8 * bytes + 63) << 32;
    k[1] = (uint64_t)xpow(8 * bytes - 1) << 32;
}

void build_v512_consts() {
    for (int l = 0; l < 4; ++l) {
        fold_consts(g_v.k256 + 2 * l, 256);
        fold_consts(g_v.k192 + 2 * l, 192);
        fold_consts(g_v.k128 + 2 * l, 128);
        fold_consts(g_v.k64 + 2 * l, 64);
    }
    fold_consts(g_v.kred + 0, 48);
    fold_consts(g_v.kred + 2, 32);
    fold_consts(g_v.kred + 4, 16);
    g_v.kred[6] = g_v.kred[7] = 0;
    fold_consts(g_v.k16, 16);
}

PCRC_V512 inline __m512i fold512(__m512i a, __m512i k, __m512i d) {
    return _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(a, k, 0x00), _mm512_clmulepi64_epi128(a, k, 0x11), d,
                                     0x96);
}

PCRC_V512 inline __m128i fold128(__m128i a, __m128i k, __m128i d) {
    return _mm_ternarylogic_epi64(_mm_clmulepi64_si128(a, k, 0x00), _mm_clmulepi64_si128(a, k, 0x11), d, 0x96);
}

PCRC_V512 uint32_t v512_engine(const uint8_t* p, size_t n, uint32_t crc) {
    // n >= kV512Min
    const __m512i k256 = _mm512_load_si512(g_v.k256);
    __m512i a0 = _mm512_xor_si512(_mm512_loadu_si512(p), _mm512_zextsi128_si512(_mm_cvtsi32_si128((int)crc)));
    __m512i a1 = _mm512_loadu_si512(p + 64);
    __m512i a2 = _mm512_loadu_si512(p + 128);
    __m512i a3 = _mm512_loadu_si512(p + 192);
    p += 256;
    n -= 256;
    for (; n >= 256; p += 256, n -= 256) {
        a0 = fold512(a0, k256, _mm512_loadu_si512(p));
        a1 = fold512(a1, k256, _mm512_loadu_si512(p + 64));
        a2 = fold512(a2, k256, _mm512_loadu_si512(p + 128));
        a3 = fold512(a3, k256, _mm512_loadu_si512(p + 192));
    }
    // The four registers onto the last one's position, then whole 64-byte blocks.
    const __m512i k64 = _mm512_load_si512(g_v.k64);
    __m512i r = fold512(a0, _mm512_load_si512(g_v.k192), a3);
    r = fold512(a1, _mm512_load_si512(g_v.k128), r);
    r = fold512(a2, k64, r);
    for (; n >= 64; p += 64, n -= 64) r = fold512(r, k64, _mm512_loadu_si512(p));
    // Four lanes onto the last one.
    const __m512i kr = _mm512_load_si512(g_v.kred);
    const __m512i t = _mm512_xor_si512(_mm512_clmulepi64_epi128(r, kr, 0x00), _mm512_clmulepi64_epi128(r, kr, 0x11));
    __m128i x = _mm_ternarylogic_epi64(_mm512_castsi512_si128(t), _mm512_extracti64x2_epi64(t, 1),
                                       _mm512_extracti64x2_epi64(t, 2), 0x96);
    x = _mm_xor_si128(x, _mm512_extracti64x2_epi64(r, 3));
    const __m128i k16 = _mm_load_si128(reinterpret_cast<const __m128i*>(g_v.k16));
    for (; n >= 16; p += 16, n -= 16) x = fold128(x, k16, _mm_loadu_si128(reinterpret_cast<const __m128i*>(p)));
    uint32_t c = (uint32_t)_mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(x));
    c = (uint32_t)_mm_crc32_u64(c, (uint64_t)_mm_extract_epi64(x, 1));
    if (n >= 8) {
        c = (uint32_t)_mm_crc32_u64(c, load64(p));
        p += 8;
        n -= 8;
    }
    for (; n; --n) c = _mm_crc32_u8(c, *p++);
    return c;
}

bool cpu_has_v512() {
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
           __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512dq") &&
           __builtin_cpu_supports("vpclmulqdq") && __builtin_cpu_supports("pclmul") &&
           __builtin_cpu_supports("sse4.2");
}

// crc32c_hw: the fastest engine this CPU has.
uint32_t hw_engine(const uint8_t* p, size_t n, uint32_t crc) {
    if (g_has_v512 && n >= kV512Min) return v512_engine(p, n, crc);
    return hw_portable_engine(p, n, crc);
}

PCRC_HW uint32_t hw_simple_engine(const uint8_t* p, size_t n, uint32_t crc) {
    while (n && ((uintptr_t)p & 7)) {
        crc = hw_byte(crc, *p++);
        --n;
    }
    for (; n >= 8; p += 8, n -= 8) crc = hw_word(crc, load64(p));
    for (; n; --n) crc = hw_byte(crc, *p++);
    return crc;
}

// crc * x^(8*len) (left) or crc * x^-(8*len) (right), one multiply per set bit
// of len (crc_apply_shifts, crc.cpp:372-380).
inline uint32_t sw_shift(uint32_t crc, uint32_t len, const uint32_t* tab) {
    for (; len; len &= len - 1) crc = mulmod(crc, tab[__builtin_ctz(len)]);
    return crc;
}
PCRC_HW inline uint32_t hw_shift(uint32_t crc, uint32_t len, const uint32_t* tab) {
    for (; len; len &= len - 1) crc = hw_mul(crc, tab[__builtin_ctz(len)]);
    return crc;
}

bool cpu_has_hw() { return __builtin_cpu_supports("sse4.2") && __builtin_cpu_supports("pclmul"); }

template <typename Combine, typename RShift>
uint32_t trim_impl(CRC32C_Component all, CRC32C_Component prefix, CRC32C_Component suffix, Combine comb,
                   RShift rsh) {
    // Same 32-bit comparison as the reference (crc.cpp:444).
    if (all.size < (uint32_t)(prefix.size + suffix.size)) {
        fprintf(stderr, "crc32c_trim: total size (%u) must be > summed sizes of prefix (%u) + suffix (%u)\n",
                all.size, prefix.size, suffix.size);
        errno = EINVAL;
        return 0;
    }
    if (!prefix.size && !suffix.size) return all.crc;
    uint32_t crc = all.crc;
    if (prefix.size) crc = comb(prefix.crc, crc, all.size - prefix.size);
    if (suffix.size) crc = rsh(crc ^ suffix.crc, suffix.size);
    return crc;
}

}  // namespace

// The host engine's generated constants, for the pinning test (tuning.h
// photon_crc_test_tables): 0 lsh_sw, 1 rsh_sw, 2 lsh_hw, 3 rsh_hw (32 each),
// 8 the slicing table slice[0] (256).
namespace pcrc {
int host_engine_table(int which, uint32_t* out, int n) {
    const uint32_t* src = which == 0 ? g_tab.lsh_sw : which == 1 ? g_tab.rsh_sw : which == 2 ? g_tab.lsh_hw
                        : which == 3 ? g_tab.rsh_hw : which == 8 ? g_tab.slice[0] : nullptr;
    const int len = which == 8 ? 256 : 32;
    if (!src || n < len) return -22;
    for (int i = 0; i < len; ++i) out[i] = src[i];
    return len;
}
}  // namespace pcrc

// ------------------------------------------------------------- exported API

uint32_t crc32c_sw(const uint8_t* p, size_t n, uint32_t crc) {
    while (n && ((uintptr_t)p & 7)) {
        crc = sw_byte(crc, *p++);
        --n;
    }
    for (; n >= 8; p += 8, n -= 8) crc = sw_word(crc, load64(p));
    for (; n; --n) crc = sw_byte(crc, *p++);
    return crc;
}

uint32_t crc32c_hw(const uint8_t* p, size_t n, uint32_t crc) { return hw_engine(p, n, crc); }
uint32_t crc32c_hw_portable(const uint8_t* p, size_t n, uint32_t crc) { return hw_portable_engine(p, n, crc); }
uint32_t crc32c_hw_simple(const uint8_t* p, size_t n, uint32_t crc) { return hw_simple_engine(p, n, crc); }

void crc32c_series_sw(const uint8_t* buffer, uint32_t part_size, uint32_t n_parts, uint32_t* crc_parts) {
    // The reference forms the part offset as uint32 * uint32 (crc.cpp:476);
    // kept so results stay identical for every input.
    for (uint32_t i = 0; i < n_parts; ++i) crc_parts[i] = crc32c_sw(buffer + (uint32_t)(i * part_size), part_size, 0);
}

void crc32c_series_hw(const uint8_t* buffer, uint32_t part_size, uint32_t n_parts, uint32_t* crc_parts) {
    // Parts shorter than 8 bytes come out as 0 in the reference
    // (crc.cpp:481-500: the tail is only folded `if (part_main)`).
    if (part_size < 8) {
        for (uint32_t i = 0; i < n_parts; ++i) crc_parts[i] = 0;
        return;
    }
    for (uint32_t i = 0; i < n_parts; ++i)
        crc_parts[i] = hw_engine(buffer + (size_t)i * part_size, part_size, 0);
}

uint32_t crc32c_combine_sw(uint32_t crc1, uint32_t crc2, uint32_t len2) {
    if (!crc1) return crc2;
    if (!len2) return crc1;
    return sw_shift(crc1, len2, g_tab.lsh_sw) ^ crc2;
}

uint32_t crc32c_combine_hw(uint32_t crc1, uint32_t crc2, uint32_t len2) {
    if (!crc1) return crc2;
    if (!len2) return crc1;
    return hw_shift(crc1, len2, g_tab.lsh_hw) ^ crc2;
}

uint32_t crc32c_combine_series_sw(uint32_t* crc, uint32_t part_size, uint32_t n_parts) {
    if (!n_parts) return 0;
    uint32_t r = crc[0];
    for (uint32_t i = 1; i < n_parts; ++i) r = crc32c_combine_sw(r, crc[i], part_size);
    return r;
}

uint32_t crc32c_combine_series_hw(uint32_t* crc, uint32_t part_size, uint32_t n_parts) {
    if (!n_parts) return 0;
    uint32_t r = crc[0];
    for (uint32_t i = 1; i < n_parts; ++i) r = crc32c_combine_hw(r, crc[i], part_size);
    return r;
}

uint32_t crc32c_trim_sw(CRC32C_Component all, CRC32C_Component prefix, CRC32C_Component suffix) {
    return trim_impl(all, prefix, suffix, crc32c_combine_sw,
                     [](uint32_t c, uint32_t len) { return sw_shift(c, len, g_tab.rsh_sw); });
}

uint32_t crc32c_trim_hw(CRC32C_Component all, CRC32C_Component prefix, CRC32C_Component suffix) {
    return trim_impl(all, prefix, suffix, crc32c_combine_hw,
                     [](uint32_t c, uint32_t len) { return hw_shift(c, len, g_tab.rsh_hw); });
}

uint32_t (*crc32c_auto)(const uint8_t*, size_t, uint32_t) = nullptr;
void (*crc32c_series_auto)(const uint8_t*, uint32_t, uint32_t, uint32_t*) = nullptr;
uint32_t (*crc32c_combine_auto)(uint32_t, uint32_t, uint32_t) = nullptr;
uint32_t (*crc32c_combine_series_auto)(uint32_t*, uint32_t, uint32_t) = nullptr;
uint32_t (*crc32c_trim_auto)(CRC32C_Component, CRC32C_Component, CRC32C_Component) = nullptr;

__attribute__((constructor(101))) static void photon_crc_cpu_init() {
    build_tables();
    g_hw.k4096a = xpow(8ull * 2 * 4096 - 33);
    g_hw.k4096b = xpow(8ull * 4096 - 33);
    g_hw.k512a = xpow(8ull * 2 * 512 - 33);
    g_hw.k512b = xpow(8ull * 512 - 33);
    g_hw.k256a = xpow(8ull * 2 * 256 - 33);
    g_hw.k256b = xpow(8ull * 256 - 33);
    g_hw.k128a = xpow(8ull * 2 * 128 - 33);
    g_hw.k128b = xpow(8ull * 128 - 33);
    g_hw.k64a = xpow(8ull * 2 * 64 - 33);
    g_hw.k64b = xpow(8ull * 64 - 33);
    build_v512_consts();
    __builtin_cpu_init();
    g_has_v512 = cpu_has_hw() && cpu_has_v512() && !getenv("PHOTON_CRC_NO_AVX512");
    if (cpu_has_hw()) {
        crc32c_auto = crc32c_hw;
        crc32c_series_auto = crc32c_series_hw;
        crc32c_combine_auto = crc32c_combine_hw;
        crc32c_combine_series_auto = crc32c_combine_series_hw;
        crc32c_trim_auto = crc32c_trim_hw;
    } else {
        crc32c_auto = crc32c_sw;
        crc32c_series_auto = crc32c_series_sw;
        crc32c_combine_auto = crc32c_combine_sw;
        crc32c_combine_series_auto = crc32c_combine_series_sw;
        crc32c_trim_auto = crc32c_trim_sw;
    }
}
