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
// crcA * x^(16L) + crcB * x^(8L) + crcC. kA/kB are the hw_mul operands.
template <size_t L>
PCRC_HW inline uint32_t hw_3way(const uint8_t* p, uint32_t crc, uint32_t kA, uint32_t kB) {
    uint32_t a = crc, b = 0, c = 0;
    for (size_t i = 0; i < L; i += 8) {
        a = hw_word(a, load64(p + i));
        b = hw_word(b, load64(p + L + i));
        c = hw_word(c, load64(p + 2 * L + i));
    }
    return hw_mul(a, kA) ^ hw_mul(b, kB) ^ c;
}

struct HwConsts {
    uint32_t k4096a, k4096b, k512a, k512b, k64a, k64b;
};
HwConsts g_hw;

PCRC_HW uint32_t hw_engine(const uint8_t* p, size_t n, uint32_t crc) {
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
    while (n >= 3 * 64) {
        crc = hw_3way<64>(p, crc, g_hw.k64a, g_hw.k64b);
        p += 3 * 64;
        n -= 3 * 64;
    }
    for (; n >= 8; p += 8, n -= 8) crc = hw_word(crc, load64(p));
    for (; n; --n) crc = hw_byte(crc, *p++);
    return crc;
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
uint32_t crc32c_hw_portable(const uint8_t* p, size_t n, uint32_t crc) { return hw_engine(p, n, crc); }
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
    g_hw.k64a = xpow(8ull * 2 * 64 - 33);
    g_hw.k64b = xpow(8ull * 64 - 33);
    __builtin_cpu_init();
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
