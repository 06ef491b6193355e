// crc64_cpu.cpp -- host-side drop-in for PhotonLibOS's CRC-64/ECMA-182
// (include/photon/common/checksum/crc64ecma.h; reference crc64ecma.h:20-87,
// crc.cpp:119-122, 511-669): same names, C++ linkage, inversion convention,
// combine/trim semantics (incl. the reference's 32-bit length arguments).
// Both engines are slicing-by-8 tables here (results identical to the
// reference's crc64ecma_sw and SSE/PCLMUL paths; its AVX-512 path disagrees
// with them for long inputs, SURVEY.md §0.4, and is not reproduced).
#include <photon/common/checksum/crc64ecma.h>

#include <errno.h>
#include <stdio.h>
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

}  // namespace

uint64_t crc64ecma_sw(const uint8_t* buffer, size_t nbytes, uint64_t crc) { return ~engine64(buffer, nbytes, ~crc); }
uint64_t crc64ecma_hw(const uint8_t* buffer, size_t nbytes, uint64_t crc) { return ~engine64(buffer, nbytes, ~crc); }

void crc64ecma_series_sw(const uint8_t* buffer, uint32_t part_size, uint32_t n_parts, uint64_t* crc_parts) {
    for (uint32_t i = 0; i < n_parts; ++i) crc_parts[i] = crc64ecma_sw(buffer + (size_t)i * part_size, part_size, 0);
}
void crc64ecma_series_hw(const uint8_t* buffer, uint32_t part_size, uint32_t n_parts, uint64_t* crc_parts) {
    crc64ecma_series_sw(buffer, part_size, n_parts, crc_parts);
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
    crc64ecma_auto = crc64ecma_hw;
    crc64ecma_series_auto = crc64ecma_series_hw;
    crc64ecma_combine_auto = crc64ecma_combine_hw;
    crc64ecma_combine_series_auto = crc64ecma_combine_series_hw;
    crc64ecma_trim_auto = crc64ecma_trim_hw;
}
