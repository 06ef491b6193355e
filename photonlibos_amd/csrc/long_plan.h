// long_plan.h -- host side of the one-long-buffer kernels (crc32c_kernels.h
// "one long buffer", crc64_kernels.h crc64_long_kernel): how a buffer is cut
// into chunks and the launch constants of a cut. Shared by the product
// (crc32c_device.hip) and the bench-only probes (probes.hip), so a probe
// times exactly the product's plan.
#pragma once
#include <stdint.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "crc64_kernels.h"
#include "gf2.h"

namespace pcrc {

struct LongPlan {
    uint64_t head, chunk, nchunks, last, grid, stride;  // stride S: lane groups in the grid
    int lanes;
};

// force_chunk (bench-only probes): that chunk size instead of the computed one.
inline LongPlan long_plan_for(const void* data, uint64_t n, int cus, uint32_t shape, uint64_t force_chunk = 0,
                              bool crc64 = false) {
    const bool small = n <= (256u << 10);
    // automatic (r03 interleaved A/B, scripts/ab_long.py):
    //  CRC-32C: 64 lanes x 2 rounds; 32 x 2 from 512 MiB (1 GiB 32x2 0.177 ms
    //    vs 64x1 0.184 / 64x2 0.196; 256 MiB 64x2 0.060 vs 32x2 0.060 / 64x1
    //    0.065); 64 x 1 from 1.5 GiB (2 GiB 0.326 vs 32x2 0.367, 4 GiB 0.633
    //    vs 0.650; chunks near 128 KiB read slowly, profiles/r03e_ab_long_crc32c_big.jsonl)
    //  CRC-64: 64 lanes; 1 round from 1 GiB, else 2 (1 GiB 64x1 0.176 vs 32x2
    //    0.180 / 64x2 0.188; 2 GiB 0.331 / 0.372 / 0.336; 512 MiB 64x2 0.100
    //    vs 0.109 / 0.111; profiles/r03e_ab_long_crc64_*.jsonl)
    const bool huge = n >= (512ull << 20), giant = n >= (3ull << 29);
    const int lanes = small ? 64 : (shape & 0xff) ? (int)(shape & 0xff) : (huge && !giant && !crc64) ? 32 : 64;
    const uint64_t one = crc64 ? n >= (1ull << 30) : giant;
    const uint64_t rounds = small ? 1 : (shape >> 8) ? shape >> 8 : one ? 1 : 2;
    const uint64_t gpw = 64 / (uint64_t)lanes;
    const uint64_t slots = small ? 16 : 16ull * (uint64_t)cus * gpw * rounds;
    LongPlan p{};
    p.lanes = lanes;
    const uintptr_t d = reinterpret_cast<uintptr_t>(data);
    const uint64_t head = ((d + 4095) & ~uintptr_t(4095)) - d;
    if (head >= n || slots < 2) {  // one chunk: the whole buffer
        p.head = n;
        p.chunk = p.last = 4096;
        p.nchunks = 1;
    } else {
        // whole rows, and at least 1 KiB: 512-byte-aligned chunks (32 lanes)
        // read 13 % slower than 1 KiB-aligned ones (r03, scripts/ab_long.py)
        const uint64_t m = n - head, gran = 1024;
        uint64_t chunk = ((m + slots - 2) / (slots - 1) + gran - 1) / gran * gran;
        const uint64_t lo = small ? 4096 : 16384;
        if (chunk < lo) chunk = lo;
        if (force_chunk) chunk = force_chunk;
        while ((m + chunk - 1) / chunk + 1 > (1u << 18)) chunk <<= 1;  // the kernels' three 64-entry power tables
        p.head = head;
        p.chunk = chunk;
        p.nchunks = 1 + (m + chunk - 1) / chunk;
        p.last = m - (p.nchunks - 2) * chunk;
    }
    const uint64_t waves = (p.nchunks + gpw - 1) / gpw;
    p.grid = (waves + kWaves - 1) / kWaves;
    if (p.grid > (uint64_t)cus) p.grid = cus;
    if (p.grid > kLongMaxGrid) p.grid = kLongMaxGrid;  // long_reduce's slots
    p.stride = p.grid * kWaves * gpw;
    return p;
}

// Launch constants of a plan, CRC-32C or CRC-64/ECMA: X^j, X^(64 j),
// X^(4096 j) for j < 64 (X = x^(8 chunk)), X^S, and the last-chunk factors
// x^(+-8 (chunk - last)). Computed on first use per (chunk, last, S) and
// kept (callers repeat sizes and alignments).
struct LongPowers {
    uint64_t chunk, last, stride;
    uint32_t p32[3][64];
    uint64_t p64[3][64];
    uint32_t xpj32[64];  // J X^j: the kernels' xp (every group's final factor carries J)
    uint64_t xpj64[64];
    uint32_t xs32, j32, jinv32;
    uint64_t xs64, j64, jinv64;
    uint64_t xsb64[64];  // (1 << i) * X^S mod P64: crc64_long_kernel's lane basis words
};

inline const LongPowers& long_powers(const LongPlan& lp, bool crc64) {
    static std::mutex mu;
    static std::vector<LongPowers*> cache[2];
    thread_local LongPowers overflow;
    {
        std::lock_guard<std::mutex> lk(mu);
        for (auto* e : cache[crc64])
            if (e->chunk == lp.chunk && e->last == lp.last && e->stride == lp.stride) return *e;
    }
    LongPowers* t = new LongPowers();
    t->chunk = lp.chunk;
    t->last = lp.last;
    t->stride = lp.stride;
    const uint64_t s = lp.stride, pad = 8 * (lp.chunk - lp.last);
    for (int lvl = 0; lvl < 3; ++lvl) {
        const uint64_t bits = (8 * lp.chunk) << (6 * lvl);  // X^(64^lvl)
        if (crc64) {
            const uint64_t y = xpow64(bits);
            t->p64[lvl][0] = kOne64;
            for (int j = 1; j < 64; ++j) t->p64[lvl][j] = mulmod64(t->p64[lvl][j - 1], y);
        } else {
            const uint32_t x = xpow(bits);
            t->p32[lvl][0] = kOne;
            for (int j = 1; j < 64; ++j) t->p32[lvl][j] = mulmod(t->p32[lvl][j - 1], x);
        }
    }
    if (crc64) {
        t->xs64 = mulmod64(mulmod64(t->p64[0][s & 63], t->p64[1][(s >> 6) & 63]), t->p64[2][(s >> 12) & 63]);
        t->jinv64 = xpow64(pad);
        t->j64 = xpow64_inv(pad);
        for (int j = 0; j < 64; ++j) t->xpj64[j] = mulmod64(t->p64[0][j], t->j64);
        for (int i = 0; i < 64; ++i) t->xsb64[i] = mulmod64(1ull << i, t->xs64);
    } else {
        t->xs32 = mulmod(mulmod(t->p32[0][s & 63], t->p32[1][(s >> 6) & 63]), t->p32[2][(s >> 12) & 63]);
        t->jinv32 = xpow(pad);
        t->j32 = xpow_inv(pad);
        for (int j = 0; j < 64; ++j) t->xpj32[j] = mulmod(t->p32[0][j], t->j32);
    }
    std::lock_guard<std::mutex> lk(mu);
    for (auto* e : cache[crc64])
        if (e->chunk == lp.chunk && e->last == lp.last && e->stride == lp.stride) {
            delete t;
            return *e;
        }
    if (cache[crc64].size() >= 256) {  // many distinct shapes: compute per call
        overflow = *t;
        delete t;
        return overflow;
    }
    cache[crc64].push_back(t);
    return *t;
}

}  // namespace pcrc
