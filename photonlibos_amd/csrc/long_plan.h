// long_plan.h -- host side of the one-long-buffer kernels (crc32c_kernels.h
// "one long buffer", crc64_kernels.h crc64_long_kernel): how a buffer is cut
// into chunks, which lane group takes which chunk, and the launch constants
// of a cut. Shared by the product (crc32c_device.hip) and the bench-only
// probes (probes.hip), so a probe times exactly the product's plan.
//
// The cut (round 4). A = the first 4 KiB boundary at or after the data start;
// the HEAD [data, A) (0..4095 bytes) carries the seed; the BODY [A, end) is
// cut into T chunks of `chunk` bytes (a 1 KiB multiple, >= 16 KiB; >= 8 KiB
// under 128 MiB), the last
// one of L bytes (0 < L <= chunk). The grid has S lane groups and R rounds:
// R*S virtual slots v = 0 .. R*S-1, slot v belongs to group v % S in round
// v / S, and body chunk t sits in slot v = t + D with D = R*S - T: the
// EMPTY slots are at the front (leading zeros do not change a CRC), so the
// last chunk is always slot R*S-1 (group S-1, last round) and every group's
// factor to the end of the buffer is X^(S-1-g) (X = x^(8 chunk)) whatever T
// is. The head is slot D-1 -- an empty slot of group D-1 when D >= 1, or a
// slot "-1" before group S-1's first round when D = 0 (then that group's
// last chunk is the short one: at the reference's 1 GiB at buf+1, head +
// last = one chunk exactly, so every group reads the same bytes). Round 3's
// cut gave the head a slot of its own: T - 1 slots for the body, chunks
// rounded up to 1 KiB, so at 1 GiB / buf+1 every group read 130 KiB instead
// of 128 and 250 groups had half as much.
#pragma once
#include <stdint.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "crc64_kernels.h"
#include "gf2.h"

// A/B switches of the cut under 128 MiB (the round-4 cut: 16384 and 0).
#ifndef PCRC_LONG_MID_FLOOR
#define PCRC_LONG_MID_FLOOR 8192
#endif
#ifndef PCRC_LONG_R1_MIB
#define PCRC_LONG_R1_MIB 64
#endif

namespace pcrc {

struct LongPlan {
    uint64_t head;    // bytes before A (the head task; 0..4095)
    uint64_t chunk;   // body chunk bytes
    uint64_t nchunks; // T body chunks
    uint64_t last;    // L: bytes of the last body chunk
    uint64_t rounds;  // R
    uint64_t grid;    // workgroups
    uint64_t stride;  // S: lane groups in the grid
    uint64_t lead;    // D = R*S - T: leading empty slots
    int lanes;
};

// force_chunk (bench-only probes): that chunk size instead of the computed one.
// Long buffers only: the small kernel takes block spans up to 256 KiB.
inline LongPlan long_plan_for(const void* data, uint64_t n, int cus, uint32_t shape, uint64_t force_chunk = 0,
                              bool crc64 = false) {
    // automatic shape (r04 interleaved A/B over this cut, one process per
    // size, scripts/ab_long.py; repo:profiles/r04b_ab_long_shapes_1g.jsonl,
    // r04c_ab_long_shapes_sizes.jsonl; medians in ms, batch kernel over 64
    // KiB pieces of the same bytes in brackets):
    //  CRC-32C: 256 MiB 64x2 0.0541 (0.0545); 512 MiB 64x1 0.0919, 32x2
    //    0.0937 (0.0889); 1 GiB 32x2 0.1679, 64x2 0.169, 64x1 0.179 (0.1647);
    //    2 GiB 64x4 0.3242, 32x2 0.3425 (0.3186); 4 GiB 64x2 0.6328 (0.6236)
    //  CRC-64: 256 MiB 64x1 0.0575 (0.058); 2 GiB 64x4 0.3273 (0.322);
    //    4 GiB 64x2 0.6341 (0.6304); with the LDS basis words
    //    (repo:profiles/r04g_ab_long_basis_barrier.jsonl): 512 MiB 64x2
    //    0.0957, 32x2 0.0979, 64x1 0.1011 (0.0893); 1 GiB 32x2 0.1709, 64x2
    //    0.1771, 64x1 0.1882 (0.1668)
    //  up to 256 KiB (CRC-64 only: CRC-32C has its small kernel): 1 round of
    //  chunks of >= 4 KiB, one workgroup
    //  under 128 MiB (round 5, repo:profiles/r05p_ab_long_chunk_floor.jsonl;
    //    the mid layout takes spans up to 16 MiB): 16 KiB
    //    chunks fill only 64-128 of 256 CUs; 8 KiB: 64 MiB 64x2 0.0215 vs
    //    0.0232, 32 MiB 64x1 0.0160 vs 64x2/16 KiB 0.0225; 128 MiB 16 KiB stays
    //    best (0.0325 vs 0.0334). The rule, A/B against the 16 KiB cut
    //    (repo:profiles/r05p_ab_floor8_vs_16.jsonl, ms medians): CRC-32C 33 MiB
    //    0.0166 vs 0.0231, 48 MiB 0.0188 vs 0.0234, 64 MiB 0.0218 vs 0.0240,
    //    127 MiB 0.0325 vs 0.0328; CRC-64 17 MiB 0.0159 vs 0.0182, 33 MiB
    //    0.0180 vs 0.0191, 48-127 MiB equal
    const bool small = n <= (256u << 10);
    const uint64_t mib = n >> 20;
    const int lanes = (shape & 0xff) ? (int)(shape & 0xff)
                    : (crc64 ? mib >= 1024 && mib < 1536 : mib >= 512 && mib < 1536) ? 32 : 64;
    uint64_t rounds = (shape >> 8) ? shape >> 8
                    : small ? 1
                    : crc64 ? (mib < 512 ? 1 : mib < 1536 ? 2 : mib < 3072 ? 4 : 2)
                            : (mib < PCRC_LONG_R1_MIB ? 1 : mib < 1536 ? 2 : mib < 3072 ? 4 : 2);
    const uint64_t gpw = 64 / (uint64_t)lanes;
    const uint64_t maxgrid = (uint64_t)cus < kLongMaxFt ? (uint64_t)cus : kLongMaxFt;
    LongPlan p{};
    p.lanes = lanes;
    p.rounds = rounds;
    const uintptr_t d = reinterpret_cast<uintptr_t>(data);
    uint64_t head = ((d + 4095) & ~uintptr_t(4095)) - d;
    if (head > n) head = n;
    const uint64_t m = n - head;  // 0 only when the whole buffer lies before A (then the head is all of it)
    const uint64_t slots = 16ull * maxgrid * gpw * rounds;
    uint64_t chunk = ((m + slots - 1) / slots + 1023) / 1024 * 1024;  // whole rows, 1 KiB aligned
    const uint64_t lo = small ? 4096 : mib < 128 ? PCRC_LONG_MID_FLOOR : 16384;
    if (chunk < lo) chunk = lo;
    if (force_chunk) chunk = force_chunk;
    p.head = head;
    p.chunk = chunk;
    p.nchunks = (m + chunk - 1) / chunk;
    p.last = m ? m - (p.nchunks - 1) * chunk : chunk;  // no body: the head is slot R S - 1, factor 1
    const uint64_t per_wg = 16ull * gpw * rounds;
    p.grid = p.nchunks ? (p.nchunks + per_wg - 1) / per_wg : 1;
    if (p.grid > maxgrid) p.grid = maxgrid;  // only with a forced chunk: then chunks > slots
    p.stride = p.grid * 16ull * gpw;
    if (p.nchunks > rounds * p.stride) p.rounds = rounds = (p.nchunks + p.stride - 1) / p.stride;
    p.lead = rounds * p.stride - p.nchunks;
    return p;
}

// Launch constants of a plan (CRC-32C or CRC-64/ECMA), X = x^(8 chunk):
// X^S and X (basis words for the lane-parallel multiplies), Z^(15-w) with
// Z = X^GPW (a wave's factor), and J Y^(grid-1-b) with Y = Z^16 and J =
// x^-(8 (chunk - L)) (a workgroup's factor, J because the last chunk is
// short: it enters the result with factor 1 instead). Computed on first use
// per plan and kept (callers repeat sizes and alignments).
struct LongPowers {
    uint64_t chunk, last, stride, grid, lanes;
    uint32_t xsb32[32], xb32[32], zt32[16], ft32[kLongMaxFt];
    uint64_t xsb64[64], x64, zt64[16], ft64[kLongMaxFt];
};

inline const LongPowers& long_powers(const LongPlan& lp, bool crc64) {
    static std::mutex mu;
    static std::vector<LongPowers*> cache[2];
    thread_local LongPowers overflow;
    auto same = [&](const LongPowers* e) {
        return e->chunk == lp.chunk && e->last == lp.last && e->stride == lp.stride && e->grid == lp.grid &&
               e->lanes == (uint64_t)lp.lanes;
    };
    {
        std::lock_guard<std::mutex> lk(mu);
        for (auto* e : cache[crc64])
            if (same(e)) return *e;
    }
    LongPowers* t = new LongPowers();
    t->chunk = lp.chunk;
    t->last = lp.last;
    t->stride = lp.stride;
    t->grid = lp.grid;
    t->lanes = (uint64_t)lp.lanes;
    const uint64_t gpw = 64 / (uint64_t)lp.lanes, pad = 8 * (lp.chunk - lp.last), bits = 8 * lp.chunk;
    if (crc64) {
        const uint64_t x = xpow64(bits), z = gpw == 2 ? mulmod64(x, x) : x;
        uint64_t y = z;
        for (int i = 0; i < 4; ++i) y = mulmod64(y, y);  // Z^16
        const uint64_t xs = xpow64(bits * lp.stride);
        for (int i = 0; i < 64; ++i) t->xsb64[i] = mulmod64(1ull << i, xs);
        t->x64 = x;
        uint64_t zk = kOne64;  // Z^(15 - w), w = 15 .. 0
        for (int w = 15; w >= 0; --w, zk = mulmod64(zk, z)) t->zt64[w] = zk;
        uint64_t f = xpow64_inv(pad);  // J Y^(grid - 1 - b), b = grid-1 .. 0
        for (int64_t b = (int64_t)lp.grid - 1; b >= 0; --b, f = mulmod64(f, y)) t->ft64[b] = f;
    } else {
        const uint32_t x = xpow(bits), z = gpw == 2 ? mulmod(x, x) : x;
        uint32_t y = z;
        for (int i = 0; i < 4; ++i) y = mulmod(y, y);
        mul_basis(xpow(bits * lp.stride), t->xsb32);
        mul_basis(x, t->xb32);
        uint32_t zk = kOne;
        for (int w = 15; w >= 0; --w, zk = mulmod(zk, z)) t->zt32[w] = zk;
        uint32_t f = xpow_inv(pad);
        for (int64_t b = (int64_t)lp.grid - 1; b >= 0; --b, f = mulmod(f, y)) t->ft32[b] = f;
    }
    std::lock_guard<std::mutex> lk(mu);
    for (auto* e : cache[crc64])
        if (same(e)) {
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

// The kernels' arguments for a plan (CRC-32C; crc64 below).
inline void long_args(LongArgs* a, const LongPlan& lp, const LongPowers& pw, const void* data, uint32_t seed,
                      uint32_t* out) {
    a->data = static_cast<const uint8_t*>(data);
    a->head = lp.head;
    a->chunk = lp.chunk;
    a->nchunks = lp.nchunks;
    a->last = lp.last;
    a->lead = lp.lead;
    a->stride = lp.stride;
    a->rounds = (uint32_t)lp.rounds;
    a->seed = seed;
    a->out = out;
    memcpy(a->xsb, pw.xsb32, sizeof(a->xsb));
    memcpy(a->xb, pw.xb32, sizeof(a->xb));
    memcpy(a->zt, pw.zt32, sizeof(a->zt));
    memcpy(a->ft, pw.ft32, sizeof(uint32_t) * lp.grid);
}

inline void long_args64(Long64Args* a, const LongPlan& lp, const LongPowers& pw, const void* data, uint64_t seed,
                        uint64_t* out) {
    a->data = static_cast<const uint8_t*>(data);
    a->head = lp.head;
    a->chunk = lp.chunk;
    a->nchunks = lp.nchunks;
    a->last = lp.last;
    a->lead = lp.lead;
    a->stride = lp.stride;
    a->rounds = (uint32_t)lp.rounds;
    a->seed = seed;
    a->out = out;
    a->x = pw.x64;
    memcpy(a->xsb, pw.xsb64, sizeof(a->xsb));
    memcpy(a->zt, pw.zt64, sizeof(a->zt));
    memcpy(a->ft, pw.ft64, sizeof(uint64_t) * lp.grid);
}

}  // namespace pcrc
