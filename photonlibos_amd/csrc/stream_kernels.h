// stream_kernels.h -- bench-only kernel variants, NOT part of the product
// library (VERDICT r4 hygiene: they measured slower than the batch kernels on
// every config and only the ablation probes still build them): the fused
// four-row CRC32C kernel, the streaming CRC32C / CRC-64 kernels whose load
// ring runs across buffer boundaries (with their ablation switches), and the
// seed kernels that finish their results. Included by probes.hip only; the
// measurements that retired them are in DESIGN.md §4/§5.
#pragma once
#include "crc32c_kernels.h"
#include "crc64_kernels.h"

namespace pcrc {

// Seed application for uniform-length batches: crc32c_extend(d, n, s) =
// crc32c(d, n) XOR s * x^(8n) (combine identity).
struct SeedConsts {
    uint32_t basis[32];        // basis of x^(8 * nbytes) mod P
};

struct SeedConsts64 {
    uint64_t basis[64];        // basis of x^(8 * nbytes) mod P64
};

struct Uniform64Args {
    const uint8_t* base;
    uint64_t stride;
    uint64_t rows;             // nbytes / (16*G)
    uint64_t count;
    uint64_t* out;
    uint64_t init_shift;       // (~seed0) * x^(8*nbytes): the inverted init's contribution
};

// ----------------------------------------------------------------- fused path
// Four rows per step with the row shifts folded into the tables. Over a step
// of rows u = 0..3 (X = x^(8*16*G), the shift of one row of the column):
//     P <- P * X^4  ^  sum_u crc16(block_u) * X^(3-u)
// crc16(b) = D(y) where y is the CRC register after the block's first three
// word steps, so crc16(b_u) * X^(3-u) = E_{3-u}(y_u) with E_j = D * X^j: one
// 4-lookup table step per block replaces the final D step AND the S step. Per
// 16 bytes a lane does 12 D + 4 E lookups + 1 S4 lookup (17, down from 20).
//
// LDS (152 KiB, one 1024-thread workgroup per CU):
//   [0, 64K)    row idx (256 B): D at t*32 + r*4, S4 (P -> P*X^4) at 128 + t*32 + r*4
//   [64K,128K)  row idx (256 B): slot m = 0..6 at m*32 + t*8 + e*4 holds E_{3-(m%4)}
//   [128K,152K) R_k lane-combine tables (as kRBase above)
// Lane l: q = (l>>1)&3 (byte rotation), D replica r = (l&1) | ((l>>3)&3)<<1,
// E replica e = l&1, rotation g = (l>>3)&3. In E-lookup k the lane reads slot
// m = k + g, i.e. it feeds block (k+g)%4's register through E_{3-((k+g)%4)}:
// the 32 lanes of a ds_read group hit 32 distinct banks (m%4, t, e) with only
// two E replicas, and the per-lane slot is the per-lane base g*32 plus the
// instruction's immediate k*32 (slots 4..6 repeat 0..2 so no wrap is needed).
// All rows of a buffer are full: the block grid is aligned to the END of the
// buffer (pad = rows*G - nblocks zero blocks in front of block 0, plus whole
// zero rows so rows % 4 == 0). Leading zeros do not change a CRC column that
// starts at 0, so every step is a full fused step and lane l always ends
// G-1-l blocks before the end.
constexpr uint32_t kFRegionE = 65536u;
constexpr uint32_t kFRBase = 131072u;
constexpr uint32_t kFLdsBytes = kFRBase + kRBytes;           // 155648 B

struct FusedConsts {
    uint32_t xrow[5];          // X^0..X^4, X = x^(8*16*G) mod P
    uint32_t basis[6][32];     // basis of x^(128 * 2^k) mod P (lane combine)
};

struct FusedLane {
    uint32_t rot;      // 8*q
    uint32_t off[4];   // D/S: ((i+q)%4)*32 + r*4
    uint32_t offe[4];  // E:   1<<16 | g*32 + ((i+q)%4)*8 + e*4
    uint32_t r4;       // r*4 (byte-serial tail, D slice 3)
    uint32_t g;        // block rotation of the E lookups
};

__device__ __forceinline__ FusedLane fused_lane(uint32_t lane) {
    FusedLane f;
    const uint32_t q = (lane >> 1) & 3u;
    const uint32_t r = (lane & 1u) | (((lane >> 3) & 3u) << 1);
    const uint32_t e = lane & 1u;
    f.g = (lane >> 3) & 3u;
    f.rot = 8u * q;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t t = (i + q) & 3u;
        f.off[i] = (t << 5) | (r << 2);
        f.offe[i] = (1u << 16) | (f.g << 5) | (t << 3) | (e << 2);
    }
    f.r4 = r << 2;
    return f;
}

template <int I, uint32_t TOFF>
__device__ __forceinline__ uint32_t flook(const uint32_t* lds, uint32_t xr, const FusedLane& a) {
    return lds_word(lds, __builtin_amdgcn_perm(xr, a.off[I], 0x0C0C0000u | ((4u + I) << 8)) + TOFF);
}

// E lookup: bytes {offe.b0, xr.b_I, offe.b2 (= 1: region E), 0}; slot offset K*32.
template <int I, int K>
__device__ __forceinline__ uint32_t elook(const uint32_t* lds, uint32_t xr, const FusedLane& a) {
    return lds_word(lds, __builtin_amdgcn_perm(xr, a.offe[I], 0x0C020000u | ((4u + I) << 8)) + 32u * K);
}

__device__ __forceinline__ uint32_t fdstep(const uint32_t* lds, uint32_t x, const FusedLane& a, uint32_t e) {
    const uint32_t xr = __builtin_amdgcn_alignbit(x, x, a.rot);
    return xor3(xor3(flook<0, 0>(lds, xr, a), flook<1, 0>(lds, xr, a), flook<2, 0>(lds, xr, a)),
                flook<3, 0>(lds, xr, a), e);
}

template <int K>
__device__ __forceinline__ uint32_t festep(const uint32_t* lds, uint32_t x, const FusedLane& a, uint32_t e) {
    const uint32_t xr = __builtin_amdgcn_alignbit(x, x, a.rot);
    return xor3(xor3(elook<0, K>(lds, xr, a), elook<1, K>(lds, xr, a), elook<2, K>(lds, xr, a)),
                elook<3, K>(lds, xr, a), e);
}

__device__ __forceinline__ uint32_t fsstep(const uint32_t* lds, uint32_t p, const FusedLane& a) {
    const uint32_t pr = __builtin_amdgcn_alignbit(p, p, a.rot);
    return xor3(xor3(flook<0, kSOff>(lds, pr, a), flook<1, kSOff>(lds, pr, a), flook<2, kSOff>(lds, pr, a)),
                flook<3, kSOff>(lds, pr, a), 0u);
}

__device__ __forceinline__ uint32_t fbytestep(const uint32_t* lds, uint32_t c, uint8_t b, const FusedLane& a) {
    const uint32_t x = (c ^ b) & 0xffu;
    return lds_word(lds, (x << 8) + 3u * 32u + a.r4) ^ (c >> 8);
}

// One fused step over the 4 rows w[0..3] of this lane's column.
__device__ __forceinline__ uint32_t fused_step(const uint32_t* lds, uint32_t p, const uint4 (&w)[4],
                                               const FusedLane& a) {
    uint32_t y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        uint32_t c = fdstep(lds, w[u].x, a, w[u].y);
        c = fdstep(lds, c, a, w[u].z);
        y[u] = fdstep(lds, c, a, w[u].w);
    }
    // z[k] = y[(k+g)%4]: rotate the four registers by g (two select levels).
    uint32_t h[4], z[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) h[k] = (a.g & 1u) ? y[(k + 1) & 3] : y[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) z[k] = (a.g & 2u) ? h[(k + 2) & 3] : h[k];
    uint32_t s = fsstep(lds, p, a);
    s = festep<0>(lds, z[0], a, s);
    s = festep<1>(lds, z[1], a, s);
    s = festep<2>(lds, z[2], a, s);
    return festep<3>(lds, z[3], a, s);
}

__device__ __forceinline__ void build_tables_fused(uint32_t* lds, const FusedConsts& kc) {
    const uint32_t tid = threadIdx.x;
    const uint32_t t = tid >> 8, b = tid & 255u;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        uint32_t r = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) r ^= (0u - ((b >> j) & 1u)) & kc.basis[k][8 * t + j];
        lds[kFRBase / 4 + k * 1024 + t * 256 + b] = r;
    }
    const uint32_t v = b << (8 * t);
    uint32_t ev[4];
    ev[0] = mulmod(v, 0x82f63b78u);  // D: v * x^32
#pragma unroll
    for (int j = 1; j < 4; ++j) ev[j] = mulmod(ev[0], kc.xrow[j]);
    const uint32_t sv = mulmod(v, kc.xrow[4]);
    const uint32_t base = ((b << 8) + (t << 5)) >> 2;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        lds[base + r] = ev[0];
        lds[base + kSOff / 4 + r] = sv;
    }
    const uint32_t ebase = (kFRegionE + (b << 8) + (t << 3)) >> 2;
#pragma unroll
    for (int m = 0; m < 7; ++m) {
        const uint32_t val = ev[3 - (m & 3)];
        lds[ebase + m * 8] = val;
        lds[ebase + m * 8 + 1] = val;
    }
    __syncthreads();
}

template <int G>
__device__ __forceinline__ uint32_t group_reduce_f(uint32_t pc, uint32_t d, const uint32_t* lds) {
    constexpr int LOG2G = G == 64 ? 6 : G == 32 ? 5 : G == 16 ? 4 : G == 8 ? 3 : 2;
#pragma unroll
    for (int k = 0; k < LOG2G; ++k) {
        const uint32_t* R = lds + kFRBase / 4 + k * 1024;
        const uint32_t m = xor3(xor3(R[pc & 0xffu], R[256 + ((pc >> 8) & 0xffu)], R[512 + ((pc >> 16) & 0xffu)]),
                                R[768 + (pc >> 24)], 0u);
        pc = ((d >> k) & 1u) ? m : pc;
    }
    return group_xor<G>(pc);
}

template <int G>
__global__ __launch_bounds__(kBlock) void crc32c_fused_kernel(BatchArgs args, FusedConsts kc) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kFLdsBytes / 4];
    build_tables_fused(lds, kc);

    constexpr int GPW = 64 / G;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = wave_id();
    const uint32_t gl = lane & (G - 1);
    const uint32_t grp = lane / G;
    const FusedLane la = fused_lane(lane);

    const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
    for (uint64_t wv = (uint64_t)blockIdx.x * kWaves + wave; wv * GPW < args.count; wv += nwaves) {
        const uint64_t bi = wv * GPW + grp;
        const bool active = bi < args.count;
        const uint8_t* p = nullptr;
        uint64_t n = 0;
        uint32_t seed = args.seed0;
        if (active) {
            if (args.iov) {
                p = static_cast<const uint8_t*>(args.iov[bi].base);
                n = args.iov[bi].len;
            } else {
                p = args.base + bi * args.stride;
                n = args.nbytes;
            }
            if (args.seeds) seed = args.seeds[bi];
        }

        uint32_t crc;
        if (n < 64) {
            crc = seed;
            if (gl == 0)
                for (uint64_t k = 0; k < n; ++k) crc = fbytestep(lds, crc, load8(p + k), la);
        } else {
            const uint8_t* a0 = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(15));
            const uint8_t* e = p + n;
            const uint8_t* eb = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(e) & ~uintptr_t(15));
            const int s0 = (int)(p - a0);
            const int64_t nb = (int64_t)((uint64_t)(eb - a0) >> 4);  // >= 3
            const int64_t rows = (nb + G - 1) / G;
            const int64_t steps = (rows + 3) / 4;
            const int64_t pad = rows * G - nb;                   // zero blocks before block 0
            const int64_t zr = steps * 4 - rows;                 // zero rows before that
            // Block index of this lane in grid row R: (R - zr)*G + gl - pad.
            const int64_t b0 = (int64_t)gl - pad - zr * G;

            // First two steps: blocks may precede block 0 (zeros) or be blocks
            // 0/1 (masked head + seed).
            auto load_checked = [&](int64_t s, uint4 (&w)[4]) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int64_t bidx = b0 + (4 * s + u) * G;
                    uint4 v = make_uint4(0, 0, 0, 0);
                    if (bidx >= 0) {
                        v = load16(a0 + 16 * bidx);
                        if (bidx < 2) {
                            const int off = (int)bidx * 16;
                            v.x = head_word(v.x, off, s0, seed);
                            v.y = head_word(v.y, off + 4, s0, seed);
                            v.z = head_word(v.z, off + 8, s0, seed);
                            v.w = head_word(v.w, off + 12, s0, seed);
                        }
                    }
                    w[u] = v;
                }
            };
            const uint8_t* lp = a0 + 16 * b0;  // grid row 0 of this lane (may precede a0)
            auto load_step = [&](int64_t s, uint4 (&w)[4]) {
#pragma unroll
                for (int u = 0; u < 4; ++u) w[u] = load16(lp + (4 * s + u) * (16 * G));
            };

            // Double-buffered: the next step's 4 rows are in flight while this
            // one is reduced (deeper rings measured slower: more VGPRs, same HBM).
            uint32_t pc = 0;
            {
                uint4 cur[4];
                load_checked(0, cur);
                int64_t s = 0;
                if (steps > 1) {
                    uint4 nxt[4];
                    load_checked(1, nxt);
                    pc = fused_step(lds, pc, cur, la);
#pragma unroll
                    for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
                    s = 1;
                }
                for (; s + 1 < steps; ++s) {
                    uint4 nxt[4];
                    load_step(s + 1, nxt);
                    pc = fused_step(lds, pc, cur, la);
#pragma unroll
                    for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
                }
                pc = fused_step(lds, pc, cur, la);
            }

            crc = group_reduce_f<G>(pc, G - 1 - gl, lds);
            if (gl == 0)
                for (const uint8_t* q = eb; q < e; ++q) crc = fbytestep(lds, crc, load8(q), la);
        }
        if (active && gl == 0) args.out[bi] = crc;
    }
}

// ------------------------------------------------------------ streaming path
// Uniform batches: base and stride 16-byte aligned, nbytes = R*16*B*G with
// R % U == 0. A row is B*G consecutive 16-byte blocks; load b of a row is the
// coalesced sweep of blocks [b*G, (b+1)*G). A DPP butterfly inside groups of
// B lanes then gives every lane a RUN of B consecutive blocks, so the
// loop-carried row shift (4 S-table lookups) is paid once per 16*B bytes.
// Each wave walks the rows of its buffers (slots j = 0,1,...: buffer tuple
// wv0 + j*nwaves) as ONE stream of steps of U rows, with a ring of D steps of
// loads in flight that never drains at buffer boundaries.
struct UniformArgs {
    const uint8_t* base;
    uint64_t stride;
    uint64_t rows;       // R = nbytes / (16*B*G)
    uint64_t count;
    uint32_t* out;       // crc32c with seed 0; seeds are folded in by crc32c_seed_kernel
};

// Exchange with lane (lane ^ BIT) (BIT = 1 or 2: DPP quad permutations).
template <int BIT>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
    constexpr int ctrl = BIT == 1 ? 0xB1 : 0x4E;  // quad_perm [1,0,3,2] / [2,3,0,1]
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xF, 0xF, false);
}

template <int BIT>
__device__ __forceinline__ void bfly_word(uint32_t& lo_reg, uint32_t& hi_reg, bool hi) {
    const uint32_t send = hi ? lo_reg : hi_reg;
    const uint32_t recv = lane_xor<BIT>(send);
    lo_reg = hi ? recv : lo_reg;
    hi_reg = hi ? hi_reg : recv;
}

template <int BIT>
__device__ __forceinline__ void bfly(uint4& lo, uint4& hi_blk, bool hi) {
    bfly_word<BIT>(lo.x, hi_blk.x, hi);
    bfly_word<BIT>(lo.y, hi_blk.y, hi);
    bfly_word<BIT>(lo.z, hi_blk.z, hi);
    bfly_word<BIT>(lo.w, hi_blk.w, hi);
}

// Transpose r[b] (lane t of a B-group holds block t + b*G) into the run
// r[b] = block (t*G + b) of the group's first block: butterfly over the bits of B.
template <int B>
__device__ __forceinline__ void to_runs(uint4 (&r)[B], uint32_t t) {
    if constexpr (B >= 2) {
#pragma unroll
        for (int m = 0; m < B; m += 2) bfly<1>(r[m], r[m + 1], (t & 1u) != 0);
    }
    if constexpr (B >= 4) {
#pragma unroll
        for (int m = 0; m < B; ++m)
            if ((m & 2) == 0) bfly<2>(r[m], r[m + 2], (t & 2u) != 0);
    }
}

// CRC (init 0) of a run of B blocks.
template <int B>
__device__ __forceinline__ uint32_t run_crc(const uint32_t* lds, const uint4 (&r)[B], const LaneAddr& a) {
    uint32_t c = crc16(lds, r[0], a);
#pragma unroll
    for (int b = 1; b < B; ++b) {
        c = dstep(lds, c ^ r[b].x, a, r[b].y);
        c = dstep(lds, c, a, r[b].z);
        c = dstep(lds, c, a, r[b].w);
        c = dstep(lds, c, a);
    }
    return c;
}

// ABL != 0 only in bench-only ablation builds (probes.hip): 1 = drop the S
// (row-shift) lookups, 2 = one word step per block instead of four, 4 = no
// table lookups at all. Results are then NOT CRCs.
template <int G, int B, int U, int D, int ABL = 0>
__global__ __launch_bounds__(kBlock) void crc32c_uniform_kernel(UniformArgs args, LaneConsts kc) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytes / 4];
    build_tables(lds, kc);

    constexpr uint64_t GPW = 64 / G;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gl = lane & (G - 1);
    const uint32_t grp = lane / G;
    const uint32_t tb = gl & (B - 1);                    // position in the B-group
    const uint32_t run = tb * (G / B) + gl / B;          // this lane's run index within a row
    const LaneAddr la = lane_addr(lane);

    const uint64_t ngroups = (args.count + GPW - 1) / GPW;
    const uint64_t wv0 = (uint64_t)blockIdx.x * kWaves + wave_id();
    const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
    if (wv0 >= ngroups) return;
    const uint64_t nslots = (ngroups - 1 - wv0) / nwaves + 1;
    const uint64_t spb = args.rows / U;               // steps per buffer
    const uint64_t nsteps = nslots * spb;
    constexpr uint64_t kSweep = 16ull * G;            // bytes of one load instruction's sweep
    constexpr uint64_t kRow = kSweep * B;

    auto buffer_of = [&](uint64_t slot) -> uint64_t {
        const uint64_t bi = (wv0 + slot * nwaves) * GPW + grp;
        return bi < args.count ? bi : args.count - 1;  // idle lanes of a last partial tuple
    };
    auto slot_base = [&](uint64_t slot) -> const uint8_t* {
        if (slot >= nslots) slot = nslots - 1;           // padding steps re-read valid rows
        return args.base + buffer_of(slot) * args.stride + 16ull * gl;
    };

    // Load cursor (slot, step-in-buffer, pointer).
    uint64_t lslot = 0, lstep = 0;
    const uint8_t* lptr = slot_base(0);
    auto advance = [&]() {
        if (++lstep == spb) {
            lstep = 0;
            ++lslot;
            lptr = slot_base(lslot);
        } else if (lslot < nslots) {
            lptr += kRow * U;
        }
    };

    // D steps in flight; D+1 register sets so that a refill never targets a
    // set that is still being read (no register copies across the loop edge,
    // which would force a vmcnt(0) drain).
    constexpr int S = D + 1;
    uint4 ring[S][U][B];
#pragma unroll
    for (int d = 0; d < D; ++d) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int b = 0; b < B; ++b) ring[d][u][b] = load16(lptr + u * kRow + b * kSweep);
        advance();
    }
    const uint64_t padded = (nsteps + S - 1) / S * S;

    uint64_t slot = 0, step = 0;
    uint32_t pc = 0;
    for (uint64_t s = 0; s < padded; s += S) {
#pragma unroll
        for (int d = 0; d < S; ++d) {
            const int refill = (d + D) % S;  // the set read by the previous stage
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int b = 0; b < B; ++b) ring[refill][u][b] = load16(lptr + u * kRow + b * kSweep);
            advance();
            uint32_t c[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                to_runs<B>(ring[d][u], tb);
                if constexpr (ABL & 4) {
                    const uint4 w = ring[d][u][0];
                    c[u] = w.x ^ w.y ^ w.z ^ w.w;
                } else if constexpr (ABL & 2) {
                    const uint4 w = ring[d][u][0];
                    c[u] = dstep(lds, w.x ^ w.y ^ w.z ^ w.w, la);
                } else if constexpr (B == 1) {
                    c[u] = lag16(lds, ring[d][u][0], la);  // lagged blocks: 16 lookups per 16 B
                } else {
                    c[u] = run_crc<B>(lds, ring[d][u], la);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if constexpr (ABL & 1) pc = (pc ^ (pc << 1)) ^ c[u];
                else pc = sstep(lds, pc, la, c[u]);
            }
            if (++step == spb) {
                // End of this buffer: this lane's last run is G-1-run runs from the end.
                if constexpr (B == 1 && ABL == 0) pc = dstep(lds, pc, la);  // Q -> P (lagged)
                const uint32_t crc = group_reduce<G>(pc, (uint32_t)(G - 1 - run), lds);
                const uint64_t bi = (wv0 + slot * nwaves) * GPW + grp;
                if (gl == 0 && slot < nslots && bi < args.count) args.out[bi] = crc;
                pc = 0;
                step = 0;
                ++slot;
            }
        }
    }
}

// out[i] ^= seed_i * x^(8*nbytes): crc32c_extend(d, n, s) = crc32c(d, n) ^ s*x^(8n).
__global__ void crc32c_seed_kernel(uint32_t* out, uint64_t count, const uint32_t* seeds, uint32_t seed0,
                                   SeedConsts sc) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    out[i] ^= mul_basis_dev(seeds ? seeds[i] : seed0, sc.basis);
}

// Uniform batches (aligned base and stride, nbytes = R*16*G with R % U == 0):
// the continuous cross-buffer load ring of crc32c_uniform_kernel (B = 1).
// Register init 0; lane 0 applies the inverted init (~seed0 * x^(8n)) and the
// final inversion; per-buffer seeds are folded in by crc64_seed_kernel.
// V interleaved partials per lane: partial j takes rows r = j (mod V), i.e.
// lane l plays virtual lane j*G + l of a V*G-lane geometry (row shift
// x^(8*16*G*V), the kc passed is lane_consts64(G*V)); V independent S chains
// of U/V steps instead of one of U steps.
// Lagged CRC (x^-64 times the CRC register, init 0) after a run of B
// consecutive 16-byte blocks (lag16_64 for B = 1).
template <int B>
__device__ __forceinline__ uint2 lag_run64(const uint32_t* lds, const uint4 (&w)[B], const LaneAddr64& a) {
    uint2 c = dstep64(lds, make_uint2(w[0].x, w[0].y), a, make_uint2(w[0].z, w[0].w));
#pragma unroll
    for (int b = 1; b < B; ++b) {
        c = dstep64(lds, c, a, make_uint2(w[b].x, w[b].y));
        c = dstep64(lds, c, a, make_uint2(w[b].z, w[b].w));
    }
    return c;
}

// B = 2: each lane reads a RUN of two consecutive blocks per row (two
// dwordx4 loads, lane stride 32 B) and pays the row shift once per 32 bytes
// (3 D + 1 S steps = 32 lookups per 32 B, as two lagged single blocks). The
// lane then plays the 2G-lane geometry's blocks 2l, 2l+1 (kc = lane_consts64(2G)).
// ABL != 0 only in bench-only ablation builds (probes.hip); results are then
// NOT CRCs: 1 = no S (row-shift) lookups, 2 = one D step on lo ^ hi per
// block (no data chain), 4 = no table lookups at all.
// V = B = 1 (one partial per lane, single blocks): the batch kernel's finish
// (finish tables A_dl / B_dh, finish_xor16 at 16 lanes: 17 lookups per lane)
// instead of a D step plus log2(G) R64 levels (8 + 16 log2(G) lookups).
template <int G, int U, int D, int V = 1, int B = 1, int ABL = 0>
__global__ __launch_bounds__(kBlock) void crc64_uniform_kernel(Uniform64Args args, LaneConsts64 kc) {
    constexpr bool kFin = V == 1 && B == 1 && ABL == 0;
    __shared__ __attribute__((aligned(16))) uint32_t lds[(kFin ? k64FLdsBytes : k64LdsBytes) / 4];
    build_tables64<kFin ? G : 0>(lds, kc);

    constexpr uint64_t GPW = 64 / G;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gl = lane & (G - 1);
    const uint32_t grp = lane / G;
    const LaneAddr64 la = lane_addr64(lane);

    const uint64_t ngroups = (args.count + GPW - 1) / GPW;
    const uint64_t wv0 = (uint64_t)blockIdx.x * kWaves + wave_id();
    const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
    if (wv0 >= ngroups) return;
    const uint64_t nslots = (ngroups - 1 - wv0) / nwaves + 1;
    const uint64_t spb = args.rows / U;
    const uint64_t nsteps = nslots * spb;
    constexpr uint64_t kRow = 16ull * G * B;

    auto buffer_of = [&](uint64_t slot) -> uint64_t {
        const uint64_t bi = (wv0 + slot * nwaves) * GPW + grp;
        return bi < args.count ? bi : args.count - 1;
    };
    auto slot_base = [&](uint64_t slot) -> const uint8_t* {
        if (slot >= nslots) slot = nslots - 1;
        return args.base + buffer_of(slot) * args.stride + 16ull * B * gl;
    };
    uint64_t lslot = 0, lstep = 0;
    const uint8_t* lptr = slot_base(0);
    auto advance = [&]() {
        if (++lstep == spb) {
            lstep = 0;
            ++lslot;
            lptr = slot_base(lslot);
        } else if (lslot < nslots) {
            lptr += kRow * U;
        }
    };
    constexpr int S = D + 1;
    uint4 ring[S][U][B];
#pragma unroll
    for (int d = 0; d < D; ++d) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int b = 0; b < B; ++b) ring[d][u][b] = load16(lptr + u * kRow + 16 * b);
        advance();
    }
    const uint64_t padded = (nsteps + S - 1) / S * S;
    static_assert(U % V == 0 && G * V * B <= 64 && (V == 1 || B == 1),
                  "interleave must divide the step; V*B*G virtual lanes <= 64; runs and interleave exclusive");
    constexpr int VGB = G * V * B;
    constexpr int LOG2VG = VGB == 64 ? 6 : VGB == 32 ? 5 : VGB == 16 ? 4 : VGB == 8 ? 3 : 2;
    uint64_t slot = 0, step = 0;
    uint2 pc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) pc[j] = make_uint2(0, 0);
    for (uint64_t s = 0; s < padded; s += S) {
#pragma unroll
        for (int d = 0; d < S; ++d) {
            const int refill = (d + D) % S;
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int b = 0; b < B; ++b) ring[refill][u][b] = load16(lptr + u * kRow + 16 * b);
            advance();
            uint2 c[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if constexpr (ABL & 4) {
                    c[u] = make_uint2(ring[d][u][0].x ^ ring[d][u][0].z, ring[d][u][0].y ^ ring[d][u][0].w);
                } else if constexpr (ABL & 2) {
                    c[u] = dstep64(lds, make_uint2(ring[d][u][0].x ^ ring[d][u][0].z, ring[d][u][0].y ^ ring[d][u][0].w),
                                   la);
                } else {
                    c[u] = lag_run64<B>(lds, ring[d][u], la);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if constexpr (ABL & 1) pc[u % V] = make_uint2((pc[u % V].x ^ (pc[u % V].y << 1)) ^ c[u].x,
                                                              (pc[u % V].y ^ (pc[u % V].x >> 1)) ^ c[u].y);
                else pc[u % V] = sstep64(lds, pc[u % V], la, c[u]);
            }
            if (++step == spb) {
                uint64_t acc = 0;
                if constexpr (kFin) {  // Q * x^(64 + 128 d), d = G - 1 - gl, XOR over the group
                    const uint32_t d = G - 1 - gl;
                    if constexpr (G == 16 && PCRC64_FIN16) {
                        acc = finish_xor16(pc[0], d, lds, gl, lane);
                    } else {
                        const uint64_t f = finish64<G>(pc[0], d, lds, lane);
                        acc = ((uint64_t)group_xor<G>((uint32_t)(f >> 32)) << 32) | group_xor<G>((uint32_t)f);
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < V; ++j)  // Q -> P (dstep), then the lane shift
                        acc ^= shift64<LOG2VG>(u64of(ABL ? pc[j] : dstep64(lds, pc[j], la)),
                                               (uint32_t)((G * V - 1 - (j * G + gl)) * B), lds);
#pragma unroll
                    for (int o = G / 2; o > 0; o >>= 1) {
                        const uint32_t lo32 = (uint32_t)__shfl_xor((int)(uint32_t)acc, o, 64);
                        const uint32_t hi32 = (uint32_t)__shfl_xor((int)(uint32_t)(acc >> 32), o, 64);
                        acc ^= ((uint64_t)hi32 << 32) | lo32;
                    }
                }
                const uint64_t bi = (wv0 + slot * nwaves) * GPW + grp;
                if (gl == 0 && slot < nslots && bi < args.count) args.out[bi] = ~(acc ^ args.init_shift);
#pragma unroll
                for (int j = 0; j < V; ++j) pc[j] = make_uint2(0, 0);
                step = 0;
                ++slot;
            }
        }
    }
}

// out[i] ^= seed_i * x^(8*nbytes) (the uniform kernel used seed0 = 0:
// ~(F ^ ~s*X) = ~(F ^ ~0*X) ^ s*X).
__global__ void crc64_seed_kernel(uint64_t* out, uint64_t count, const uint64_t* seeds, SeedConsts64 sc) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    out[i] ^= mul_basis64(seeds[i], sc.basis);
}


}  // namespace pcrc
