// crc32c_kernels.h -- device code of the MI355X CRC32C engine (see the
// overview at the top of crc32c_device.hip and DESIGN.md "Kernels"). Included
// by crc32c_device.hip (the product) and probes.hip (bench-only ablations).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/photon_crc/crc32c_gpu.h"
#include "gf2.h"

namespace pcrc {

// ------------------------------------------------------------------ LDS map
constexpr uint32_t kDataBytes = 2u * 65536u;   // 4 slices x 256 idx x 32 replicas x 4 B
constexpr uint32_t kShiftBase = kDataBytes;    // S tables follow
constexpr uint32_t kShiftBytes = 4u * 4096u;   // 4 slices x 256 idx x 4 replicas x 4 B
constexpr uint32_t kBasisBase = kShiftBase + kShiftBytes;  // lane-combine constants
constexpr uint32_t kBasisBytes = 6u * 32u * 4u;
constexpr uint32_t kLdsBytes = kBasisBase + kBasisBytes;   // 148224 B of the 160 KiB
constexpr int kBlock = 1024;                   // 16 waves, one workgroup per CU
constexpr int kWaves = kBlock / 64;

// Kernel constants computed on the host (gf2.h) per lanes-per-buffer G.
struct LaneConsts {
    uint32_t kshift;           // x^(8*16*G) mod P: one row of the lane's column
    uint32_t basis[6][32];     // basis of x^(128 * 2^k) mod P, k = 0..5
};

// Seed application for uniform-length batches: crc32c_extend(d, n, s) =
// crc32c(d, n) XOR s * x^(8n) (combine identity).
struct SeedConsts {
    uint32_t basis[32];        // basis of x^(8 * nbytes) mod P
};

struct BatchArgs {
    const uint8_t* base;       // strided mode
    uint64_t stride;
    uint64_t nbytes;
    const photon_crc_iovec* iov;  // iov mode when non-null
    uint64_t count;
    const uint32_t* seeds;     // optional
    uint32_t* out;
    uint32_t seed0;
};

__device__ __forceinline__ uint32_t lds_word(const uint32_t* lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

// Per-lane LDS base addresses: D slice t lives at ((t>>1)<<16) + idx*256 +
// ((t&1)<<7) + (lane&31)*4, so its address is (idx << 8) | d[t].
struct LaneAddr {
    uint32_t d0, d1, d2, d3, s;
};

// x * x^32 mod P = CRC register after absorbing the 32-bit word x.
// Address of slice t for byte t of x in ONE v_perm_b32: result bytes are
// {d.byte0, x.byte t, d.byte2, 0} (selector 0..3 = second operand's bytes,
// 4..7 = first operand's bytes, 12 = 0x00).
template <int T>
__device__ __forceinline__ uint32_t daddr(uint32_t x, uint32_t d) {
    return __builtin_amdgcn_perm(x, d, 0x0C020000u | ((4u + T) << 8));
}

__device__ __forceinline__ uint32_t dstep(const uint32_t* lds, uint32_t x, const LaneAddr& a) {
    const uint32_t t0 = lds_word(lds, daddr<0>(x, a.d0));
    const uint32_t t1 = lds_word(lds, daddr<1>(x, a.d1));
    const uint32_t t2 = lds_word(lds, daddr<2>(x, a.d2));
    const uint32_t t3 = lds_word(lds, daddr<3>(x, a.d3));
    return t0 ^ t1 ^ t2 ^ t3;
}

// P * x^(8*gap+32) mod P through the S tables (slice t at s + t*4096 + idx*16).
__device__ __forceinline__ uint32_t sstep(const uint32_t* lds, uint32_t p, uint32_t s) {
    const uint32_t t0 = lds_word(lds, s + ((p << 4) & 0xff0u));
    const uint32_t t1 = lds_word(lds, s + 4096u + ((p >> 4) & 0xff0u));
    const uint32_t t2 = lds_word(lds, s + 8192u + ((p >> 12) & 0xff0u));
    const uint32_t t3 = lds_word(lds, s + 12288u + ((p >> 20) & 0xff0u));
    return t0 ^ t1 ^ t2 ^ t3;
}

// Byte-serial step with the D3 slice (D3[b] = b<<24 * x^32 = b * x^8, the
// classic byte table).
__device__ __forceinline__ uint32_t bytestep(const uint32_t* lds, uint32_t c, uint8_t b, const LaneAddr& a) {
    const uint32_t x = c ^ b;
    return lds_word(lds, daddr<0>(x, a.d3)) ^ (c >> 8);
}

// CRC (init 0, no xorout) of one 16-byte block: four chained word steps.
__device__ __forceinline__ uint32_t crc16(const uint32_t* lds, uint4 w, const LaneAddr& a) {
    uint32_t c = dstep(lds, w.x, a);
    c = dstep(lds, c ^ w.y, a);
    c = dstep(lds, c ^ w.z, a);
    return dstep(lds, c ^ w.w, a);
}

// U blocks of one lane's column: the crc16s are independent (ILP), only the
// row shift is carried.
template <int U>
__device__ __forceinline__ uint32_t column_step(const uint32_t* lds, uint32_t p, const uint4 (&w)[U],
                                                const LaneAddr& a) {
    uint32_t c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) c[u] = crc16(lds, w[u], a);
#pragma unroll
    for (int u = 0; u < U; ++u) p = sstep(lds, p, a.s) ^ c[u];
    return p;
}

__device__ __forceinline__ uint32_t column_step1(const uint32_t* lds, uint32_t p, uint4 w, const LaneAddr& a) {
    return sstep(lds, p, a.s) ^ crc16(lds, w, a);
}

// Word at byte offset `off` (relative to the aligned start A0) of the first
// two blocks: zero the bytes before the data start s0 and XOR the seed into
// data bytes s0..s0+3 (CRC with init s == CRC with init 0 of the data whose
// first 4 bytes are XORed with s; leading zeros do not change a CRC).
__device__ __forceinline__ uint32_t head_word(uint32_t w, int off, int s0, uint32_t seed) {
    const int k = s0 - off;
    if (k >= 4) return 0u;
    if (k > 0) w &= 0xffffffffu << (8 * k);
    if (k >= 0) w ^= seed << (8 * k);
    else if (k > -4) w ^= seed >> (8 * -k);
    return w;
}

__device__ __forceinline__ uint32_t mul_basis_dev(uint32_t p, const uint32_t* basis) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) r ^= (0u - ((p >> i) & 1u)) & basis[i];
    return r;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(1))) const uint8_t g_u8;

// Streaming 16-byte global load (every payload byte is read exactly once).
// The explicit global address space keeps it a global_load_dwordx4: a flat
// load would also count on lgkmcnt and serialise against the LDS lookups.
__device__ __forceinline__ uint4 load16(const uint8_t* p) {
    const u32x4 v = __builtin_nontemporal_load((g_u32x4*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint8_t load8(const uint8_t* p) { return *(g_u8*)p; }

// Build the D and S tables in LDS (every workgroup; 1024 threads = one entry of
// each table per thread).
__device__ __forceinline__ void build_tables(uint32_t* lds, const LaneConsts& kc) {
    const uint32_t kshift = kc.kshift;
    const uint32_t tid = threadIdx.x;
    if (tid < 6 * 32) lds[kBasisBase / 4 + tid] = kc.basis[tid >> 5][tid & 31];
    const uint32_t t = tid >> 8, b = tid & 255u;
    const uint32_t v = b << (8 * t);
    const uint32_t dv = mulmod(v, 0x82f63b78u);  // x^32 mod P
    const uint32_t dbase = (((t >> 1) << 16) + (b << 8) + ((t & 1) << 7)) >> 2;
#pragma unroll
    for (int r = 0; r < 32; ++r) lds[dbase + r] = dv;
    const uint32_t sv = mulmod(v, kshift);
    const uint32_t sbase = (kShiftBase + t * 4096u + b * 16u) >> 2;
#pragma unroll
    for (int r = 0; r < 4; ++r) lds[sbase + r] = sv;
    __syncthreads();
}

__device__ __forceinline__ LaneAddr lane_addr(uint32_t lane) {
    LaneAddr la;
    la.d0 = ((lane & 31u) << 2);
    la.d1 = (1u << 7) | ((lane & 31u) << 2);
    la.d2 = (1u << 16) | ((lane & 31u) << 2);
    la.d3 = (1u << 16) | (1u << 7) | ((lane & 31u) << 2);
    la.s = kShiftBase + ((lane & 3u) << 2);
    return la;
}

// Shift lane partials to the end of the body (d blocks of 16 bytes) and
// XOR-reduce over the G lanes of the group.
// p * K with K's basis (32 words) in LDS, read 4 words at a time (broadcast).
__device__ __forceinline__ uint32_t mul_basis_lds(uint32_t p, const uint32_t* basis) {
    uint32_t r = 0;
#pragma unroll 2
    for (int q = 0; q < 8; ++q) {
        const uint4 b = reinterpret_cast<const uint4*>(basis)[q];
        r ^= (0u - ((p >> (4 * q)) & 1u)) & b.x;
        r ^= (0u - ((p >> (4 * q + 1)) & 1u)) & b.y;
        r ^= (0u - ((p >> (4 * q + 2)) & 1u)) & b.z;
        r ^= (0u - ((p >> (4 * q + 3)) & 1u)) & b.w;
    }
    return r;
}

template <int G>
__device__ __forceinline__ uint32_t group_reduce(uint32_t pc, uint32_t d, const uint32_t* lds) {
    constexpr int LOG2G = G == 64 ? 6 : G == 32 ? 5 : G == 16 ? 4 : G == 8 ? 3 : 2;
    // basis[k][i] of x^(128*2^k), staged in LDS by build_tables.
    const uint32_t* basis = lds + kBasisBase / 4;
#pragma unroll 1
    for (int k = 0; k < LOG2G; ++k)
        if ((d >> k) & 1u) pc = mul_basis_lds(pc, basis + 32 * k);
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) pc ^= (uint32_t)__shfl_xor((int)pc, o, 64);
    return pc;
}

__device__ __forceinline__ uint32_t wave_id() {
    return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

// -------------------------------------------------------------- generic path
// Any pointer, any length, any seed; one group of G lanes per buffer.
template <int G>
__global__ __launch_bounds__(kBlock) void crc32c_batch_kernel(BatchArgs args, LaneConsts kc) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytes / 4];
    build_tables(lds, kc);

    constexpr int GPW = 64 / G;  // buffers per wavefront
    constexpr int U = 4;         // blocks per lane per step
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = wave_id();
    const uint32_t gl = lane & (G - 1);
    const uint32_t grp = lane / G;
    const LaneAddr la = lane_addr(lane);

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
            // Tiny buffer: byte-serial on the group's first lane.
            crc = seed;
            if (gl == 0)
                for (uint64_t k = 0; k < n; ++k) crc = bytestep(lds, crc, load8(p + k), la);
        } else {
            const uint8_t* a0 = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(15));
            const uint8_t* e = p + n;
            const uint8_t* eb = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(e) & ~uintptr_t(15));
            const int s0 = (int)(p - a0);
            const uint64_t nb = (uint64_t)(eb - a0) >> 4;  // >= 3 blocks since n >= 64
            const uint64_t full = nb / G;                   // rows where every lane has a block
            const uint64_t rows = (nb + G - 1) / G;
            const uint32_t rlast = (uint32_t)(nb - (rows - 1) * G);  // blocks in the last row, 1..G
            const uint8_t* lp = a0 + 16 * gl;               // this lane's block in row 0

            // Row 0 (holds the head: masked leading bytes + seed).
            uint32_t pc = 0;
            if (gl < nb) {
                uint4 w = load16(lp);
                if (gl < 2) {
                    const int off = (int)gl * 16;
                    w.x = head_word(w.x, off, s0, seed);
                    w.y = head_word(w.y, off + 4, s0, seed);
                    w.z = head_word(w.z, off + 8, s0, seed);
                    w.w = head_word(w.w, off + 12, s0, seed);
                }
                pc = crc16(lds, w, la);
            }
            // Full rows 1..full-1: U rows per step, the next U in flight.
            uint64_t row = 1;
            if (row + U <= full) {
                uint4 cur[U];
#pragma unroll
                for (int u = 0; u < U; ++u) cur[u] = load16(lp + (row + u) * (16 * G));
                for (; row + 2 * U <= full; row += U) {
                    uint4 nxt[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) nxt[u] = load16(lp + (row + U + u) * (16 * G));
                    pc = column_step<U>(lds, pc, cur, la);
#pragma unroll
                    for (int u = 0; u < U; ++u) cur[u] = nxt[u];
                }
                pc = column_step<U>(lds, pc, cur, la);
                row += U;
            }
            for (; row < full; ++row) pc = column_step1(lds, pc, load16(lp + row * (16 * G)), la);
            // Partial last row.
            if (full >= 1 && full < rows && full * G + gl < nb)
                pc = column_step1(lds, pc, load16(lp + full * (16 * G)), la);

            crc = group_reduce<G>(pc, (rlast + G - 1 - gl) & (G - 1), lds);
            // Ragged tail (< 16 bytes) after the last aligned block.
            if (gl == 0)
                for (const uint8_t* q = eb; q < e; ++q) crc = bytestep(lds, crc, load8(q), la);
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
        c = dstep(lds, c ^ r[b].x, a);
        c = dstep(lds, c ^ r[b].y, a);
        c = dstep(lds, c ^ r[b].z, a);
        c = dstep(lds, c ^ r[b].w, a);
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
                } else {
                    c[u] = run_crc<B>(lds, ring[d][u], la);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if constexpr (ABL & 1) pc = (pc ^ (pc << 1)) ^ c[u];
                else pc = sstep(lds, pc, la.s) ^ c[u];
            }
            if (++step == spb) {
                // End of this buffer: this lane's last run is G-1-run runs from the end.
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

// Per-message fold of per-segment CRCs: acc = seed; acc = acc*x^(8 len)+crc.
// (Crc32Hasher::extend_hash, rpc/serialize.h:244-252, equals this fold.)
struct PowTable {
    uint32_t x8pow2[64];  // x^(8 * 2^i) mod P
};

__device__ __forceinline__ uint32_t shift_bytes_tab(uint32_t crc, uint64_t n, const PowTable& t) {
    for (int i = 0; n; ++i, n >>= 1)
        if (n & 1) crc = mulmod(crc, t.x8pow2[i]);
    return crc;
}

__global__ void crc32c_msg_fold_kernel(const photon_crc_iovec* iov, const uint64_t* msg_start, uint64_t nmsg,
                                       const uint32_t* seg_crc, uint32_t seed0, const uint32_t* seeds,
                                       uint32_t* out, PowTable pt) {
    const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= nmsg) return;
    uint32_t acc = seeds ? seeds[m] : seed0;
    for (uint64_t s = msg_start[m]; s < msg_start[m + 1]; ++s)
        acc = shift_bytes_tab(acc, iov[s].len, pt) ^ seg_crc[s];
    out[m] = acc;
}

__global__ void crc32c_combine_kernel(const uint32_t* c1, const uint32_t* c2, const uint32_t* l2, uint64_t n,
                                      uint32_t* out, PowTable pt) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t a = c1[i], b = c2[i], len = l2[i];
    // crc.cpp:394-395 / 425-426 shortcuts, then crc1 * x^(8 len2) ^ crc2.
    out[i] = !a ? b : !len ? a : (shift_bytes_tab(a, len, pt) ^ b);
}

// ------------------------------------------- device series / trim / extend
// (crc32c.h:52-57, 71-74, 84-87 over device memory.)

// combine_series with part_size > 0 is linear (the crc1 == 0 shortcut of
// crc.cpp:394 agrees with the formula): result = XOR_i crc[i] * K^(n-1-i),
// K = x^(8*part_size). Thread t Horner-folds kSeriesChunk consecutive parts,
// shifts its partial by K^(parts after its chunk) and XOR-reduces into
// *result (zeroed by the caller; XOR is order-free, so atomics stay exact).
constexpr int kSeriesChunk = 16;

__global__ __launch_bounds__(256) void crc32c_combine_series_kernel(const uint32_t* crc, uint64_t n,
                                                                    uint32_t* result, PowTable kp) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t lo = t * kSeriesChunk;
    uint32_t acc = 0;
    if (lo < n) {
        const uint64_t hi = lo + kSeriesChunk < n ? lo + kSeriesChunk : n;
        for (uint64_t i = lo; i < hi; ++i) acc = mulmod(acc, kp.x8pow2[0]) ^ crc[i];
        acc = shift_bytes_tab(acc, n - hi, kp);  // kp.x8pow2[j] = K^(2^j)
    }
    for (int off = 32; off; off >>= 1) acc ^= __shfl_xor(acc, off);
    if ((threadIdx.x & 63u) == 0 && acc) atomicXor(result, acc);
}

// combine_series with part_size == 0: every combine takes a shortcut
// (crc.cpp:394-395), so the fold is the first non-zero crc (0 if none).
__global__ __launch_bounds__(1024) void crc32c_first_nonzero_kernel(const uint32_t* crc, uint64_t n,
                                                                    uint32_t* result) {
    __shared__ unsigned long long first;
    if (threadIdx.x == 0) first = ~0ull;
    __syncthreads();
    for (uint64_t base = 0; base < n; base += blockDim.x) {
        const uint64_t i = base + threadIdx.x;
        if (i < n && crc[i]) atomicMin(&first, (unsigned long long)i);
        __syncthreads();
        if (first != ~0ull) break;
        __syncthreads();
    }
    if (threadIdx.x == 0) *result = first == ~0ull ? 0u : crc[first];
}

// crc32c_trim (crc.cpp:442-464) per element, including its 32-bit size sum
// and the combine shortcuts. Inconsistent sizes give 0 and count an error
// (the reference sets errno = EINVAL and returns 0).
__global__ void crc32c_trim_kernel(const photon_crc_component* all, const photon_crc_component* pre,
                                   const photon_crc_component* suf, uint64_t n, uint32_t* out, uint32_t* nerr,
                                   PowTable lsh, PowTable rsh) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const photon_crc_component a = all[i], p = pre[i], s = suf[i];
    if (a.size < (uint32_t)(p.size + s.size)) {
        out[i] = 0;
        if (nerr) atomicAdd(nerr, 1u);
        return;
    }
    uint32_t crc = a.crc;
    if (p.size) {
        const uint32_t len = a.size - p.size;
        crc = !p.crc ? crc : !len ? p.crc : (shift_bytes_tab(p.crc, len, lsh) ^ crc);
    }
    if (s.size) crc = shift_bytes_tab(crc ^ s.crc, s.size, rsh);
    out[i] = crc;
}

// Split one long buffer into `k` pieces of `piece` bytes (the last one
// shorter) for the batch kernel (photon_crc32c_extend_device).
__global__ void crc32c_split_kernel(const uint8_t* data, uint64_t nbytes, uint64_t piece, uint64_t k,
                                    photon_crc_iovec* iov) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k) return;
    const uint64_t off = i * piece;
    iov[i].base = data + off;
    iov[i].len = i + 1 < k ? piece : nbytes - off;
}

// out = (out * x^(8*last_len) ^ last_crc) ^ seed * x^(8*nbytes): append the
// last piece to the folded equal pieces and apply crc32c_extend's seed.
__global__ void crc32c_extend_finish_kernel(uint32_t* out, const uint32_t* last_crc, uint64_t last_len,
                                            uint32_t seed, uint64_t nbytes, PowTable pt) {
    uint32_t c = shift_bytes_tab(*out, last_len, pt) ^ *last_crc;
    *out = c ^ shift_bytes_tab(seed, nbytes, pt);
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void fill_splitmix_kernel(uint8_t* base, uint64_t stride, uint64_t nbytes, uint64_t count,
                                     uint64_t seed_base) {
    const uint64_t wpb = (nbytes + 7) / 8;
    const uint64_t total = wpb * count;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t b = g / wpb, k = g - b * wpb;
        const uint64_t w = mix64(seed_base + b + (k + 1) * 0x9E3779B97F4A7C15ull);
        uint8_t* dst = base + b * stride + k * 8;
        const uint64_t m = nbytes - k * 8 < 8 ? nbytes - k * 8 : 8;
        if (m == 8 && (reinterpret_cast<uintptr_t>(dst) & 7) == 0) {
            *reinterpret_cast<uint64_t*>(dst) = w;
        } else {
            for (uint64_t j = 0; j < m; ++j) dst[j] = (uint8_t)(w >> (8 * j));
        }
    }
}

// Read-only HBM stream (bench reference for the achievable read roofline):
// every 16-byte word read once with the same nontemporal dwordx4 loads as the
// CRC kernels, XOR-folded so nothing is dead code.
__global__ __launch_bounds__(256) void read_stream_kernel(const uint8_t* p, uint64_t nvec, uint32_t* sink) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    uint64_t i = tid;
    for (; i + 7 * nth < nvec; i += 8 * nth) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = load16(p + 16 * (i + k * nth));
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    for (; i < nvec; i += nth) {
        const uint4 v = load16(p + 16 * i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    sink[tid] = acc;
}

// ============================================================ CRC-64/ECMA
// Same column algorithm at 64 bits (reference crc64ecma_sw, crc.cpp:119-122:
// reflected poly 0xC96C5795D7870F42, register inverted in and out). 64-bit
// table entries are read with ds_read_b64; LDS holds
//   D64: x -> x * x^64 mod P, 8 byte slices x 256 x 4 replicas x 8 B = 64 KiB
//   S64: P -> P * x^(8*16*G),  same shape                            = 64 KiB
//   lane-combine bases x^(128*2^k), k < 6: 6 x 64 x 8 B              =  3 KiB
constexpr uint32_t k64SBase = 65536u;
constexpr uint32_t k64BasisBase = 131072u;
constexpr uint32_t k64LdsBytes = k64BasisBase + 6u * 64u * 8u;

struct LaneConsts64 {
    uint64_t kshift;           // x^(8*16*G) mod P64
    uint64_t basis[6][64];     // basis of x^(128 * 2^k)
};

struct Batch64Args {
    const uint8_t* base;
    uint64_t stride;
    uint64_t nbytes;
    const photon_crc_iovec* iov;
    uint64_t count;
    const uint64_t* seeds;
    uint64_t* out;
    uint64_t seed0;
};

__device__ __forceinline__ uint64_t lds_dword(const uint64_t* lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

// Slice t of table base `tb` (layout [slice][idx][lane%4], 8-byte entries).
template <int T>
__device__ __forceinline__ uint64_t look64(const uint64_t* lds, uint64_t x, uint32_t tb) {
    const uint32_t idx = (uint32_t)(x >> (8 * T)) & 0xffu;
    return lds_dword(lds, tb + T * 8192u + idx * 32u);
}

__device__ __forceinline__ uint64_t step64(const uint64_t* lds, uint64_t x, uint32_t tb) {
    return look64<0>(lds, x, tb) ^ look64<1>(lds, x, tb) ^ look64<2>(lds, x, tb) ^ look64<3>(lds, x, tb) ^
           look64<4>(lds, x, tb) ^ look64<5>(lds, x, tb) ^ look64<6>(lds, x, tb) ^ look64<7>(lds, x, tb);
}

__device__ __forceinline__ uint64_t bytestep64(const uint64_t* lds, uint64_t c, uint8_t b, uint32_t db) {
    // D64 slice 7: (b << 56) * x^64 = b * x^8, the classic byte table.
    return look64<7>(lds, (uint64_t)((c ^ b) & 0xffu) << 56, db) ^ (c >> 8);
}

__device__ __forceinline__ uint64_t mul_basis64(uint64_t p, const uint64_t* basis) {
    uint64_t r = 0;
#pragma unroll 4
    for (int i = 0; i < 64; ++i) r ^= (0ull - ((p >> i) & 1ull)) & basis[i];
    return r;
}

// Words at byte offset `off` of the first 16-byte blocks: zero the bytes
// before the data start s0, XOR the (already inverted) 64-bit init into data
// bytes s0..s0+7.
__device__ __forceinline__ uint64_t head_word64(uint64_t w, int off, int s0, uint64_t init) {
    const int k = s0 - off;
    if (k >= 8) return 0ull;
    if (k > 0) w &= ~0ull << (8 * k);
    if (k >= 0) w ^= init << (8 * k);
    else if (k > -8) w ^= init >> (8 * -k);
    return w;
}

template <int G>
__global__ __launch_bounds__(kBlock) void crc64_batch_kernel(Batch64Args args, LaneConsts64 kc) {
    __shared__ __attribute__((aligned(16))) uint64_t lds[k64LdsBytes / 8];
    {
        // 1024 threads: thread -> (slice t, index b); 2048 entries per table.
        const uint32_t tid = threadIdx.x;
        for (uint32_t e = tid; e < 2048u; e += kBlock) {
            const uint32_t t = e >> 8, b = e & 255u;
            const uint64_t v = (uint64_t)b << (8 * t);
            const uint64_t dv = mulmod64(v, kPoly64 /* x^64 mod P64 = the reflected polynomial */);
            const uint64_t sv = mulmod64(v, kc.kshift);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                lds[(t * 8192u + b * 32u + r * 8u) / 8] = dv;
                lds[(k64SBase + t * 8192u + b * 32u + r * 8u) / 8] = sv;
            }
        }
        if (tid < 6 * 64) lds[k64BasisBase / 8 + tid] = kc.basis[tid >> 6][tid & 63];
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gl = lane & (G - 1);
    const uint32_t grp = lane / G;
    constexpr int GPW = 64 / G;
    constexpr int LOG2G = G == 64 ? 6 : G == 32 ? 5 : G == 16 ? 4 : G == 8 ? 3 : 2;
    const uint32_t db = (lane & 3u) * 8u;            // D64 base for this lane's replica
    const uint32_t sb = k64SBase + (lane & 3u) * 8u;  // S64 base
    const uint64_t* basis = lds + k64BasisBase / 8;

    const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
    for (uint64_t wv = (uint64_t)blockIdx.x * kWaves + wave_id(); wv * GPW < args.count; wv += nwaves) {
        const uint64_t bi = wv * GPW + grp;
        const bool active = bi < args.count;
        const uint8_t* p = nullptr;
        uint64_t n = 0, seed = args.seed0;
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
        const uint64_t init = ~seed;  // crc.cpp:119-122: register starts at ~crc
        uint64_t reg;
        if (n < 64) {
            reg = init;
            if (gl == 0)
                for (uint64_t k = 0; k < n; ++k) reg = bytestep64(lds, reg, load8(p + k), db);
        } else {
            const uint8_t* a0 = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(15));
            const uint8_t* e = p + n;
            const uint8_t* eb = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(e) & ~uintptr_t(15));
            const int s0 = (int)(p - a0);
            const uint64_t nb = (uint64_t)(eb - a0) >> 4;
            const uint64_t rows = (nb + G - 1) / G;
            const uint32_t rlast = (uint32_t)(nb - (rows - 1) * G);
            const uint8_t* lp = a0 + 16 * gl;
            uint64_t pc = 0;
            for (uint64_t row = 0; row < rows; row += 2) {
                uint4 w[2];
                bool have[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const uint64_t i = (row + u) * G + gl;
                    have[u] = row + u < rows && i < nb;
                    w[u] = have[u] ? load16(lp + (row + u) * (16 * G)) : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    if (!have[u]) continue;
                    uint64_t lo = ((uint64_t)w[u].y << 32) | w[u].x, hi = ((uint64_t)w[u].w << 32) | w[u].z;
                    if (row + u == 0 && gl < 2) {
                        lo = head_word64(lo, (int)gl * 16, s0, init);
                        hi = head_word64(hi, (int)gl * 16 + 8, s0, init);
                    }
                    const uint64_t c = step64(lds, step64(lds, lo, db) ^ hi, db);
                    pc = step64(lds, pc, sb) ^ c;
                }
            }
            const uint32_t d = (rlast + G - 1 - gl) & (G - 1);
#pragma unroll 1
            for (int k = 0; k < LOG2G; ++k)
                if ((d >> k) & 1u) pc = mul_basis64(pc, basis + 64 * k);
#pragma unroll
            for (int o = G / 2; o > 0; o >>= 1) {
                const uint32_t lo32 = (uint32_t)__shfl_xor((int)(uint32_t)pc, o, 64);
                const uint32_t hi32 = (uint32_t)__shfl_xor((int)(uint32_t)(pc >> 32), o, 64);
                pc ^= ((uint64_t)hi32 << 32) | lo32;
            }
            reg = pc;
            if (gl == 0)
                for (const uint8_t* q = eb; q < e; ++q) reg = bytestep64(lds, reg, load8(q), db);
        }
        if (active && gl == 0) args.out[bi] = ~reg;
    }
}

}  // namespace pcrc
