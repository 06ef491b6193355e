// crc32c_device.hip -- MI355X (gfx950) CRC32C engine behind the C-ABI of
// include/photon_crc/crc32c_gpu.h.
//
// What it computes: PhotonLibOS's raw CRC-32C, crc32c_extend(data, n, seed)
// (reference common/checksum/crc32c.h:30-33; engines crc.cpp:114-117,
// 339-368), for batches of independent device-resident buffers.
//
// How (DESIGN.md "Kernel"): a group of G lanes (G = 64: one wavefront per
// buffer; G < 64 packs 64/G small buffers per wavefront) walks the buffer in
// rows of G 16-byte blocks: lane l of the group loads block (row*G + l) with
// one coalesced global_load_dwordx4, so a row is one contiguous 16*G-byte
// sweep. Each lane keeps a partial CRC P over "its" column of blocks, as if
// the other lanes' bytes were zeros:
//     P <- P * x^(8*16*G) mod P  XOR  crc16(block)
// crc16(block) (the CRC of the 16 bytes alone) does not depend on P, so the
// U blocks a lane holds are reduced in parallel and only the cheap shift is
// on the loop-carried chain. All GF(2) products by constants are byte-sliced
// LDS table lookups (no carry-less multiply on CDNA4, no MFMA: this is GF(2)):
//   D tables: x -> x * x^32 mod P, 4 byte slices, replicated 32x so that lane
//             l always hits bank l%32 (conflict-free random lookups), 128 KiB;
//   S tables: P -> P * x^(8*16*G) mod P, 4 slices, 4 replicas, 16 KiB.
// At the end lane l multiplies its partial by x^(128*d_l), d_l = number of
// 16-byte blocks between its last block and the end (constant-basis GF(2)
// multiplies on the bits of d_l), and the group XOR-reduces with __shfl_xor.
// Unaligned heads use zero-prefix invariance (crc.md:24-32): the leading
// bytes of the first aligned block are masked to 0 and the seed is XORed into
// the first four data bytes (init-value linearity), so every load is an
// aligned 16-byte load. Ragged tails (<16 B) are finished byte-serially.
// Uniform batches (aligned, equal length, whole rows) take a streaming kernel
// whose load ring runs continuously across buffer boundaries.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

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

template <int G, int B, int U, int D>
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
                c[u] = run_crc<B>(lds, ring[d][u], la);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) pc = sstep(lds, pc, la.s) ^ c[u];
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

// ------------------------------------------------------------------ host side
namespace {

thread_local std::string g_err;
int g_lanes_override = 0;
int g_stream_b = 1, g_stream_u = 4, g_stream_d = 3;  // streaming kernel: run blocks, rows/step, steps in flight
bool g_stream_enabled = true;

int fail(int code, const std::string& what) {
    g_err = what;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(-EIO, std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceInfo {
    bool probed = false;
    bool ok = false;
    int cus = 0;
};

std::mutex g_mu;
std::vector<DeviceInfo> g_dev;

// Resolve the current device; only gfx950 is supported (no other code path).
int current_device(int* cus) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    std::lock_guard<std::mutex> lk(g_mu);
    if ((int)g_dev.size() <= dev) g_dev.resize(dev + 1);
    DeviceInfo& di = g_dev[dev];
    if (!di.probed) {
        hipDeviceProp_t prop;
        e = hipGetDeviceProperties(&prop, dev);
        if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
        di.ok = strncmp(prop.gcnArchName, "gfx950", 6) == 0;
        di.cus = prop.multiProcessorCount;
        di.probed = true;
        if (!di.ok) g_err = std::string("device is ") + prop.gcnArchName + ", need gfx950";
    }
    if (!di.ok) return fail(-ENODEV, "photon_crc: no gfx950 device (got other arch)");
    *cus = di.cus;
    return dev;
}

// Constants for G lanes per buffer and runs of B blocks per lane per row:
// row shift x^(8*16*B*G), lane-combine basis of x^(8*16*B*2^k).
LaneConsts make_lane_consts(int g, int b) {
    LaneConsts c;
    c.kshift = xpow(8ull * 16ull * (uint64_t)b * (uint64_t)g);
    for (int k = 0; k < 6; ++k) mul_basis(xpow((128ull * (uint64_t)b) << k), c.basis[k]);
    return c;
}

const LaneConsts& lane_consts(int g, int b = 1) {
    static LaneConsts tab[7][3];
    static std::once_flag once;
    std::call_once(once, [] {
        for (int lg = 2; lg <= 6; ++lg)
            for (int lb = 0; lb <= 2; ++lb) tab[lg][lb] = make_lane_consts(1 << lg, 1 << lb);
    });
    const int lg = g == 64 ? 6 : g == 32 ? 5 : g == 16 ? 4 : g == 8 ? 3 : 2;
    const int lb = b == 4 ? 2 : b == 2 ? 1 : 0;
    return tab[lg][lb];
}

const PowTable& pow_table() {
    static PowTable t;
    static std::once_flag once;
    std::call_once(once, [] {
        uint32_t v = xpow(8);  // x^8
        for (int i = 0; i < 64; ++i) {
            t.x8pow2[i] = v;
            v = mulmod(v, v);
        }
    });
    return t;
}

// Lanes per buffer: one wavefront per buffer for large buffers; pack small
// buffers so every lane still walks >= 16 rows (DESIGN.md "Lane groups").
int choose_lanes(uint64_t typical_len) {
    if (g_lanes_override) return g_lanes_override;
    // Measured with scripts/tune_gpu.py (profiles/tune_r01.md): 1 MiB buffers
    // G=64, 64 KiB G=32, 4-8 KiB G=8.
    if (typical_len >= (512u << 10)) return 64;
    if (typical_len >= (32u << 10)) return 32;
    if (typical_len >= 2048) return 8;
    return 4;
}

int launch_batch(const BatchArgs& a, uint64_t typical_len, hipStream_t stream) {
    if (a.count == 0) return 0;
    int cus = 0;
    int dev = current_device(&cus);
    if (dev < 0) return dev;
    const int g = choose_lanes(typical_len);
    const uint64_t gpw = 64 / g;
    const uint64_t waves = (a.count + gpw - 1) / gpw;
    uint64_t grid = (waves + kWaves - 1) / kWaves;
    if (grid > (uint64_t)cus) grid = cus;
    const LaneConsts& kc = lane_consts(g);
    switch (g) {
        case 64: hipLaunchKernelGGL(crc32c_batch_kernel<64>, dim3(grid), dim3(kBlock), 0, stream, a, kc); break;
        case 32: hipLaunchKernelGGL(crc32c_batch_kernel<32>, dim3(grid), dim3(kBlock), 0, stream, a, kc); break;
        case 16: hipLaunchKernelGGL(crc32c_batch_kernel<16>, dim3(grid), dim3(kBlock), 0, stream, a, kc); break;
        case 8: hipLaunchKernelGGL(crc32c_batch_kernel<8>, dim3(grid), dim3(kBlock), 0, stream, a, kc); break;
        default: hipLaunchKernelGGL(crc32c_batch_kernel<4>, dim3(grid), dim3(kBlock), 0, stream, a, kc); break;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "crc32c_batch_kernel launch");
    return 0;
}

SeedConsts seed_consts(uint64_t nbytes) {
    static std::mutex mu;
    static uint64_t cached_n = ~0ull;
    static SeedConsts cached;
    std::lock_guard<std::mutex> lk(mu);
    if (cached_n != nbytes) {
        mul_basis(xpow(8ull * nbytes), cached.basis);
        cached_n = nbytes;
    }
    return cached;
}

template <int G, int B, int U, int D>
void launch_uniform_t(const UniformArgs& a, dim3 grid, hipStream_t stream) {
    hipLaunchKernelGGL((crc32c_uniform_kernel<G, B, U, D>), grid, dim3(kBlock), 0, stream, a, lane_consts(G, B));
}

// The instantiated (B, U, D) shapes: ring registers (D+1)*U*B*4 <= 80 VGPRs.
template <int G>
bool launch_uniform_g(const UniformArgs& a, dim3 grid, hipStream_t stream) {
    const int b = g_stream_b, u = g_stream_u, d = g_stream_d;
    if (b == 2 && u == 2 && d == 3) launch_uniform_t<G, 2, 2, 3>(a, grid, stream);
    else if (b == 1 && u == 4 && d == 3) launch_uniform_t<G, 1, 4, 3>(a, grid, stream);
    else if (b == 4 && u == 1 && d == 3) launch_uniform_t<G, 4, 1, 3>(a, grid, stream);
    else if (b == 2 && u == 2 && d == 4) launch_uniform_t<G, 2, 2, 4>(a, grid, stream);
    else if (b == 4 && u == 1 && d == 4) launch_uniform_t<G, 4, 1, 4>(a, grid, stream);
    else if (b == 1 && u == 2 && d == 4) launch_uniform_t<G, 1, 2, 4>(a, grid, stream);
    else return false;
    return true;
}

bool stream_shape_ok(int b, int u, int d) {
    return (b == 2 && u == 2 && (d == 3 || d == 4)) || (b == 1 && ((u == 4 && d == 3) || (u == 2 && d == 4))) ||
           (b == 4 && u == 1 && (d == 3 || d == 4));
}

int try_launch_uniform(const uint8_t* base, uint64_t stride, uint64_t nbytes, uint64_t count, uint32_t seed0,
                       const uint32_t* seeds, uint32_t* out, hipStream_t stream) {
    if (!g_stream_enabled || count == 0) return 1;
    const int g = choose_lanes(nbytes);
    const uint64_t row = 16ull * g * (uint64_t)g_stream_b;
    if ((reinterpret_cast<uintptr_t>(base) & 15) || (stride & 15) || nbytes < row || nbytes % row) return 1;
    const uint64_t rows = nbytes / row;
    if (rows % (uint64_t)g_stream_u) return 1;
    int cus = 0;
    int dev = current_device(&cus);
    if (dev < 0) return dev;
    const uint64_t gpw = 64 / g;
    const uint64_t waves = (count + gpw - 1) / gpw;
    uint64_t grid = (waves + kWaves - 1) / kWaves;
    if (grid > (uint64_t)cus) grid = cus;
    UniformArgs a{base, stride, rows, count, out};
    bool ok = false;
    switch (g) {
        case 64: ok = launch_uniform_g<64>(a, dim3(grid), stream); break;
        case 32: ok = launch_uniform_g<32>(a, dim3(grid), stream); break;
        case 16: ok = launch_uniform_g<16>(a, dim3(grid), stream); break;
        case 8: ok = launch_uniform_g<8>(a, dim3(grid), stream); break;
        default: ok = launch_uniform_g<4>(a, dim3(grid), stream); break;
    }
    if (!ok) return fail(-EINVAL, "unsupported streaming configuration");
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "crc32c_uniform_kernel launch");
    if (seeds || seed0) {
        const int bs = 256;
        hipLaunchKernelGGL(crc32c_seed_kernel, dim3((count + bs - 1) / bs), dim3(bs), 0, stream, out, count, seeds,
                           seed0, seed_consts(nbytes));
        e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(e, "crc32c_seed_kernel launch");
    }
    return 0;
}

// Host-memory pipeline (photon_crc32c_host_batch_strided): per device, a copy
// stream and a compute stream, kNumStage device staging chunks. Chunk i is
// copied (H2D, 2-D so any host stride packs densely) while chunk i-1 is
// checksummed; events order reuse of a staging chunk after its kernel.
constexpr int kNumStage = 3;
constexpr uint64_t kStageBytes = 256ull << 20;

struct HostPipe {
    bool ready = false;
    hipStream_t copy = nullptr, comp = nullptr;
    void* stage[kNumStage] = {};
    hipEvent_t copied[kNumStage] = {}, consumed[kNumStage] = {};
    uint32_t* d_out = nullptr;
    uint32_t* d_seeds = nullptr;
    uint64_t out_cap = 0;
};

std::mutex g_pipe_mu;
std::vector<HostPipe> g_pipes;

int pipe_for(int dev, HostPipe** out) {
    if ((int)g_pipes.size() <= dev) g_pipes.resize(dev + 1);
    HostPipe& p = g_pipes[dev];
    if (!p.ready) {
        hipError_t e;
        if ((e = hipStreamCreateWithFlags(&p.copy, hipStreamNonBlocking)) != hipSuccess) return hip_fail(e, "stream");
        if ((e = hipStreamCreateWithFlags(&p.comp, hipStreamNonBlocking)) != hipSuccess) return hip_fail(e, "stream");
        for (int i = 0; i < kNumStage; ++i) {
            if ((e = hipMalloc(&p.stage[i], kStageBytes)) != hipSuccess) return hip_fail(e, "hipMalloc(stage)");
            if ((e = hipEventCreateWithFlags(&p.copied[i], hipEventDisableTiming)) != hipSuccess)
                return hip_fail(e, "event");
            if ((e = hipEventCreateWithFlags(&p.consumed[i], hipEventDisableTiming)) != hipSuccess)
                return hip_fail(e, "event");
        }
        p.ready = true;
    }
    *out = &p;
    return 0;
}

}  // namespace
}  // namespace pcrc

using namespace pcrc;

extern "C" {

int photon_crc_device_count(void) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
    int ok = 0;
    for (int d = 0; d < n; ++d) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) == hipSuccess && strncmp(prop.gcnArchName, "gfx950", 6) == 0) ++ok;
    }
    if (!ok) return fail(-ENODEV, "photon_crc: no gfx950 device");
    return ok;
}

const char* photon_crc_last_error(void) { return g_err.c_str(); }

int photon_crc_set_lanes_per_buffer(int g) {
    if (g != 0 && g != 4 && g != 8 && g != 16 && g != 32 && g != 64)
        return fail(-EINVAL, "lanes per buffer must be 0, 4, 8, 16, 32 or 64");
    g_lanes_override = g;
    return 0;
}

int photon_crc_set_stream_config(int run_blocks, int rows_per_step, int steps_in_flight) {
    if (run_blocks == 0) {
        g_stream_enabled = false;
        return 0;
    }
    if (!stream_shape_ok(run_blocks, rows_per_step, steps_in_flight))
        return fail(-EINVAL, "unsupported (run_blocks, rows_per_step, steps_in_flight)");
    g_stream_enabled = true;
    g_stream_b = run_blocks;
    g_stream_u = rows_per_step;
    g_stream_d = steps_in_flight;
    return 0;
}

int photon_crc32c_batch_strided(const void* d_base, uint64_t stride, uint64_t nbytes, uint64_t count,
                                uint32_t seed0, const uint32_t* d_seeds, uint32_t* d_out, void* stream) {
    if (count && (!d_out || (!d_base && nbytes))) return fail(-EINVAL, "null buffer or output");
    int rc = try_launch_uniform(static_cast<const uint8_t*>(d_base), stride, nbytes, count, seed0, d_seeds, d_out,
                                static_cast<hipStream_t>(stream));
    if (rc <= 0) return rc;
    BatchArgs a{};
    a.base = static_cast<const uint8_t*>(d_base);
    a.stride = stride;
    a.nbytes = nbytes;
    a.iov = nullptr;
    a.count = count;
    a.seeds = d_seeds;
    a.out = d_out;
    a.seed0 = seed0;
    return launch_batch(a, nbytes, static_cast<hipStream_t>(stream));
}

int photon_crc32c_batch_strided_sync(const void* d_base, uint64_t stride, uint64_t nbytes, uint64_t count,
                                     uint32_t seed0, const uint32_t* d_seeds, uint32_t* d_out, void* stream) {
    int rc = photon_crc32c_batch_strided(d_base, stride, nbytes, count, seed0, d_seeds, d_out, stream);
    if (rc) return rc;
    hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    return 0;
}

int photon_crc32c_host_batch_strided(const void* h_base, uint64_t stride, uint64_t nbytes, uint64_t count,
                                     uint32_t seed0, const uint32_t* h_seeds, uint32_t* h_out) {
    if (!count) return 0;
    if (!h_base || !h_out || stride < nbytes) return fail(-EINVAL, "bad arguments");
    const uint64_t pitch = (nbytes + 255) & ~uint64_t(255);
    if (pitch > kStageBytes) return fail(-EINVAL, "buffer larger than a staging chunk (256 MiB)");
    int cus = 0;
    int dev = current_device(&cus);
    if (dev < 0) return dev;
    std::lock_guard<std::mutex> lk(g_pipe_mu);
    HostPipe* p = nullptr;
    int rc = pipe_for(dev, &p);
    if (rc) return rc;
    hipError_t e;
    if (p->out_cap < count) {
        if (p->d_out) (void)hipFree(p->d_out);
        if (p->d_seeds) (void)hipFree(p->d_seeds);
        p->d_out = p->d_seeds = nullptr;
        p->out_cap = 0;
        if ((e = hipMalloc(&p->d_out, count * 4)) != hipSuccess) return hip_fail(e, "hipMalloc(out)");
        if ((e = hipMalloc(&p->d_seeds, count * 4)) != hipSuccess) return hip_fail(e, "hipMalloc(seeds)");
        p->out_cap = count;
    }
    if (h_seeds) {
        e = hipMemcpyAsync(p->d_seeds, h_seeds, count * 4, hipMemcpyHostToDevice, p->comp);
        if (e != hipSuccess) return hip_fail(e, "seeds H2D");
    }
    const uint64_t per_chunk = kStageBytes / pitch;
    const uint8_t* src = static_cast<const uint8_t*>(h_base);
    for (uint64_t first = 0, i = 0; first < count; first += per_chunk, ++i) {
        const int slot = (int)(i % kNumStage);
        const uint64_t k = count - first < per_chunk ? count - first : per_chunk;
        if ((e = hipStreamWaitEvent(p->copy, p->consumed[slot], 0)) != hipSuccess) return hip_fail(e, "wait");
        e = hipMemcpy2DAsync(p->stage[slot], pitch, src + first * stride, stride, nbytes, k, hipMemcpyHostToDevice,
                             p->copy);
        if (e != hipSuccess) return hip_fail(e, "hipMemcpy2DAsync H2D");
        if ((e = hipEventRecord(p->copied[slot], p->copy)) != hipSuccess) return hip_fail(e, "record");
        if ((e = hipStreamWaitEvent(p->comp, p->copied[slot], 0)) != hipSuccess) return hip_fail(e, "wait");
        rc = photon_crc32c_batch_strided(p->stage[slot], pitch, nbytes, k, seed0, h_seeds ? p->d_seeds + first : nullptr,
                                         p->d_out + first, p->comp);
        if (rc) return rc;
        if ((e = hipEventRecord(p->consumed[slot], p->comp)) != hipSuccess) return hip_fail(e, "record");
    }
    e = hipMemcpyAsync(h_out, p->d_out, count * 4, hipMemcpyDeviceToHost, p->comp);
    if (e != hipSuccess) return hip_fail(e, "out D2H");
    e = hipStreamSynchronize(p->comp);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    return 0;
}

int photon_crc32c_batch_iov(const photon_crc_iovec* d_iov, uint64_t count, uint32_t seed0,
                            const uint32_t* d_seeds, uint32_t* d_out, void* stream) {
    if (count && (!d_iov || !d_out)) return fail(-EINVAL, "null descriptor array or output");
    BatchArgs a{};
    a.iov = d_iov;
    a.count = count;
    a.seeds = d_seeds;
    a.out = d_out;
    a.seed0 = seed0;
    // Descriptors live on the device; lengths are unknown to the host, so the
    // lane-group size is the generic one unless overridden.
    return launch_batch(a, 65536, static_cast<hipStream_t>(stream));
}

int photon_crc32c_batch_msg(const photon_crc_iovec* d_iov, const uint64_t* d_msg_start, uint64_t nmsg,
                            uint32_t seed0, const uint32_t* d_seeds, uint32_t* d_seg_out, uint32_t* d_out,
                            void* stream) {
    if (!nmsg) return 0;
    if (!d_iov || !d_msg_start || !d_seg_out || !d_out) return fail(-EINVAL, "null argument");
    hipStream_t st = static_cast<hipStream_t>(stream);
    uint64_t nseg = 0;
    hipError_t e = hipMemcpyAsync(&nseg, d_msg_start + nmsg, sizeof(nseg), hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(msg_start)");
    e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    BatchArgs a{};
    a.iov = d_iov;
    a.count = nseg;
    a.out = d_seg_out;
    a.seed0 = 0;
    int rc = launch_batch(a, 8192, st);
    if (rc) return rc;
    const int bs = 256;
    hipLaunchKernelGGL(crc32c_msg_fold_kernel, dim3((nmsg + bs - 1) / bs), dim3(bs), 0, st, d_iov, d_msg_start,
                       nmsg, d_seg_out, seed0, d_seeds, d_out, pow_table());
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "crc32c_msg_fold_kernel launch");
    return 0;
}

int photon_crc32c_combine_batch(const uint32_t* d_crc1, const uint32_t* d_crc2, const uint32_t* d_len2,
                                uint64_t count, uint32_t* d_out, void* stream) {
    if (!count) return 0;
    if (!d_crc1 || !d_crc2 || !d_len2 || !d_out) return fail(-EINVAL, "null argument");
    int cus = 0;
    int dev = current_device(&cus);
    if (dev < 0) return dev;
    const int bs = 256;
    hipLaunchKernelGGL(crc32c_combine_kernel, dim3((count + bs - 1) / bs), dim3(bs), 0,
                       static_cast<hipStream_t>(stream), d_crc1, d_crc2, d_len2, count, d_out, pow_table());
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "crc32c_combine_kernel launch");
    return 0;
}

int photon_crc_util_read_stream(const void* d_base, uint64_t nbytes, uint32_t* d_sink, uint64_t sink_words,
                                void* stream) {
    if (!d_base || !d_sink || (reinterpret_cast<uintptr_t>(d_base) & 15)) return fail(-EINVAL, "bad arguments");
    int cus = 0;
    int dev = current_device(&cus);
    if (dev < 0) return dev;
    uint64_t grid = (uint64_t)cus * 8;
    if (grid * 256 > sink_words) grid = sink_words / 256;
    if (!grid) return fail(-EINVAL, "sink too small (need >= 256 words)");
    hipLaunchKernelGGL(read_stream_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<const uint8_t*>(d_base), nbytes / 16, d_sink);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "read_stream_kernel launch");
    return 0;
}

int photon_crc_util_fill_splitmix(void* d_base, uint64_t stride, uint64_t nbytes, uint64_t count,
                                  uint64_t seed_base, void* stream) {
    if (!count || !nbytes) return 0;
    if (!d_base) return fail(-EINVAL, "null buffer");
    int cus = 0;
    int dev = current_device(&cus);
    if (dev < 0) return dev;
    const uint64_t words = (nbytes + 7) / 8 * count;
    uint64_t grid = (words + 255) / 256;
    if (grid > (uint64_t)cus * 16) grid = (uint64_t)cus * 16;
    hipLaunchKernelGGL(fill_splitmix_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<uint8_t*>(d_base), stride, nbytes, count, seed_base);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "fill_splitmix_kernel launch");
    return 0;
}

}  // extern "C"
