// crc64_kernels.h -- device code of the CRC-64/ECMA engine:
// batch and streaming kernels, message fold, combine, trim and one-buffer
// fold. Shares the LDS helpers and lane-group conventions of crc32c_kernels.h.
#pragma once
#include "crc32c_kernels.h"

#ifndef PCRC64_U
#define PCRC64_U 2  // rows per step of the CRC-64 batch kernel (2 > 4 by 0.9 points on the C2 shape; A/B builds: -DPCRC64_U=4)
#endif
// 16-lane groups: the finish's second level lane-parallel (finish_xor16);
// A/B builds: -DPCRC64_FIN16=0 for the two dependent 16-lookup levels.
#ifndef PCRC64_FIN16
#define PCRC64_FIN16 1
#endif
// Aligned strided batches take the init at the end (Batch64Args::shift_init;
// A/B builds: -DPCRC64_SHIFT_INIT=0).
#ifndef PCRC64_SHIFT_INIT
#define PCRC64_SHIFT_INIT 1
#endif
// Bench-only ablation builds of buffer_reg64 (-DPCRC64_ABL=bits; results are
// then NOT CRCs): 1 = no head masking, 2 = no finish multiply, 4 = no group
// XOR, 8 = row shift replaced by an XOR (no S lookups), 16 = lagged block
// replaced by lo ^ hi (no D lookups). 0 in the product.
#ifndef PCRC64_ABL
#define PCRC64_ABL 0
#endif
// The generic batch kernel's row loop: 1 = reload each row's registers as it
// is consumed (no copies on the loop edge; C2 shape 0.850 vs 0.848
// frac_kernel over 3 alternating rounds, steady 0.8516 vs 0.8495 at the
// same J/GiB, repo:profiles/r06f_ab_roll64_c2.jsonl, r06f_power_roll64_*.jsonl),
// 0 = the next step into a second set and copied back (A/B builds).
#ifndef PCRC64_ROLL
#define PCRC64_ROLL 1
#endif
// Table steps: 0 = the value rotated per lane (2 v_perm) so that lookup i
// takes byte i, conflict-free; 1 = no rotation, lookup i takes byte
// (i + q) % 4 of half i / 4 through a per-lane selector (4 fewer v_perm per
// 16-byte block, 2-way bank conflicts: lanes l and l + 16 share a bank pair).
// 1 measured slower, the LDS array being near its limit: C3 shape 0.790 vs
// 0.805, C2 shape 0.806 vs 0.847 (repo:profiles/r06s_ab_crc64_half_local.jsonl).
#ifndef PCRC64_HALF
#define PCRC64_HALF 0
#endif
// Finish-table addresses (nib_mul64): 1 = nibble and position joined by an
// OR (2 VALU per lookup), 0 = shift, mask and add (3; A/B builds).
#ifndef PCRC64_NIB_OR
#define PCRC64_NIB_OR 1
#endif

namespace pcrc {

// ============================================================ CRC-64/ECMA
// Same column algorithm at 64 bits (reference crc64ecma_sw, crc.cpp:119-122:
// reflected poly 0xC96C5795D7870F42, register inverted in and out). Values
// are kept as two 32-bit halves (uint2: .x = low, .y = high); 64-bit table
// entries are read with ds_read_b64 (bank = (addr/4) mod 64, lane groups of
// 32 lanes, 2 banks per lane). LDS holds
//   D64: x -> x * x^64 mod P64, 8 byte slices x 256 x 4 replicas,
//        layout [idx][slice t][lane%4] (256 B per index)             64 KiB
//   S64: P -> P * x^(8*16*G), same layout, at +64 KiB                   64 KiB
//   batch kernel: finish tables A_dl / B_dh, nibble-sliced       16-30 KiB
//   streaming kernel: lane-combine tables x^(128*2^k), k < 6      12 KiB
// Conflict-free lookups with only 4 replicas: lane l takes its 8 slices in
// the rotated order t = (i + q) % 8, q = (l/4) % 8, so in every lookup
// instruction i the 32 lanes of a group hit 32 distinct (t, replica) bank
// pairs. The rotation is applied to the looked-up VALUE (two v_perm_b32 with
// per-lane selectors: byte i of x_rot = byte (i+q)%8 of x), so the address
// of lookup i is ONE v_perm_b32 {off_i.byte0, x_rot.byte i, 0 | off_i.byte2, 0}
// with off_i = ((i+q)%8)*32 + (l%4)*8 (+ 1<<16, selected for S).
constexpr uint32_t k64SBase = 65536u;
// Lane-combine tables R64_k: p -> p * x^(128*2^k), k < 6, NIBBLE-sliced
// (16 positions x 16 values x 8 B = 2 KiB per k): used once per buffer by the
// streaming kernel (the batch kernel uses the finish tables below).
constexpr uint32_t k64RBase = 131072u;
constexpr uint32_t k64LdsBytes = k64RBase + 6u * 16u * 16u * 8u;  // 143360 B
// Finish tables of the batch kernel (in place of R64_k): the lane's partial Q
// (= P * x^-64) times x^(64 + 128 d), d = 16-byte blocks after its last block,
// d < G, split d = 8 dh + dl:
//   A_dl: p -> p * x^(64 + 128 dl), dl < 8 (Q -> P and the low lane shift)
//   B_dh: p -> p * x^(1024 dh), 1 <= dh < G/8
// nibble-sliced, 2 KiB per table, layout [value v][position t] (entry at
// v*128 + t*8): lane l reads position t = (i + l) % 16 in lookup i, so a
// 32-lane half hits bank pair (v%2)*32 + 2t: at most 2-way conflicts. One (G
// <= 8) or two dependent 16-lookup levels instead of a D step plus log2(G)
// 16-lookup R64 levels (88 lookups at G = 32, 56 at G = 8).
constexpr uint32_t k64FBase = 131072u;
constexpr uint32_t k64FBBase = k64FBase + 8u * 2048u;
constexpr uint32_t k64FLdsBytes = k64FBBase + 7u * 2048u;  // 161792 B of the 163840

struct LaneConsts64 {
    uint64_t kshift;           // x^(8*16*G) mod P64
    uint64_t sbasis[64];       // basis of kshift (S64 entries by select-XOR)
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
    // Aligned strided batches without per-buffer seeds: buffers start at 16-B
    // boundaries, so nothing is masked, and the inverted init enters at the
    // end as (~seed0) * x^(8 nbytes) (linearity, crc.cpp:393-405) instead of
    // being XORed into every buffer's first words by two lanes per group.
    uint64_t init_shift;
    uint32_t shift_init;
};

__device__ __forceinline__ uint2 lds_u2(const uint32_t* lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

__device__ __forceinline__ uint2 xor2(uint2 a, uint2 b) { return make_uint2(a.x ^ b.x, a.y ^ b.y); }

struct LaneAddr64 {
    uint32_t rot_lo, rot_hi;   // v_perm selectors rotating a 64-bit value right by 8q bits
    uint32_t off[8];           // off_i = ((i+q)%8)*32 + (lane%4)*8 | 1<<16
    uint32_t r8;               // (lane%4)*8, for the byte-serial tail
    uint32_t hoff[4];          // PCRC64_HALF: b_j*32 + (lane%4)*8 | 1<<16, b_j = (j + q) % 4
    uint32_t hsel[2][4];       // PCRC64_HALF: {off.byte0, half.byte b_j, 0 | off.byte2, 0} (D | S)
};

__device__ __forceinline__ LaneAddr64 lane_addr64(uint32_t lane) {
    LaneAddr64 a;
    const uint32_t q = (lane >> 2) & 7u, r = lane & 3u;
    // perm(hi, lo, sel): source bytes 0-3 = lo, 4-7 = hi; result byte i = byte (i+q)%8.
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        lo |= ((i + q) & 7u) << (8 * i);
        hi |= ((i + 4 + q) & 7u) << (8 * i);
    }
    a.rot_lo = lo;
    a.rot_hi = hi;
#pragma unroll
    for (int i = 0; i < 8; ++i) a.off[i] = (((i + q) & 7u) << 5) | (r << 3) | (1u << 16);
    a.r8 = r << 3;
    if constexpr (PCRC64_HALF) {
        const uint32_t qh = (lane >> 2) & 3u;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t b = (j + qh) & 3u;
            a.hoff[j] = (b << 5) | (r << 3) | (1u << 16);
            a.hsel[0][j] = 0x0C0C0000u | ((4u + b) << 8);
            a.hsel[1][j] = 0x0C020000u | ((4u + b) << 8);
        }
    }
    return a;
}

__device__ __forceinline__ uint2 rot64(uint2 x, const LaneAddr64& a) {
    return make_uint2(__builtin_amdgcn_perm(x.y, x.x, a.rot_lo), __builtin_amdgcn_perm(x.y, x.x, a.rot_hi));
}

// Lookup i (0..7) of the rotated value's byte i; TS = 0 for D64, 1 for S64.
template <int I, int TS>
__device__ __forceinline__ uint2 look64(const uint32_t* lds, uint2 xr, const LaneAddr64& a) {
    const uint32_t half = I < 4 ? xr.x : xr.y;
    const uint32_t sel = (TS ? 0x0C020000u : 0x0C0C0000u) | ((4u + (I & 3)) << 8);
    return lds_u2(lds, __builtin_amdgcn_perm(half, a.off[I], sel));
}

// PCRC64_HALF: lookup i of the unrotated value, slice 4 (i / 4) + b_(i % 4)
// (the second half's slices at +128 B: the instruction's offset field).
template <int I, int TS>
__device__ __forceinline__ uint2 look64h(const uint32_t* lds, uint2 x, const LaneAddr64& a) {
    const uint32_t half = I < 4 ? x.x : x.y;
    return lds_u2(lds, __builtin_amdgcn_perm(half, a.hoff[I & 3], a.hsel[TS][I & 3]) + (I < 4 ? 0u : 128u));
}

// Table product of x (8 lookups) XORed with e: 4 v_bitop3 per half.
template <int TS>
__device__ __forceinline__ uint2 step64(const uint32_t* lds, uint2 x, const LaneAddr64& a, uint2 e) {
    if constexpr (PCRC64_HALF) {
        const uint2 l0 = look64h<0, TS>(lds, x, a), l1 = look64h<1, TS>(lds, x, a);
        const uint2 l2 = look64h<2, TS>(lds, x, a), l3 = look64h<3, TS>(lds, x, a);
        const uint2 l4 = look64h<4, TS>(lds, x, a), l5 = look64h<5, TS>(lds, x, a);
        const uint2 l6 = look64h<6, TS>(lds, x, a), l7 = look64h<7, TS>(lds, x, a);
        return make_uint2(xor3(xor3(l0.x, l1.x, l2.x), xor3(l3.x, l4.x, l5.x), xor3(l6.x, l7.x, e.x)),
                          xor3(xor3(l0.y, l1.y, l2.y), xor3(l3.y, l4.y, l5.y), xor3(l6.y, l7.y, e.y)));
    }
    const uint2 xr = rot64(x, a);
    const uint2 l0 = look64<0, TS>(lds, xr, a), l1 = look64<1, TS>(lds, xr, a);
    const uint2 l2 = look64<2, TS>(lds, xr, a), l3 = look64<3, TS>(lds, xr, a);
    const uint2 l4 = look64<4, TS>(lds, xr, a), l5 = look64<5, TS>(lds, xr, a);
    const uint2 l6 = look64<6, TS>(lds, xr, a), l7 = look64<7, TS>(lds, xr, a);
    return make_uint2(xor3(xor3(l0.x, l1.x, l2.x), xor3(l3.x, l4.x, l5.x), xor3(l6.x, l7.x, e.x)),
                      xor3(xor3(l0.y, l1.y, l2.y), xor3(l3.y, l4.y, l5.y), xor3(l6.y, l7.y, e.y)));
}

// x * x^64 mod P64 (^ e).
__device__ __forceinline__ uint2 dstep64(const uint32_t* lds, uint2 x, const LaneAddr64& a,
                                         uint2 e = make_uint2(0, 0)) {
    return step64<0>(lds, x, a, e);
}

// P * x^(8*16*G) mod P64 (^ e).
__device__ __forceinline__ uint2 sstep64(const uint32_t* lds, uint2 p, const LaneAddr64& a,
                                         uint2 e = make_uint2(0, 0)) {
    if constexpr ((PCRC64_ABL & 8) != 0) return make_uint2(p.y ^ e.x, p.x ^ e.y);
    return step64<1>(lds, p, a, e);
}

// Lagged block CRC: the CRC register (init 0) after a 16-byte block is
// crc16(w) = (lo * x^64 ^ hi) * x^64 = v * x^64 with v = D(lo) ^ hi. The
// column recurrence P <- P * X ^ crc16(w) (X = x^(128G)) is run on
// Q = P * x^-64 instead: Q <- Q * X ^ v, so each block costs one D step (8
// lookups) + one S step (8) instead of 24 lookups; P = D(Q) once per buffer.
__device__ __forceinline__ uint2 lag16_64(const uint32_t* lds, uint4 w, const LaneAddr64& a) {
    if constexpr ((PCRC64_ABL & 16) != 0) return make_uint2(w.x ^ w.z, w.y ^ w.w);
    return dstep64(lds, make_uint2(w.x, w.y), a, make_uint2(w.z, w.w));
}

__device__ __forceinline__ uint64_t u64of(uint2 v) { return ((uint64_t)v.y << 32) | v.x; }
__device__ __forceinline__ uint2 u2of(uint64_t v) { return make_uint2((uint32_t)v, (uint32_t)(v >> 32)); }

// Byte-serial step: D64 slice 7 = (b << 56) * x^64 = b * x^8, the classic byte table.
__device__ __forceinline__ uint64_t bytestep64(const uint32_t* lds, uint64_t c, uint8_t b, const LaneAddr64& a) {
    const uint2 t = lds_u2(lds, ((uint32_t)((c ^ b) & 0xffu) << 8) + 7u * 32u + a.r8);
    return u64of(t) ^ (c >> 8);
}

// p * x^(128*2^k) through the nibble tables R64_k (16 lookups).
__device__ __forceinline__ uint64_t mul_r64(uint64_t p, const uint32_t* lds, int k) {
    const char* R = reinterpret_cast<const char*>(lds) + k64RBase + k * 2048;
    uint2 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m)
        v[m] = *reinterpret_cast<const uint2*>(R + m * 128 + (((uint32_t)(p >> (4 * m)) & 15u) << 3));
    uint32_t lo = xor3(xor3(v[0].x, v[1].x, v[2].x), xor3(v[3].x, v[4].x, v[5].x), xor3(v[6].x, v[7].x, v[8].x));
    uint32_t hi = xor3(xor3(v[0].y, v[1].y, v[2].y), xor3(v[3].y, v[4].y, v[5].y), xor3(v[6].y, v[7].y, v[8].y));
    lo = xor3(lo, xor3(v[9].x, v[10].x, v[11].x), xor3(v[12].x, v[13].x, v[14].x)) ^ v[15].x;
    hi = xor3(hi, xor3(v[9].y, v[10].y, v[11].y), xor3(v[12].y, v[13].y, v[14].y)) ^ v[15].y;
    return ((uint64_t)hi << 32) | lo;
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

// Compile-time basis of x^64 mod P64 (= the reflected polynomial): D64
// entries by select-XOR of 8 words instead of a 64-step bit-serial multiply
// (which made the prologue ~15 us longer than CRC32C's per launch).
struct Basis64 {
    uint64_t w[64];
};
constexpr Basis64 make_basis64(uint64_t k) {
    Basis64 r{};
    for (int i = 0; i < 64; ++i) r.w[i] = mulmod64(1ull << i, k);
    return r;
}
__constant__ const Basis64 kBasisD64 = make_basis64(kPoly64);
static_assert(make_basis64(kPoly64).w[63] == kPoly64, "bit 63 is x^0: its image under x^64 is x^64 mod P64");
// Lane-combine multipliers x^(128*2^k), k < 6 (independent of G).
__constant__ const Basis64 kBasisR64[6] = {make_basis64(xpow64(128)),  make_basis64(xpow64(256)),
                                           make_basis64(xpow64(512)),  make_basis64(xpow64(1024)),
                                           make_basis64(xpow64(2048)), make_basis64(xpow64(4096))};

// Finish multipliers (A_dl, B_dh above).
__constant__ const Basis64 kBasisA64[8] = {
    make_basis64(xpow64(64)),       make_basis64(xpow64(64 + 128)),     make_basis64(xpow64(64 + 2 * 128)),
    make_basis64(xpow64(64 + 3 * 128)), make_basis64(xpow64(64 + 4 * 128)), make_basis64(xpow64(64 + 5 * 128)),
    make_basis64(xpow64(64 + 6 * 128)), make_basis64(xpow64(64 + 7 * 128))};
__constant__ const Basis64 kBasisB64[7] = {make_basis64(xpow64(1024)),     make_basis64(xpow64(2 * 1024)),
                                           make_basis64(xpow64(3 * 1024)), make_basis64(xpow64(4 * 1024)),
                                           make_basis64(xpow64(5 * 1024)), make_basis64(xpow64(6 * 1024)),
                                           make_basis64(xpow64(7 * 1024))};
static_assert(xpow64(64) == kPoly64, "x^64 mod P64 is the reflected polynomial");

template <typename B>
__device__ __forceinline__ uint64_t basis_entry64(const B& basis, uint32_t t, uint32_t b) {
    uint64_t r = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r ^= (0ull - ((b >> j) & 1u)) & basis[8 * t + j];
    return r;
}

// FIN = 0: R64_k lane-combine tables; FIN = G: the finish tables A_dl, B_dh.
template <int FIN = 0>
__device__ __forceinline__ void build_tables64(uint32_t* lds, const LaneConsts64& kc) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t e = tid; e < 2048u; e += kBlock) {
        const uint32_t t = e >> 8, b = e & 255u;  // t is uniform per wavefront
        const uint2 dv = u2of(basis_entry64(kBasisD64.w, t, b));
        const uint2 sv = u2of(basis_entry64(kc.sbasis, t, b));
        const uint32_t base = (b << 8) + (t << 5);
        // replica (i + e) % 4 in step i: the lanes (same t, rows 256 B apart)
        // spread over 4 bank pairs instead of one (crc32c_kernels.h build_tables)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t r = (i + e) & 3u;
            *reinterpret_cast<uint2*>(reinterpret_cast<char*>(lds) + base + r * 8) = dv;
            *reinterpret_cast<uint2*>(reinterpret_cast<char*>(lds) + k64SBase + base + r * 8) = sv;
        }
    }
    if constexpr (FIN == 0) {
        // R64_k[m][v] = (v << 4m) * x^(128*2^k): XOR of the basis words of v's bits.
        for (uint32_t e = tid; e < 6u * 256u; e += kBlock) {
            const uint32_t k = e >> 8, m = (e >> 4) & 15u, v = e & 15u;
            uint64_t r = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) r ^= (0ull - ((v >> j) & 1u)) & kBasisR64[k].w[4 * m + j];
            *reinterpret_cast<uint2*>(reinterpret_cast<char*>(lds) + k64RBase + e * 8u) = u2of(r);
        }
    } else {
        // Table k < 8: A_k; 8 <= k < 7 + FIN/8: B_(k-7). Entry (v, t) = (v << 4t) * K.
        constexpr uint32_t ntab = 8u + (FIN > 8 ? FIN / 8 - 1 : 0);
        for (uint32_t e = tid; e < ntab * 256u; e += kBlock) {
            const uint32_t k = e >> 8, t = (e >> 4) & 15u, v = e & 15u;
            const uint64_t* w = k < 8 ? kBasisA64[k].w : kBasisB64[k - 8].w;
            uint64_t r = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) r ^= (0ull - ((v >> j) & 1u)) & w[4 * t + j];
            *reinterpret_cast<uint2*>(reinterpret_cast<char*>(lds) + k64FBase + k * 2048u + v * 128u + t * 8u) =
                u2of(r);
        }
    }
    __syncthreads();
}

// The CRC-64 prologue from a per-device image (crc32c_kernels.h load_tables):
// the bytes build_tables64<G> writes (D, S, the finish tables of G), copied.
static __device__ const uint32_t* g_table_image64[5];
template <int G>
constexpr uint32_t lds64_used() {
    return k64FBase + (8u + (G > 8 ? G / 8 - 1 : 0)) * 2048u;
}
template <int G>
__device__ __forceinline__ void load_tables64(uint32_t* lds, const LaneConsts64& kc) {
    const uint32_t* img = PCRC_TABLE_BUILD ? nullptr : g_table_image64[table_slot<G>()];
    if (img)
        copy_tables<lds64_used<G>()>(lds, img);
    else
        build_tables64<G>(lds, kc);
}
template <int G>
__global__ __launch_bounds__(kBlock) void table_image64_kernel(LaneConsts64 kc, uint32_t* img) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[k64FLdsBytes / 4];
    build_tables64<G>(lds, kc);
    for (uint32_t j = threadIdx.x; j < lds64_used<G>() / 16; j += kBlock)
        *reinterpret_cast<u32x4*>(img + 4 * j) = *reinterpret_cast<const u32x4*>(lds + 4 * j);
}

// p * x^(128*d) for d < 2^LOG2 (basis multiplies on the bits of d).
template <int LOG2>
__device__ __forceinline__ uint64_t shift64(uint64_t pc, uint32_t d, const uint32_t* lds) {
#pragma unroll
    for (int k = 0; k < LOG2; ++k) {
        const uint64_t m = mul_r64(pc, lds, k);
        pc = ((d >> k) & 1u) ? m : pc;  // every lane runs every level: no divergence
    }
    return pc;
}

// x * K through one nibble-sliced finish table at byte offset `base` (16
// lookups; lane l reads position (i + l) % 16 in lookup i).
__device__ __forceinline__ uint64_t nib_mul64(uint64_t x, const uint32_t* lds, uint32_t base, uint32_t lane) {
    const uint32_t r = lane & 15u;
    const uint32_t sh = 4u * r;
    const uint64_t xr = (x >> sh) | (x << ((64u - sh) & 63u));  // nibble i of xr = nibble (i + r) % 16 of x
    uint2 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t half = i < 8 ? (uint32_t)xr : (uint32_t)(xr >> 32);
#if PCRC64_NIB_OR
        // base is a multiple of 2 KiB and the position offset < 128: the
        // nibble goes to bits 7-10 by one shift and (sh & 0x780) | pos in one
        // v_bitop3 (truth table 0xEA), instead of shift, mask and add
        const uint32_t sh = 4 * (i & 7) >= 7 ? half >> (4 * (i & 7) - 7) : half << (7 - 4 * (i & 7));
        v[i] = lds_u2(lds, __builtin_amdgcn_bitop3_b32(sh, 0x780u, base + (((uint32_t)i + r) & 15u) * 8u, 0xEA));
#else
        const uint32_t nib = (half >> (4 * (i & 7))) & 15u;
        v[i] = lds_u2(lds, base + nib * 128u + (((uint32_t)i + r) & 15u) * 8u);
#endif
    }
    uint32_t lo = xor3(xor3(v[0].x, v[1].x, v[2].x), xor3(v[3].x, v[4].x, v[5].x), xor3(v[6].x, v[7].x, v[8].x));
    uint32_t hi = xor3(xor3(v[0].y, v[1].y, v[2].y), xor3(v[3].y, v[4].y, v[5].y), xor3(v[6].y, v[7].y, v[8].y));
    lo = xor3(lo, xor3(v[9].x, v[10].x, v[11].x), xor3(v[12].x, v[13].x, v[14].x)) ^ v[15].x;
    hi = xor3(hi, xor3(v[9].y, v[10].y, v[11].y), xor3(v[12].y, v[13].y, v[14].y)) ^ v[15].y;
    return ((uint64_t)hi << 32) | lo;
}

// Q * x^(64 + 128 d), d < G (the finish tables; every lane runs every level).
template <int G>
__device__ __forceinline__ uint64_t finish64(uint2 q, uint32_t d, const uint32_t* lds, uint32_t lane) {
    uint64_t x = nib_mul64(u64of(q), lds, k64FBase + (d & 7u) * 2048u, lane);
    if constexpr (G > 8) {
        const uint32_t dh = d >> 3;
        const uint64_t y = nib_mul64(x, lds, k64FBBase + (dh ? dh - 1u : 0u) * 2048u, lane);
        x = dh ? y : x;
    }
    return x;
}

__device__ __forceinline__ uint64_t group_xor64_16(uint64_t v) {
    return ((uint64_t)group_xor<16>((uint32_t)(v >> 32)) << 32) | group_xor<16>((uint32_t)v);
}

// finish64<16> and the group XOR in one, with the second level lane-parallel:
// lanes with d < 8 keep Q * A_d; the lanes with d >= 8 first XOR their Q *
// A_(d-8) (= U), and U * x^1024 = XOR over positions t of B_1[t][nibble t of
// U] is looked up ONE position per lane (lane gl takes position gl) and XORed
// across the group: 16 + 1 lookups per lane instead of 16 + 16 dependent.
__device__ __forceinline__ uint64_t finish_xor16(uint2 q, uint32_t d, const uint32_t* lds, uint32_t gl,
                                                 uint32_t lane) {
    const uint64_t x = nib_mul64(u64of(q), lds, k64FBase + (d & 7u) * 2048u, lane);
    const bool hi = d >= 8u;
    const uint64_t lo_sum = group_xor64_16(hi ? 0ull : x);
    const uint64_t u = group_xor64_16(hi ? x : 0ull);
    const uint64_t b = u64of(lds_u2(lds, k64FBBase + (((uint32_t)(u >> (4u * gl))) & 15u) * 128u + gl * 8u));
    return lo_sum ^ group_xor64_16(b);
}

// The raw CRC-64 register after the bytes [p, p+n) from `init` (a group of
// G lanes; valid on the group's first lane; crc64ecma_extend = ~reg with
// init = ~crc, crc.cpp:119-122).
template <int G>
__device__ __forceinline__ uint64_t buffer_reg64(const uint32_t* lds, const uint8_t* p, uint64_t n, uint64_t init,
                                                 uint32_t gl, uint32_t lane, const LaneAddr64& la,
                                                 bool head = true) {
    constexpr int U = PCRC64_U;
    uint64_t reg;
    if (n < 64) {
        reg = init;
        if (gl == 0)
            for (uint64_t k = 0; k < n; ++k) reg = bytestep64(lds, reg, load8(p + k), la);
    } else {
        const uint8_t* a0 = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(15));
        const uint8_t* e = p + n;
        const uint8_t* eb = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(e) & ~uintptr_t(15));
        const int s0 = (int)(p - a0);
        const uint64_t nb = (uint64_t)(eb - a0) >> 4;
        const uint64_t full = nb / G;
        const uint64_t rows = (nb + G - 1) / G;
        const uint32_t rlast = (uint32_t)(nb - (rows - 1) * G);
        const uint8_t* lp = a0 + 16 * gl;
        uint2 pc = make_uint2(0, 0);
        // Row 0, the lead rows ((full-1) % U, so the U-row loop ends at the
        // last full row), the first step's U rows and the partial last row
        // are issued together: no row is loaded on its own and waited for.
        const uint32_t lead = full >= 1 ? (uint32_t)((full - 1) % U) : 0u;
        uint4 w0, wl[U - 1], cur[U], wp;
        if (gl < nb) w0 = load16(lp);
#pragma unroll
        for (int u = 0; u < U - 1; ++u)
            if ((uint32_t)u < lead) wl[u] = load16(lp + (1 + u) * (16 * G));
        const bool steps = 1 + lead + U <= full;
        if (steps) {
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = load16(lp + (1 + lead + u) * (16 * G));
        }
        const bool part = full >= 1 && full < rows && full * G + gl < nb;
        if (part) wp = load16(lp + full * (16 * G));
        // Row 0 (head: masked leading bytes + inverted init).
        if (gl < nb) {
            uint4 w = w0;
            if (head && !(PCRC64_ABL & 1) && gl < 2) {  // head == false: aligned, init 0
                const uint64_t lo = head_word64(((uint64_t)w.y << 32) | w.x, (int)gl * 16, s0, init);
                const uint64_t hi = head_word64(((uint64_t)w.w << 32) | w.z, (int)gl * 16 + 8, s0, init);
                w = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
            }
            pc = lag16_64(lds, w, la);
        }
#pragma unroll
        for (int u = 0; u < U - 1; ++u)
            if ((uint32_t)u < lead) pc = sstep64(lds, pc, la, lag16_64(lds, wl[u], la));
        uint64_t row = 1 + lead;
        // U lagged blocks (independent) then U row shifts (the carried chain).
        auto column_step = [&](const uint4(&w)[U]) {
            uint2 c[U];
#pragma unroll
            for (int u = 0; u < U; ++u) c[u] = lag16_64(lds, w[u], la);
#pragma unroll
            for (int u = 0; u < U; ++u) pc = sstep64(lds, pc, la, c[u]);
        };
        if (steps) {
            for (; row + 2 * U <= full; row += U) {
                if constexpr (PCRC64_ROLL) {
                    // each row's registers reloaded as soon as its lagged
                    // block is taken: no copies on the loop edge
                    uint2 c[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        c[u] = lag16_64(lds, cur[u], la);
                        cur[u] = load16(lp + (row + U + u) * (16 * G));
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) pc = sstep64(lds, pc, la, c[u]);
                } else {
                    uint4 nxt[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) nxt[u] = load16(lp + (row + U + u) * (16 * G));
                    column_step(cur);
#pragma unroll
                    for (int u = 0; u < U; ++u) cur[u] = nxt[u];
                }
            }
            column_step(cur);
        }
        if (part) pc = sstep64(lds, pc, la, lag16_64(lds, wp, la));
        // Q * x^(64 + 128 d) (Q -> P and the shift to the end of the blocks), XOR over the group.
        const uint32_t d = (rlast + G - 1 - gl) & (G - 1);
        if constexpr (G == 16 && PCRC64_FIN16 && !(PCRC64_ABL & 6)) {
            reg = finish_xor16(pc, d, lds, gl, lane);
        } else {
            const uint64_t f = (PCRC64_ABL & 2) ? u64of(pc) : finish64<G>(pc, d, lds, lane);
            reg = (PCRC64_ABL & 4) ? f : ((uint64_t)group_xor<G>((uint32_t)(f >> 32)) << 32) | group_xor<G>((uint32_t)f);
        }
        if (gl == 0)
            for (const uint8_t* q = eb; q < e; ++q) reg = bytestep64(lds, reg, load8(q), la);
    }
    return reg;
}

// Per-wave s_memrealtime stamps of the bench-only probe builds (probes.hip;
// the product passes nullptr and STAMP = false): 8 words per wave.
__device__ __forceinline__ void stamp64_write(uint64_t* t, const uint64_t (&v)[5]) {
    if ((threadIdx.x & 63u) == 0) {
        uint64_t* o = t + 8 * ((uint64_t)blockIdx.x * kWaves + wave_id());
#pragma unroll
        for (int i = 0; i < 5; ++i) o[i] = v[i];
        o[5] = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_ID
        o[6] = __builtin_amdgcn_s_getreg(20 | (3 << 11));   // XCC_ID
        o[7] = 0;
    }
}

// Any pointer / length / seed (iovec batches, ragged and unaligned buffers).
// STAMP (probe builds): t0, tables built, first buffer done, loop done, end.
template <int G, bool STAMP = false>
__device__ __forceinline__ void crc64_batch_run(const Batch64Args& args, const LaneConsts64& kc, uint32_t* lds,
                                                uint64_t* t) {
    uint64_t ts[5] = {0, 0, 0, 0, 0};
    if constexpr (STAMP) ts[0] = __builtin_amdgcn_s_memrealtime();
    load_tables64<G>(lds, kc);
    if constexpr (STAMP) ts[1] = __builtin_amdgcn_s_memrealtime();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gl = lane & (G - 1);
    const uint32_t grp = lane / G;
    constexpr int GPW = 64 / G;
    const LaneAddr64 la = lane_addr64(lane);

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
        // crc.cpp:119-122: the register starts at ~crc and the result is inverted
        const uint64_t reg = args.shift_init ? buffer_reg64<G>(lds, p, n, 0ull, gl, lane, la, false) ^ args.init_shift
                                             : buffer_reg64<G>(lds, p, n, ~seed, gl, lane, la);
        if (active && gl == 0) args.out[bi] = ~reg;
        if constexpr (STAMP) {
            if (ts[2] == 0) ts[2] = __builtin_amdgcn_s_memrealtime();
        }
    }
    if constexpr (STAMP) {
        ts[3] = __builtin_amdgcn_s_memrealtime();
        ts[4] = ts[3];
        stamp64_write(t, ts);
    }
}

template <int G>
__global__ __launch_bounds__(kBlock) void crc64_batch_kernel(Batch64Args args, LaneConsts64 kc) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[k64FLdsBytes / 4];
    crc64_batch_run<G>(args, kc, lds, nullptr);
}

// ------------------------------------------------ full-row uniform batches
// Strided batches whose buffers are made of whole steps: base and stride
// 16-byte aligned, nbytes a multiple of 2 * 16 G U (an even number of U-row
// steps), one seed for all (its inverted init enters at the end, shift_init).
// Every lane has a block in every row, so nothing in the loop depends on the
// lane: the trip counts are wave-uniform (scalar loop control, no exec-mask
// loops), every load is unconditional and the compiler counts vmcnt exactly.
// Two register sets in turn (no copies on the loop edge, round 4's body
// copied U rows every step): the next step's U rows are issued before the
// current step's lookups, one step in flight as in the generic kernel.
// XB: the next buffer's first step is issued before this buffer's last step
// (the last buffer of a wave re-reads its own first step there: one step of
// extra reads per wave and launch, so that no load sits behind a branch)
// and finish (the lane-group finish runs with loads in flight instead of none).
// The first step of a buffer starts from Q = 0, so its first row needs no
// row shift (the generic kernel shifted 0 through the S tables). Lane gl's
// last block is G - 1 - gl blocks before the end of every buffer: its finish
// factor x^(64 + 128 (G - 1 - gl)) is fixed per lane.
// Reference semantics: crc64ecma_sw (crc.cpp:119-122, 511-669).
template <int G, int U, bool FIRST>
__device__ __forceinline__ uint2 column_step64(const uint32_t* lds, uint2 pc, const uint4 (&w)[U],
                                               const LaneAddr64& la) {
    uint2 c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) c[u] = lag16_64(lds, w[u], la);
    if constexpr (FIRST) {
        pc = c[0];
#pragma unroll
        for (int u = 1; u < U; ++u) pc = sstep64(lds, pc, la, c[u]);
    } else {
#pragma unroll
        for (int u = 0; u < U; ++u) pc = sstep64(lds, pc, la, c[u]);
    }
    return pc;
}

template <int G, int U>
__device__ __forceinline__ void load_step64(uint4 (&w)[U], const uint8_t* p) {
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = load16(p + u * (16 * G));
}

template <int G, int U, bool XB>
__global__ __launch_bounds__(kBlock) void crc64_full_kernel(Batch64Args args, LaneConsts64 kc) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[k64FLdsBytes / 4];
    load_tables64<G>(lds, kc);
    constexpr int GPW = 64 / G;
    constexpr uint32_t kStep = 16u * G * U;  // bytes of one step of a lane group
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gl = lane & (G - 1);
    const uint32_t grp = lane / G;
    const LaneAddr64 la = lane_addr64(lane);
    const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
    const uint32_t steps = __builtin_amdgcn_readfirstlane((uint32_t)(args.nbytes / kStep));  // even, >= 2
    const uint32_t d = G - 1 - gl;
    uint64_t wv = (uint64_t)blockIdx.x * kWaves + wave_id();
    if (wv * GPW >= args.count) return;
    // This lane's first block of wave-iteration w's buffer (a group past the
    // end of the batch re-reads the last buffer; its result is not stored).
    auto lane_ptr = [&](uint64_t w) {
        const uint64_t bi = w * GPW + grp;
        return args.base + (bi < args.count ? bi : args.count - 1) * args.stride + 16u * gl;
    };
    uint4 a[U], b[U];
    const uint8_t* p = lane_ptr(wv);
    load_step64<G, U>(a, p);
    for (;;) {
        const uint64_t next = wv + nwaves;
        const bool more = next * GPW < args.count;  // wave-uniform
        const uint8_t* pn = more ? lane_ptr(next) : p;
        uint2 pc;
        // steps 0 and 1 (peeled: step 0 starts from Q = 0)
        load_step64<G, U>(b, p + kStep);
        pc = column_step64<G, U, true>(lds, make_uint2(0, 0), a, la);
        if constexpr (XB) {  // unconditional (a select of the address): vmcnt stays exact
            load_step64<G, U>(a, steps > 2 ? p + 2 * kStep : pn);
        } else if (steps > 2) {
            load_step64<G, U>(a, p + 2 * kStep);
        }
        pc = column_step64<G, U, false>(lds, pc, b, la);
        for (uint32_t s = 2; s < steps; s += 2) {
            load_step64<G, U>(b, p + (uint64_t)(s + 1) * kStep);
            pc = column_step64<G, U, false>(lds, pc, a, la);
            if constexpr (XB) {
                load_step64<G, U>(a, s + 2 < steps ? p + (uint64_t)(s + 2) * kStep : pn);
            } else if (s + 2 < steps) {
                load_step64<G, U>(a, p + (uint64_t)(s + 2) * kStep);
            }
            pc = column_step64<G, U, false>(lds, pc, b, la);
        }
        // Q * x^(64 + 128 d) (Q -> P and the lane's shift to the end), XOR over the group.
        uint64_t reg;
        if constexpr (G == 16 && PCRC64_FIN16 && !(PCRC64_ABL & 6)) {
            reg = finish_xor16(pc, d, lds, gl, lane);
        } else {
            const uint64_t f = (PCRC64_ABL & 2) ? u64of(pc) : finish64<G>(pc, d, lds, lane);
            reg = (PCRC64_ABL & 4) ? f
                                   : ((uint64_t)group_xor<G>((uint32_t)(f >> 32)) << 32) | group_xor<G>((uint32_t)f);
        }
        const uint64_t bi = wv * GPW + grp;
        if (gl == 0 && bi < args.count) args.out[bi] = ~(reg ^ args.init_shift);  // crc.cpp:119-122
        if (!more) break;
        if (!XB) load_step64<G, U>(a, pn);
        wv = next;
        p = pn;
    }
}

// ---------------------------------------------- CRC-64 combine / fold / extend
// crc64ecma_combine(c1, c2, len2) = c1 ? c2 ^ c1 * x^(8*len2) : c2
// (crc.cpp crc64ecma_combine_sw: the inverted-CRC combine is linear). A
// message's CRC chained over its segments (crc64ecma_extend, seg after seg)
// is therefore acc = seed; acc = acc * x^(8*len_s) ^ crc64ecma(seg_s, 0).
struct PowTable64 {
    uint64_t x8pow2[64];  // x^(8 * 2^i) mod P64
};

constexpr uint64_t kOne64 = 1ull << 63;

__device__ __forceinline__ uint64_t xpow8_tab64(uint64_t n, const PowTable64& t) {
    uint64_t k = kOne64;
    for (int i = 0; n; ++i, n >>= 1)
        if (n & 1) k = mulmod64(k, t.x8pow2[i]);
    return k;
}

__global__ void crc64_combine_kernel(const uint64_t* c1, const uint64_t* c2, const uint32_t* l2, uint64_t n,
                                     uint64_t* out, PowTable64 pt) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = c1[i], b = c2[i];
    out[i] = a ? b ^ mulmod64(a, xpow8_tab64(l2[i], pt)) : b;
}

// crc64ecma_trim per element (do_crc_trim, crc.cpp:442-456, with
// T = CRC64ECMA_Component): 64-bit size check; shifts by the 32-bit lengths
// crc_apply_shifts takes; combine's crc1 == 0 shortcut.
__global__ void crc64_trim_kernel(const photon_crc64_component* all, const photon_crc64_component* pre,
                                  const photon_crc64_component* suf, uint64_t n, uint64_t* out, uint32_t* nerr,
                                  PowTable64 lsh, PowTable64 rsh) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const photon_crc64_component a = all[i], p = pre[i], s = suf[i];
    if (a.size < p.size + s.size) {
        out[i] = 0;
        if (nerr) atomicAdd(nerr, 1u);
        return;
    }
    uint64_t crc = a.crc;
    if (p.size && p.crc) crc ^= mulmod64(p.crc, xpow8_tab64((uint32_t)(a.size - p.size), lsh));
    if (s.size) crc = mulmod64(crc ^ s.crc, xpow8_tab64((uint32_t)s.size, rsh));
    out[i] = crc;
}

// One thread per message (as crc32c_msg_fold_kernel).
__global__ void crc64_msg_fold_kernel(const photon_crc_iovec* iov, const uint64_t* msg_start, uint64_t nmsg,
                                      const uint64_t* seg_crc, uint64_t seed0, const uint64_t* seeds,
                                      uint64_t* out, PowTable64 pt) {
    const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= nmsg) return;
    const uint64_t s0 = msg_start[m], s1 = msg_start[m + 1];
    uint64_t acc = seeds ? seeds[m] : seed0;
    uint64_t klen = 0, k = kOne64;
    for (uint64_t s = s0; s < s1; s += 4) {
        uint64_t len[4], c[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (s + j < s1) {
                len[j] = iov[s + j].len;
                c[j] = seg_crc[s + j];
            }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (s + j < s1) {
                if (len[j] != klen) {
                    k = xpow8_tab64(len[j], pt);
                    klen = len[j];
                }
                acc = mulmod64(acc, k) ^ c[j];
            }
    }
    out[m] = acc;
}

// photon_crc64ecma_extend_device in one launch: crc32c_long_kernel's scheme
// (crc32c_kernels.h "one long buffer": the same cut and slots, Horner per
// lane group with a lane-parallel multiply by X^S, the wave / workgroup
// factors applied in stages, workgroups XOR-reduced by long_reduce) on the
// raw CRC-64 register: the head starts from ~seed, body chunks from 0, the
// result is inverted (crc.cpp:119-122). A 64-bit lane-parallel multiply
// takes 64 basis words: one per lane of a wave, or two per lane of a 32-lane
// group. Round 3 applied each group's own factor after the chunk loop with
// two dependent 64-step bit-serial multiplies per wave.
struct Long64Args {
    const uint8_t* data;
    uint64_t head, chunk;
    int64_t nchunks;
    uint64_t last;
    int64_t lead;
    uint64_t stride;
    uint32_t rounds;
    uint64_t seed;
    uint64_t* out;
    uint64_t* acc;      // long_reduce state (8 + 8 * kLongMaxGrid bytes; grid > 1 only)
    uint64_t tbase;     // long_reduce: the state's ticket count before this launch
    uint32_t treset;    // long_reduce: put the ticket back to 0 (a leased state)
    uint64_t x;         // X (its basis words are computed on the device, G = 32 only)
    uint64_t xsb[64];   // basis words of X^S: (1 << i) * X^S (host-computed, long_powers)
    uint64_t zt[16];    // Z^(15 - w)
    uint64_t ft[kLongMaxFt];  // J Y^(grid - 1 - b)
    uint32_t out_tag;   // routed calls: nonzero = the result as two tagged words in pinned memory (long_reduce)
};

__device__ __forceinline__ uint64_t mulx64(uint64_t v) { return (v >> 1) ^ ((0ull - (v & 1ull)) & kPoly64); }

__device__ __forceinline__ uint64_t xor_lanes64(uint64_t v, int width) {
    const uint32_t lo = width == 64 ? group_xor<64>((uint32_t)v) : group_xor<32>((uint32_t)v);
    const uint32_t hi = width == 64 ? group_xor<64>((uint32_t)(v >> 32)) : group_xor<32>((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// The same basis word from the D64 tables in LDS (after build_tables64):
// c * x^k with k = 63 - i = 8a + b. Bit part: c * x^b = (c >> b) ^ T[(c <<
// (8 - b)) & 0xff] with T = slice 7 (v * x^8: the b bits shifted out are a
// byte shifted out 8 - b positions early). Byte part: c1 * x^(8a) = (c1 >>
// 8a) ^ XOR_(j < a) byte_j(c1) * x^(8 (a - j)), slice 8 - (a - j) holding v *
// x^(8 (a - j)) (slice t = (v << 8t) * x^64). 8 lookups and ~30 VALU instead
// of 63 dependent select steps (4-12 us of every launch's prologue at 64- /
// 32-lane groups, repo:profiles/r04_probe_long_vs_batch64.jsonl). Lanes
// whose a <= j look up entry 0 (= 0) of some slice.
__device__ __forceinline__ uint64_t basis_word64_lds(const uint32_t* lds, uint64_t c, uint32_t i, uint32_t r8) {
    const uint32_t k = 63u - i, b = k & 7u, a = k >> 3;
    const uint32_t y = (uint32_t)(c << (8u - b)) & 0xffu;
    const uint64_t v = (c >> b) ^ u64of(lds_u2(lds, (y << 8) + (7u << 5) + r8));
    uint64_t r = v >> (8u * a);
#pragma unroll
    for (uint32_t j = 0; j < 7; ++j) {
        const uint32_t byte = j < a ? (uint32_t)(v >> (8u * j)) & 0xffu : 0u;
        r ^= u64of(lds_u2(lds, (byte << 8) + (((8u + j - a) & 7u) << 5) + r8));
    }
    return r;
}

// v * c for a v held by every lane of a wave, lane l holding basis word l of c.
__device__ __forceinline__ uint64_t mul_wave64(uint64_t v, uint64_t bw, uint32_t lane) {
    return xor_lanes64(((v >> lane) & 1ull) ? bw : 0ull, 64);
}

// STAMP (probe builds): t0, tables built, basis words done, rounds done, end.
template <int G, bool STAMP = false>
__device__ __forceinline__ void crc64_long_run(const Long64Args& a, const LaneConsts64& kc, uint32_t* lds,
                                               uint64_t* red, uint64_t* t) {
    uint64_t ts[5] = {0, 0, 0, 0, 0};
    if constexpr (STAMP) ts[0] = __builtin_amdgcn_s_memrealtime();
    load_tables64<G>(lds, kc);
    if constexpr (STAMP) ts[1] = __builtin_amdgcn_s_memrealtime();
    constexpr int GPW = 64 / G;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = wave_id();
    const uint32_t gl = lane & (G - 1), grp = lane / G;
    const LaneAddr64 la = lane_addr64(lane);
    const int64_t S = (int64_t)a.stride;
    const int64_t g = ((int64_t)blockIdx.x * kWaves + wave) * GPW + grp;
    // Basis words of X^S from the host: 64 lanes one each (G = 64), or two
    // per lane of a 32-lane half (bits l and l + 32). Nothing but the chunk
    // loop's own work sits in the loop (crc32c_kernels.h long_run).
    const uint32_t l = G == 64 ? lane : (lane & 31u);
    const uint64_t bw0 = a.xsb[l], bw1 = G == 64 ? 0ull : a.xsb[l + 32];
    auto mul_group = [&](uint64_t v, uint64_t b0, uint64_t b1) {
        uint64_t term = ((v >> l) & 1ull) ? b0 : 0ull;
        if (G != 64) term ^= ((v >> (l + 32)) & 1ull) ? b1 : 0ull;
        return xor_lanes64(term, G == 64 ? 64 : 32);
    };
    // The wave's and (wave 0) the workgroup's factor: basis words computed
    // here, one per lane, before any chunk; X's for the 32-lane form.
    const uint64_t bw_z = basis_word64_lds(lds, a.zt[wave], lane, la.r8);
    const uint64_t bw_f = wave == 0 ? basis_word64_lds(lds, a.ft[blockIdx.x], lane, la.r8) : 0ull;
    const uint64_t bx0 = G == 32 ? basis_word64_lds(lds, a.x, l, la.r8) : 0ull;
    const uint64_t bx1 = G == 32 ? basis_word64_lds(lds, a.x, l + 32, la.r8) : 0ull;
    // Complete them here: left to the scheduler, their LDS lookups were
    // spread into the round loop and slowed it (1 GiB, 32 lanes: 0.192 vs
    // 0.169 ms with this barrier, repo:profiles/r04f_ab_long_basis_lds.jsonl).
    asm volatile("" ::"v"(bw_z), "v"(bw_f), "v"(bx0), "v"(bx1));
    if constexpr (STAMP) ts[2] = __builtin_amdgcn_s_memrealtime();
    uint64_t acc = 0, lastc = 0;  // uniform across the group (reg and the lane XOR are)
    for (int r = long_first_round(a); r < (int)a.rounds; ++r) {
        const int64_t v = g + (int64_t)r * S;
        const uint8_t* p;
        uint64_t n;
        bool last, head;  // the head carries the (inverted) seed
        long_slot(a, v, &p, &n, &last, &head);
        uint64_t reg = 0;
        if (__ballot(n != 0 || head)) {
            reg = buffer_reg64<G>(lds, p, n, head ? ~a.seed : 0ull, gl, lane, la);  // valid on gl == 0
            reg = __shfl(reg, lane & ~(uint32_t)(G - 1), 64);                        // the whole group
        }
        const uint64_t m = mul_group(acc, bw0, bw1);
        acc = last ? m : m ^ reg;
        lastc = last ? reg : lastc;
    }
    if constexpr (STAMP) ts[3] = __builtin_amdgcn_s_memrealtime();
    uint64_t v = acc;
    if constexpr (G == 32) {  // acc_0 * X ^ acc_1
        const uint64_t m = mul_group(acc, bx0, bx1);
        v = lane < 32 ? m : acc;
        v ^= ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), 32, 64) << 32) |
             (uint32_t)__shfl_xor((int)(uint32_t)v, 32, 64);
        lastc ^= ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(lastc >> 32), 32, 64) << 32) |
                 (uint32_t)__shfl_xor((int)(uint32_t)lastc, 32, 64);
    }
    v = mul_wave64(v, bw_z, lane);  // * Z^(15 - w)
    if (lane == 0) {
        red[wave] = v;
        red[kWaves + wave] = lastc;
    }
    __syncthreads();
    if (wave == 0) {
        uint64_t u = 0, e = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            u ^= red[w];
            e ^= red[kWaves + w];
        }
        u = mul_wave64(u, bw_f, lane) ^ e;  // * J Y^(grid - 1 - b), then the last chunk
        long_reduce(u, a.acc, a.out, [](uint64_t x) { return ~x; }, a.tbase, a.treset,
                    a.out_tag);  // crc.cpp:119-122: inverted out
    }
    if constexpr (STAMP) {
        ts[4] = __builtin_amdgcn_s_memrealtime();
        stamp64_write(t, ts);
    }
}

template <int G>
__global__ __launch_bounds__(kBlock) void crc64_long_kernel(Long64Args a, LaneConsts64 kc) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[k64FLdsBytes / 4];
    __shared__ uint64_t red[2 * kWaves];
    crc64_long_run<G>(a, kc, lds, red, nullptr);
}

// photon_crc64ecma_extend_device for buffers whose 16-byte block span is at
// most kSmallBlocks (256 KiB): crc32c_kernels.h crc32c_small_kernel's layout
// (up to kSmallWg = 33 workgroups x 256 threads = V = 8448 virtual lanes walking rows of
// V blocks anchored at the end, every factor a constant of the layout, tables
// copied from a device image) at 64 bits: a block's lagged value is lo * x^64
// ^ hi (ONE nibble-sliced multiply), Q <- Q * x^(128 V) ^ v per row, then
// Q * x^(64 + 128 dl), x^(1024 dh) (d = 63 - lane), the wave's
// x^(8192 (127 - wave)) and x^(-8k) lane-parallel (basis words from the
// image), long_reduce over the workgroups. The inverted init is XORed into
// the data's first 8 bytes (the grid covers them even for n < 8: with the
// x^(-8k) undo it contributes init * x^(8n), crc.cpp:119-122). Nibble tables:
// 16 positions x 16 values x 8 B per multiplier (2 KiB); in lookup t all 64
// lanes read position t's 16 entries: 128 contiguous bytes, no conflicts.
// The reference times crc64ecma on 128 KiB at buf+1 (test_checksum.cpp:204-216).
constexpr uint32_t kNib64 = 2048;
// The mid layout at 64 bits: the same 8 rows (16 MiB) as CRC-32C.
constexpr uint32_t kMid64Rows = kMidRows, kMid64Blocks = kMid64Rows * kMidLanes;
constexpr uint32_t kSm64D = 0, kSm64S = kNib64, kSm64A = 2 * kNib64, kSm64B = kSm64A + 8 * kNib64;
constexpr uint32_t kSm64S2 = kSm64B + 7 * kNib64;                       // the mid layout's row shift
constexpr uint32_t kSm64Lds = kSm64S2 + kNib64;                         // 36 KiB of tables in LDS
constexpr uint32_t kSm64Wave = kSm64Lds;  // 4 kMidWg x 64 words: x^(8192 d), d = waves after this one
constexpr uint32_t kSm64Tail = kSm64Wave + 4u * kMidWg * 64u * 8u;      // 32 x 64 words: x^(-8 k), k < 32
constexpr uint32_t kSm64Image = kSm64Tail + 32u * 64u * 8u;

struct Small64Args {
    const uint8_t* a0;       // aligned start (data start & ~15)
    const uint64_t* image;
    uint64_t* out;           // the CRC (device), through long_reduce when grid > 1
    uint64_t* acc;           // long_reduce state
    uint64_t tbase;
    uint32_t treset;
    uint32_t nb;             // blocks of the grid, <= kSmallBlocks + 1
    uint32_t s0;             // data start - a0
    uint32_t eoff;           // data end - a0
    uint32_t k;              // grid end - data end: the register is multiplied by x^(-8k)
    uint32_t wg0;            // workgroup index of blockIdx.x == 0
    uint64_t init;           // ~seed (the register's start, crc.cpp:119-122)
    uint64_t* slots;         // routed calls: workgroup b's raw value as {tag, low word}, {tag, high word}
    uint32_t tag;            //   at slots[2b], slots[2b + 1] (system scope; the host spins on the tags)
};

// p * K through the [position][value] nibble tables of K at byte offset `off`.
__device__ __forceinline__ uint64_t nib_mul64_pos(const uint32_t* lds, uint32_t off, uint64_t p) {
    uint2 v[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) v[t] = lds_u2(lds, off + (uint32_t)(t * 16 + (int)((p >> (4 * t)) & 15u)) * 8u);
    uint32_t lo = xor3(xor3(v[0].x, v[1].x, v[2].x), xor3(v[3].x, v[4].x, v[5].x), xor3(v[6].x, v[7].x, v[8].x));
    uint32_t hi = xor3(xor3(v[0].y, v[1].y, v[2].y), xor3(v[3].y, v[4].y, v[5].y), xor3(v[6].y, v[7].y, v[8].y));
    lo = xor3(lo, xor3(v[9].x, v[10].x, v[11].x), xor3(v[12].x, v[13].x, v[14].x)) ^ v[15].x;
    hi = xor3(hi, xor3(v[9].y, v[10].y, v[11].y), xor3(v[12].y, v[13].y, v[14].y)) ^ v[15].y;
    return ((uint64_t)hi << 32) | lo;
}

// Bytes of the 8-byte word at `off` (from a0) at or past `eoff` zeroed.
__device__ __forceinline__ uint64_t tail_word64(uint64_t w, int off, int eoff) {
    const int m = eoff - off;
    return m >= 8 ? w : m <= 0 ? 0ull : w & ((1ull << (8 * m)) - 1ull);
}

// Steps 2-3 of one workgroup's share (blocks w[] loaded for virtual lane vt):
// the column, the shift to the end of the wave, the wave's factor, the XOR
// over the 4 waves and the tail factor; the value on wave 0, one barrier.
template <uint32_t V, int R>
__device__ __forceinline__ uint64_t small64_value(const Small64Args& a, const uint32_t* lds, const uint4 (&w)[R],
                                                  uint32_t vt, uint64_t bw_wave, uint64_t bw_tail, uint64_t* red) {
    const uint32_t lane = threadIdx.x & 63u, wave = wave_id();
    const uint32_t rows = __builtin_amdgcn_readfirstlane((a.nb + V - 1) / V);
    const int first = (int)a.nb - (int)(rows * V) + (int)vt;
    // 2. The column: lagged blocks and the row shift (rows that do not exist
    //    cost nothing: crc32c_kernels.h small_wave_value).
    uint64_t c[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        c[r] = 0;
        if ((uint32_t)r >= rows) continue;
        const int b = first + r * (int)V;
        uint64_t lo = ((uint64_t)w[r].y << 32) | w[r].x, hi = ((uint64_t)w[r].w << 32) | w[r].z;
        if (b <= 1 || b >= (int)a.nb - 2) {  // the head's and the tail's blocks: masks + init
            const int off = b * 16;
            lo = head_word64(tail_word64(lo, off, (int)a.eoff), off, (int)a.s0, a.init);
            hi = head_word64(tail_word64(hi, off + 8, (int)a.eoff), off + 8, (int)a.s0, a.init);
            if (b < 0) lo = hi = 0ull;
        }
        c[r] = nib_mul64_pos(lds, kSm64D, lo) ^ hi;
    }
    uint64_t q = c[0];
#pragma unroll
    for (int r = 1; r < R; ++r)
        if ((uint32_t)r < rows) q = nib_mul64_pos(lds, V == kSmallLanes ? kSm64S : kSm64S2, q) ^ c[r];
    // 3. Q -> P and the shift to the end of the wave, the wave's and the tail's factors.
    const uint32_t d = 63u - lane, dh = d >> 3;
    const uint64_t x = nib_mul64_pos(lds, kSm64A + (d & 7u) * kNib64, q);
    const uint64_t y = nib_mul64_pos(lds, kSm64B + (dh ? dh - 1u : 0u) * kNib64, x);
    uint64_t v = xor_lanes64(dh ? y : x, 64);
    v = mul_wave64(v, bw_wave, lane);
    if (lane == 0) red[wave] = v;
    __syncthreads();
    uint64_t u = 0;
    if (wave == 0) {
        u = red[0] ^ red[1] ^ red[2] ^ red[3];
        u = mul_wave64(u, bw_tail, lane);
    }
    return u;
}

template <uint32_t V, int R>  // the small or the mid layout (crc32c_small_kernel)
__global__ __launch_bounds__(256) void crc64_small_kernel(Small64Args a) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kSm64Lds / 4];
    __shared__ uint64_t red[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const uint32_t wg = a.wg0 + blockIdx.x;
    const uint32_t vt = wg * 256u + tid;
    // 1. Table copy first, then the payload rows, then the basis words.
    constexpr uint32_t kVec = kSm64Lds / 16;  // 2304 16-byte pieces: 9 per thread
    constexpr uint32_t kPer = (kVec + 255) / 256;
    u32x4 tv[kPer];
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) {
        const uint32_t j = i * 256u + tid;
        tv[i] = j < kVec ? *((const g_u32x4*)a.image + j) : u32x4{0, 0, 0, 0};
    }
    uint4 w[R];
    small_load<false, V>(a, vt, w);  // as crc32c_small_kernel: only blocks that overlap the data
    const uint64_t bw_wave = a.image[kSm64Wave / 8 + (V / 64u - 1u - (wg * 4u + wave)) * 64u + lane];
    const uint64_t bw_tail = a.image[kSm64Tail / 8 + a.k * 64u + lane];
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) {
        const uint32_t j = i * 256u + tid;
        if (j < kVec) *reinterpret_cast<u32x4*>(lds + 4 * j) = tv[i];
    }
    lds_barrier();
    const uint64_t u = small64_value<V, R>(a, lds, w, vt, bw_wave, bw_tail, red);
    if (wave == 0) {
        if (a.slots) {  // routed: the host XORs the workgroups' raw values and inverts
            if (lane == 0) {
                __hip_atomic_store(a.slots + 2 * blockIdx.x, (uint64_t)a.tag << 32 | (uint32_t)u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(a.slots + 2 * blockIdx.x + 1, (uint64_t)a.tag << 32 | (uint32_t)(u >> 32),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        } else {
            long_reduce(u, a.acc, a.out, [](uint64_t x) { return ~x; }, a.tbase, a.treset, a.tag);  // crc.cpp:119-122
        }
    }
}

// The resident small-buffer service for routed crc64ecma_extend calls
// (crc32c_kernels.h crc32c_small_service_kernel, the same doorbell and poll
// loop): the CRC-64 tables (34 KiB) stay in LDS, a workgroup's raw value goes
// to its slot as {seq, low}, {seq, high}; the host XORs and inverts. The
// request's seed words carry the inverted init.
__global__ __launch_bounds__(256) void crc64_small_service_kernel(ServiceArgs s) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kSm64Lds / 4];
    __shared__ uint32_t cmd[2][8];
    __shared__ uint64_t red[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const uint32_t wg = blockIdx.x, vt = wg * 256u + tid;
    const uint64_t* image = static_cast<const uint64_t*>(s.image);
    for (uint32_t j = tid; j < kSm64Lds / 16; j += 256u)
        *reinterpret_cast<u32x4*>(lds + 4 * j) = *((const g_u32x4*)image + j);
    const uint64_t bw_wave = image[kSm64Wave / 8 + (4u * kSmallWg - 1u - (wg * 4u + wave)) * 64u + lane];
    __syncthreads();
    service_loop(s, cmd, nullptr, [&](const SvcReq& r) {
        Small64Args a{};
        a.a0 = r.a0;
        a.nb = r.nb;
        a.s0 = r.s0;
        a.k = r.k;
        a.eoff = r.eoff;
        a.init = r.seed;
        const uint64_t bw_tail = image[kSm64Tail / 8 + a.k * 64u + lane];  // L2-resident: 16 KiB for all k
        uint64_t u;
        if (a.nb > kSmallRows * kSmallLanes) {  // uniform: a call of up to kSvcRows rows
            uint4 w[kSvcRows];
            small_load<true, kSmallLanes>(a, vt, w);
            u = small64_value<kSmallLanes, kSvcRows>(a, lds, w, vt, bw_wave, bw_tail, red);
        } else {
            uint4 w[kSmallRows];
            small_load<true, kSmallLanes>(a, vt, w);
            u = small64_value<kSmallLanes, kSmallRows>(a, lds, w, vt, bw_wave, bw_tail, red);
        }
        if (wave == 0 && lane < 2)
            __hip_atomic_store(s.area + kSvcSlots + kSvcSlotStride * wg + lane,
                               (uint64_t)r.seq << 32 | (uint32_t)(lane ? u >> 32 : u), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    });
}

}  // namespace pcrc
