// crc32c_kernels.h -- device code of the MI355X CRC32C engine (see the
// overview at the top of crc32c_device.hip and DESIGN.md "Kernels"). Included
// by crc32c_device.hip (the product) and probes.hip (bench-only ablations).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/photon_crc/crc32c_gpu.h"
#include "gf2.h"

#ifndef PCRC_LANE_SEL
#define PCRC_LANE_SEL 1  // per-lane v_perm selectors instead of rotating the word (+0.3 % on C2)
#endif
#ifndef PCRC_LONG_LEAD
#define PCRC_LONG_LEAD true  // long kernels: lead rows + partial row preloaded (A/B: false)
#endif
#ifndef PCRC_LONG_MERGE_HEAD
#define PCRC_LONG_MERGE_HEAD 1  // long kernels: the head read with body chunk 0 (A/B: 0)
#endif
#ifndef PCRC_BATCH_LEAD
#define PCRC_BATCH_LEAD false  // the same in the buffer batch (A/B: true)
#endif
// ... for the batch kernel's 2-row steps only (C3: 16 lanes, 16 rows per lane,
// so row 15 was loaded on its own and waited for): 0.8578 vs 0.8567 in 3 of
// 3 rounds; with 4-row steps (C2) it measured 0.2 points lower in the
// driver's window, C4 +-0 (repo:profiles/r06p_ab_*_lead*.jsonl).
#ifndef PCRC_BATCH_LEAD2
#define PCRC_BATCH_LEAD2 true
#endif
#ifndef PCRC_MSG_LEAD
#define PCRC_MSG_LEAD 0  // A/B builds: 1 = lead rows preloaded in the message kernels (C5 -0.2, repo:profiles/r06p_ab_c5_msg_lead.jsonl)
#endif
// buf_body's row loop (A/B variants): 0 = one register set
// copied cur <- nxt on the loop edge (the default); 1 = the compiler's unroll
// by two (no copies; the next step's loads issued before this step's land:
// 8 rows in flight); 2 = two register sets by hand, the next step's loads
// issued only once this step's have landed (4 rows in flight, no copies);
// 3 = one register set reloaded row by row as each row is consumed.
#ifndef PCRC_BODY
#define PCRC_BODY 0
#endif
// With PCRC_BODY 0: steps of U >= 4 rows take variant 3's rolling reload
// (the C2 / C4 batch kernels and the long kernels; no v_mov copies on the
// loop edge): C2 in the driver's 5 + 20 launches 0.834 vs 0.826 frac_kernel
// over 5 alternating rounds, C4 +0.25 points, 1 GiB long kernel 0.170 vs
// 0.174 ms; at U = 2 (C3, messages) it cost 2 points, so U < 4 keeps the
// copies (repo:profiles/r06d_ab_roll_*.jsonl). A/B builds: -DPCRC_BODY_ROLL=0.
#ifndef PCRC_BODY_ROLL
#define PCRC_BODY_ROLL 1
#endif
// Aligned strided batches take the seed at the end (BatchArgs::shift_init;
// A/B builds: -DPCRC_SHIFT_INIT=0).
#ifndef PCRC_SHIFT_INIT
#define PCRC_SHIFT_INIT 1
#endif
#ifndef PCRC_SVC_STAMP
#define PCRC_SVC_STAMP 0  // bench-only builds: s_memrealtime stamps of each small-buffer service request
#endif

namespace pcrc {

// ------------------------------------------------------------------ LDS map
// One 256-byte row per table index idx:
//   [idx][  0..127]: D tables, x -> x * x^32 mod P, 4 byte slices t x 8 replicas
//   [idx][128..255]: S tables, P -> P * x^(8*16*G),  4 byte slices t x 8 replicas
// (entry (t, r) at t*32 + r*4). ds_read_b32 banks are (addr/4) mod 32 in lane
// groups of 32; lane l takes its 4 slices in the rotated order t = (i+q)%4,
// q = (l/8)%4, r = l%8, so in every lookup instruction the 32 lanes of a group
// hit 32 distinct banks: conflict-free random lookups with 8 replicas.
constexpr uint32_t kTableBytes = 256u * 256u;                // 64 KiB
constexpr uint32_t kSOff = 128u;                             // S half of a row
// Lane-combine tables R_k: p -> p * x^(128*B*2^k) mod P, k < 6, 4 byte slices,
// one replica ([k][t][idx]); used once per buffer (group_reduce).
constexpr uint32_t kRBase = kTableBytes;
constexpr uint32_t kRBytes = 6u * 4u * 256u * 4u;            // 24 KiB
constexpr uint32_t kLdsBytes = kRBase + kRBytes;             // 90112 B of the 160 KiB
// Finish tables F_d (batch kernel, G <= 8, in place of R_k): p -> p * x^(32 +
// 128*d) mod P for d < G, i.e. Q -> P and the lane's shift to the end of the
// buffer (d = 16-byte blocks after its last block) in ONE 4-lookup step.
// Index row b (256 B stride, 128 B used): word d*4 + t (G = 8) or
// (d*4 + t)*2 + r2 (G = 4, r2 = (lane/4)&1). In a lookup instruction the 8
// lanes of a group read 8 distinct d (d = const - gl mod G) and the groups
// of a 32-lane half read distinct slices t = (i + q) % 4 (q = lane/8 % 4;
// G = 4: two groups per q, told apart by r2): 32 distinct banks, no replicas.
constexpr uint32_t kFBase = kTableBytes;
constexpr uint32_t kLdsBytesF = kFBase + 65536u;             // 128 KiB
// Finish tables for G >= 16 (batch kernel, in place of R_k): d = 8*dh + dl,
//   A_dl: p -> p * x^(32 + 128*dl), dl < 8 (Q -> P and the low lane shift)
//   B_dh: p -> p * x^(1024*dh),     1 <= dh < G/8
// 4 byte slices, one replica, [table][t][idx] (4 KiB each): two dependent
// 4-lookup levels instead of a D step and log2(G) R_k levels (24 lookups in
// 6 dependent levels at G = 32).
constexpr uint32_t kABase = kTableBytes;
constexpr uint32_t kBBase = kABase + 8u * 4096u;
template <int G>
constexpr uint32_t lds_bytes_for() {
    return G <= 8 ? kLdsBytesF : kBBase + (uint32_t)(G / 8 - 1) * 4096u;  // 64: 124 KiB
}
constexpr int kBlock = 1024;                   // 16 waves, one workgroup per CU
constexpr int kWaves = kBlock / 64;

// Kernel constants computed on the host (gf2.h) per lanes-per-buffer G.
struct LaneConsts {
    uint32_t kshift;           // x^(8*16*G) mod P: one row of the lane's column
    uint32_t sbasis[32];       // basis of kshift (S table entries by select-XOR)
    uint32_t basis[6][32];     // basis of x^(128 * 2^k) mod P, k = 0..5
    uint32_t fbasis[8][32];    // basis of x^(32 + 128 * d) mod P, d < 8 (F_d tables)
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
    // Message mode (crc32c_batch_kernel<G, U, 1|2>): unit m = message m,
    // segments iov[msg_start[m] .. msg_start[m+1]); out[] = per-segment CRCs
    // (seed 0), msg_out[m] = the chained CRC from seed_m (seeds[m] or seed0).
    const uint64_t* msg_start;
    uint64_t nmsg;
    uint32_t* msg_out;
    // Aligned strided batches without per-buffer seeds (buffer mode only):
    // no head to mask, and the seed enters at the end as seed0 * x^(8 nbytes)
    // (linearity, crc.cpp:393-405) instead of through every lane's head words.
    uint32_t init_shift;
    uint32_t shift_init;
};

__device__ __forceinline__ uint32_t lds_word(const uint32_t* lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

// Per-lane lookup constants: the data word is rotated right by 8q bits
// (byte i of the rotated word = byte (i+q)%4), and off[i] = ((i+q)%4)*32 +
// r*4 locates slice (i+q)%4, replica r inside a table row.
struct LaneAddr {
    uint32_t rot;      // 8*q
    uint32_t off[4];
    uint32_t r4;       // r*4 (byte-serial tail)
    uint32_t sel[4];   // v_perm selector of lookup i: {off.byte0, x.byte((i+q)%4), 0, 0}
};

__device__ __forceinline__ uint32_t rot32(uint32_t x, const LaneAddr& a) {
    return __builtin_amdgcn_alignbit(x, x, a.rot);
}

// Lookup i of a rotated word: address (xr.byte i << 8) | off[i] in ONE
// v_perm_b32 (result bytes {off.byte0, xr.byte i, 0, 0}; selector 0..3 = the
// second operand's bytes, 4..7 = the first's, 12 = 0x00); TOFF selects the
// D (0) or S (kSOff) half of the row through the instruction's offset field.
// Bench-only energy ablations of the CRC32C lookups (-DPCRC_ABL=bits; results
// are then NOT CRCs): 1 = no LDS lookup (the v_perm'd address
// itself enters the XOR tree), 2 = no address v_perm (a per-lane fixed
// address made opaque to the compiler, still dependent on x, is read), 4 = no
// table prologue in the batch kernel, 8 = no segment-CRC stores in the
// message kernel, 16 = no fold there (acc = c). 0 in the product.
#ifndef PCRC_ABL
#define PCRC_ABL 0
#endif
#if PCRC_LANE_SEL
// Per-lane selectors: the v_perm of lookup i takes byte (i+q)%4 of the
// UNROTATED word (the selector is a per-lane register), so no v_alignbit per
// table step; one VALU per lookup either way.
template <int I, uint32_t TOFF>
__device__ __forceinline__ uint32_t look(const uint32_t* lds, uint32_t x, const LaneAddr& a) {
    if constexpr ((PCRC_ABL & 2) != 0) {
        uint32_t ad = a.off[I];
        asm volatile("" : "+v"(ad) : "v"(x));  // no instruction; keeps the read per step and its x dependence
        return lds_word(lds, ad + TOFF);
    }
    if constexpr ((PCRC_ABL & 1) != 0) return __builtin_amdgcn_perm(x, a.off[I], a.sel[I]) + TOFF;
    return lds_word(lds, __builtin_amdgcn_perm(x, a.off[I], a.sel[I]) + TOFF);
}
#else
template <int I, uint32_t TOFF>
__device__ __forceinline__ uint32_t look(const uint32_t* lds, uint32_t xr, const LaneAddr& a) {
    return lds_word(lds, __builtin_amdgcn_perm(xr, a.off[I], 0x0C0C0000u | ((4u + I) << 8)) + TOFF);
}
#endif

// a ^ b ^ c in ONE instruction (gfx950 v_bitop3_b32, truth table 0x96).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// x * x^32 mod P (the CRC register after absorbing the 32-bit word x), XORed
// with e (the next data word, or 0).
__device__ __forceinline__ uint32_t dstep(const uint32_t* lds, uint32_t x, const LaneAddr& a, uint32_t e = 0) {
    const uint32_t xr = PCRC_LANE_SEL ? x : rot32(x, a);
    return xor3(xor3(look<0, 0>(lds, xr, a), look<1, 0>(lds, xr, a), look<2, 0>(lds, xr, a)),
                look<3, 0>(lds, xr, a), e);
}

// P * x^(8*16*G) mod P through the S tables, XORed with e.
__device__ __forceinline__ uint32_t sstep(const uint32_t* lds, uint32_t p, const LaneAddr& a, uint32_t e = 0) {
    const uint32_t pr = PCRC_LANE_SEL ? p : rot32(p, a);
    return xor3(xor3(look<0, kSOff>(lds, pr, a), look<1, kSOff>(lds, pr, a), look<2, kSOff>(lds, pr, a)),
                look<3, kSOff>(lds, pr, a), e);
}

// Byte-serial step with the D3 slice (D3[b] = b<<24 * x^32 = b * x^8, the
// classic byte table).
__device__ __forceinline__ uint32_t bytestep(const uint32_t* lds, uint32_t c, uint8_t b, const LaneAddr& a) {
    const uint32_t x = (c ^ b) & 0xffu;
    return lds_word(lds, (x << 8) + 3u * 32u + a.r4) ^ (c >> 8);
}

// CRC (init 0, no xorout) of one 16-byte block: four chained word steps.
__device__ __forceinline__ uint32_t crc16(const uint32_t* lds, uint4 w, const LaneAddr& a) {
    uint32_t c = dstep(lds, w.x, a, w.y);
    c = dstep(lds, c, a, w.z);
    c = dstep(lds, c, a, w.w);
    return dstep(lds, c, a);
}

// Lagged block CRC: crc16(w) = v * x^32 with v the register after the first
// three word steps. The generic kernel runs the column recurrence on
// Q = P * x^-32 (Q <- Q * X ^ v): 16 instead of 20 lookups per block, and
// P = D(Q) once per lane per buffer. Measured +1-2 points on C2-C5.
__device__ __forceinline__ uint32_t lag16(const uint32_t* lds, uint4 w, const LaneAddr& a) {
    uint32_t c = dstep(lds, w.x, a, w.y);
    c = dstep(lds, c, a, w.z);
    return dstep(lds, c, a, w.w);
}

// U lagged blocks of one lane's column: independent (ILP), only the row
// shift is carried.
template <int U>
__device__ __forceinline__ uint32_t lag_column_step(const uint32_t* lds, uint32_t q, const uint4 (&w)[U],
                                                    const LaneAddr& a) {
    uint32_t c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) c[u] = lag16(lds, w[u], a);
#pragma unroll
    for (int u = 0; u < U; ++u) q = sstep(lds, q, a, c[u]);
    return q;
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

// head_word without branches (selects only): every lane can run it (lanes
// whose words lie past the first data word get k <= -4: unchanged), so the
// head needs no divergent region, whose join made the compiler wait for ALL
// loads in flight (vmcnt(0)) instead of row 0 alone.
__device__ __forceinline__ uint32_t head_word_sel(uint32_t w, int off, int s0, uint32_t seed) {
    const int k = s0 - off;  // the data starts k bytes into this word
    const int kc = k < -3 ? -3 : k > 3 ? 3 : k;
    const int kk = k < 0 ? 0 : k > 4 ? 4 : k;
    // bytes >= k survive; the seed's bytes land at byte offset k (64-bit
    // shifts, no per-case shift amounts: the compiler keeps it straight-line)
    const uint32_t keep = (uint32_t)(0xffffffffull << (8 * kk));
    const uint32_t in = (uint32_t)(k + 3) <= 6u ? 0xffffffffu : 0u;
    const uint32_t sv = (uint32_t)((((uint64_t)seed) << 32) >> (32 - 8 * kc)) & in;
    return (w & keep) ^ sv;
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

// Basis of a multiplication by a fixed constant (image of every register bit),
// computed at compile time: a table entry (b << 8t) * K is then the XOR of 8
// basis words (16 VALU) instead of a 32-step bit-serial multiply per entry --
// the prologue of every launch builds 1024 D and 1024 S entries per workgroup.
struct Basis32 {
    uint32_t w[32];
};
constexpr Basis32 make_basis32(uint32_t k) {
    Basis32 r{};
    for (int i = 0; i < 32; ++i) r.w[i] = mulmod(1u << i, k);
    return r;
}
__constant__ const Basis32 kBasisD32 = make_basis32(kPoly);  // x^32 mod P
static_assert(make_basis32(kPoly).w[31] == kPoly, "bit 31 is x^0: its image under x^32 is x^32 mod P");
static_assert(make_basis32(kOne).w[7] == (1u << 7), "multiplying by x^0 keeps every bit");

// Finish multipliers of the G >= 16 tables (A_dl, B_dh above).
__constant__ const Basis32 kBasisA32[8] = {
    make_basis32(xpow(32)),           make_basis32(xpow(32 + 128)),     make_basis32(xpow(32 + 2 * 128)),
    make_basis32(xpow(32 + 3 * 128)), make_basis32(xpow(32 + 4 * 128)), make_basis32(xpow(32 + 5 * 128)),
    make_basis32(xpow(32 + 6 * 128)), make_basis32(xpow(32 + 7 * 128))};
__constant__ const Basis32 kBasisB32[7] = {make_basis32(xpow(1024)),     make_basis32(xpow(2 * 1024)),
                                           make_basis32(xpow(3 * 1024)), make_basis32(xpow(4 * 1024)),
                                           make_basis32(xpow(5 * 1024)), make_basis32(xpow(6 * 1024)),
                                           make_basis32(xpow(7 * 1024))};
static_assert(xpow(32) == kPoly, "x^32 mod P is the reflected polynomial");

// (b << 8t) * K from its basis: byte b selects 8 of the 32 words (t is
// uniform per wavefront, so the basis reads are scalar).
template <typename B>
__device__ __forceinline__ uint32_t basis_entry(const B& basis, uint32_t t, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r ^= (0u - ((b >> j) & 1u)) & basis[8 * t + j];
    return r;
}

// Workgroup barrier after LDS writes: this wave's LDS stores complete
// (lgkmcnt(0)), then s_barrier. Unlike __syncthreads it does not wait for
// the wave's global loads (vmcnt), so rows issued before the table prologue
// stay in flight across it.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt, expcnt: no wait
    __builtin_amdgcn_s_barrier();
}

// Build the D and S tables in LDS (every workgroup; 1024 threads = one entry of
// each table per thread).
// FG = 0: R_k lane-combine tables; FG = 4 or 8: F_d finish tables for G = FG;
// FG >= 16: the A_dl / B_dh finish tables for G = FG.
#ifndef PCRC_ABL_NO_PROLOGUE
#define PCRC_ABL_NO_PROLOGUE 0  // A/B builds only: skip the table build (wrong CRCs; the prologue's cost)
#endif
template <int FG = 0>
__device__ __forceinline__ void build_tables(uint32_t* lds, const LaneConsts& kc) {
    if (PCRC_ABL_NO_PROLOGUE) {
        lds_barrier();
        return;
    }
    const uint32_t tid = threadIdx.x;
    const uint32_t t = tid >> 8, b = tid & 255u;
    if constexpr (FG >= 16) {
        // Table k (uniform) and slice t (uniform per wavefront): scalar basis reads.
#pragma unroll
        for (int k = 0; k < 8 + FG / 8 - 1; ++k) {
            const uint32_t* w = k < 8 ? kBasisA32[k].w : kBasisB32[k - 8].w;
            uint32_t r = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) r ^= (0u - ((b >> j) & 1u)) & w[8 * t + j];
            lds[kABase / 4 + k * 1024 + t * 256 + b] = r;
        }
    } else if constexpr (FG == 0) {
        // R_k[t][b] = (b << 8t) * x^(128*B*2^k): XOR of the basis words of b's
        // bits (t is uniform per wavefront, so the basis reads are scalar).
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            uint32_t r = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) r ^= (0u - ((b >> j) & 1u)) & kc.basis[k][8 * t + j];
            lds[kRBase / 4 + k * 1024 + t * 256 + b] = r;
        }
    } else {
        // F_d: words w = 8*t' .. 8*t'+7 of row b (t' = tid >> 8, wave-uniform).
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t w = 8 * t + k;
            const uint32_t d = FG == 8 ? w >> 2 : w >> 3;
            const uint32_t ts = FG == 8 ? w & 3u : (w >> 1) & 3u;
            uint32_t r = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) r ^= (0u - ((b >> j) & 1u)) & kc.fbasis[d][8 * ts + j];
            lds[kFBase / 4 + b * 64 + w] = r;
        }
    }
    const uint32_t dv = basis_entry(kBasisD32.w, t, b);  // (b << 8t) * x^32
    const uint32_t sv = basis_entry(kc.sbasis, t, b);    // (b << 8t) * x^(8*16*G)
    // Row b holds slice t's 8 replicas in words t*8 .. t*8+7 (bank t*8 + r):
    // lanes of a wavefront share t and differ in b (row stride 64 words, the
    // same bank), so writing replica r in step r put all 64 lanes on ONE bank
    // (≈5 µs of a launch, scripts/probe_long_times.py). Lane l writes replica
    // (i + l) % 8 in step i: 8 banks per instruction.
    const uint32_t base = ((b << 8) + (t << 5)) >> 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t r = (i + tid) & 7u;
        lds[base + r] = dv;
        lds[base + kSOff / 4 + r] = sv;
    }
    lds_barrier();
}

// The table prologue from a per-device IMAGE (round 5): build_tables costs
// ≈4.7 µs of VALU at the start of every launch (repo:scripts/probe_long_times.py,
// prologue_us_med), ≈0.6 points of C2 and 2.6 % of the 1 GiB long kernel
// (an A/B build that skips it, repo:profiles/r05r_ab_noprol_*). Each device
// keeps the LDS contents build_tables<G> leaves, written once by
// table_image_kernel<G> (the same code, so the image is exact by
// construction); a launch copies them into LDS with 16-byte loads instead
// (L2-resident: one image per G, read by every workgroup). Slot by G: 4, 8,
// 16, 32, 64 -> 0..4; a null slot (no image yet, or an A/B build with
// PCRC_TABLE_BUILD) builds as before.
#ifndef PCRC_TABLE_BUILD
#define PCRC_TABLE_BUILD 0
#endif
static __device__ const uint32_t* g_table_image[5];
template <int G>
constexpr int table_slot() {
    return G == 4 ? 0 : G == 8 ? 1 : G == 16 ? 2 : G == 32 ? 3 : 4;
}

// PCRC_TABLE_DMA (A/B builds): the copy as LDS-DMA loads
// (global_load_lds_dwordx4: no VGPR round trip, no ds_write; one wave
// instruction fills 1 KiB of LDS at a wave-uniform base, the image being
// lane-linear), then vmcnt(0) -- nothing else is in flight at a kernel's
// start. Measured neutral against the register copy (C3, C5, CRC-64 C2/C3
// shapes within 0.1 point, 1 GiB long kernel 0.1699 vs 0.1693 ms, 430 GPU
// tests green on it; repo:profiles/r05y_ab_dma_vs_regcopy.jsonl), so the
// register copy stays the default.
#ifndef PCRC_TABLE_DMA
#define PCRC_TABLE_DMA 0
#endif
template <uint32_t BYTES>
__device__ __forceinline__ void copy_tables(uint32_t* lds, const uint32_t* img) {
    constexpr uint32_t kVec = BYTES / 16, kPer = (kVec + kBlock - 1) / kBlock;
    const uint32_t tid = threadIdx.x;
    if constexpr (PCRC_TABLE_DMA) {
        static_assert(kVec % 64 == 0, "whole 1 KiB wave pieces");
        typedef __attribute__((address_space(1))) const void g_void;
        typedef __attribute__((address_space(3))) void l_void;
        const uint32_t lane = tid & 63u, w64 = tid & ~63u;
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            const uint32_t j0 = i * kBlock + w64;  // wave-uniform
            if (j0 < kVec)
                __builtin_amdgcn_global_load_lds((g_void*)(img + 4 * (j0 + lane)), (l_void*)(lds + 4 * j0), 16, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the DMA writes have landed
        lds_barrier();
        return;
    }
    u32x4 v[kPer];
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) {
        const uint32_t j = i * kBlock + tid;
        v[i] = j < kVec ? *((const g_u32x4*)img + j) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) {
        const uint32_t j = i * kBlock + tid;
        if (j < kVec) *reinterpret_cast<u32x4*>(lds + 4 * j) = v[i];
    }
    lds_barrier();
}

template <int G>
__device__ __forceinline__ void load_tables(uint32_t* lds, const LaneConsts& kc) {
    const uint32_t* img = PCRC_TABLE_BUILD ? nullptr : g_table_image[table_slot<G>()];
    if (img)
        copy_tables<lds_bytes_for<G>()>(lds, img);
    else
        build_tables<G>(lds, kc);
}

// Writes the image of G (once per device; crc32c_device.hip table_images).
template <int G>
__global__ __launch_bounds__(kBlock) void table_image_kernel(LaneConsts kc, uint32_t* img) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[lds_bytes_for<G>() / 4];
    build_tables<G>(lds, kc);
    for (uint32_t j = threadIdx.x; j < lds_bytes_for<G>() / 16; j += kBlock)
        *reinterpret_cast<u32x4*>(img + 4 * j) = *reinterpret_cast<const u32x4*>(lds + 4 * j);
}

__device__ __forceinline__ LaneAddr lane_addr(uint32_t lane) {
    LaneAddr la;
    const uint32_t q = (lane >> 3) & 3u, r = lane & 7u;
    la.rot = 8u * q;
#pragma unroll
    for (int i = 0; i < 4; ++i) la.off[i] = (((i + q) & 3u) << 5) | (r << 2);
#pragma unroll
    for (int i = 0; i < 4; ++i) la.sel[i] = 0x0C0C0000u | ((4u + ((i + q) & 3u)) << 8);
    la.r4 = r << 2;
    return la;
}

// Shift lane partials to the end of the body (d blocks of 16 bytes) and
// XOR-reduce over the G lanes of the group.
// XOR over the G lanes of an aligned lane group, result in EVERY lane of
// the group. Steps inside a 16-lane row are DPP moves (VALU: quad_perm
// [1,0,3,2], [2,3,0,1], then row_half_mirror and row_mirror, which pair each
// quad / half-row with the other one); only 32- and 64-lane groups use
// ds_bpermute (__shfl_xor), which costs an LDS round trip.
template <int G>
__device__ __forceinline__ uint32_t group_xor(uint32_t v) {
    if constexpr (G >= 2) v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
    if constexpr (G >= 4) v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
    if constexpr (G >= 8) v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
    if constexpr (G >= 16) v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);
    if constexpr (G >= 32) v ^= (uint32_t)__shfl_xor((int)v, 16, 64);
    if constexpr (G >= 64) v ^= (uint32_t)__shfl_xor((int)v, 32, 64);
    return v;
}

template <int G>
__device__ __forceinline__ uint32_t group_reduce(uint32_t pc, uint32_t d, const uint32_t* lds) {
    constexpr int LOG2G = G == 64 ? 6 : G == 32 ? 5 : G == 16 ? 4 : G == 8 ? 3 : 2;
    // pc * x^(128*B*d) via the R_k tables on the bits of d (every lane runs
    // every level; a select keeps the wavefront convergent).
#pragma unroll
    for (int k = 0; k < LOG2G; ++k) {
        const uint32_t* R = lds + kRBase / 4 + k * 1024;
        const uint32_t m = xor3(xor3(R[pc & 0xffu], R[256 + ((pc >> 8) & 0xffu)], R[512 + ((pc >> 16) & 0xffu)]),
                                R[768 + (pc >> 24)], 0u);
        pc = ((d >> k) & 1u) ? m : pc;
    }
    return group_xor<G>(pc);
}

// Up to two pending 4-byte result stores of one lane (see the message kernel).
struct HeldStores {
    uint32_t *a0 = nullptr, *a1 = nullptr;
    uint32_t v0 = 0, v1 = 0;
    __device__ __forceinline__ void put(uint32_t* dst, uint32_t v) {
        if (a1) {
            *a0 = v0;
            *a1 = v1;
            a0 = a1 = nullptr;
        }
        if (!a0) {
            a0 = dst;
            v0 = v;
        } else {
            a1 = dst;
            v1 = v;
        }
    }
    __device__ __forceinline__ void flush() {
        if (a0) *a0 = v0;
        if (a1) *a1 = v1;
    }
};

__device__ __forceinline__ uint32_t wave_id() {
    return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

// x^(8 * 2^i) mod P, i < 64 (shift-by-bytes constants).
struct PowTable {
    uint32_t x8pow2[64];  // x^(8 * 2^i) mod P
};

// (a * b) mod P with the 32 steps as a loop (code size, not speed: for the
// message fold's once-per-wave basis rebuild).
__device__ __forceinline__ uint32_t mulmod_rolled(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll 1
    for (int i = 0; i < 32; ++i, b >>= 1) r = (r >> 1) ^ ((0u - (r & 1u)) & kPoly) ^ ((0u - (b & 1u)) & a);
    return r;
}
// The message fold's basis rebuild as rolled loops: C5 0.853 vs 0.852 steady
// in 3 of 3 alternating rounds, 119 -> 107 VGPRs, 2,860 -> 1,285 instructions
// (repo:profiles/r06h_ab_c5_fold_compact.jsonl). A/B builds: 0 = unrolled.
#ifndef PCRC_FOLD_COMPACT
#define PCRC_FOLD_COMPACT 1
#endif

// x^(8n) mod P: product of the x^(8*2^i) entries over the set bits of n.
__device__ __forceinline__ uint32_t xpow8_tab(uint64_t n, const PowTable& t) {
    uint32_t k = kOne;
    for (int i = 0; n; ++i, n >>= 1)
        if (n & 1) k = mulmod(k, t.x8pow2[i]);
    return k;
}


// -------------------------------------------------------------- generic path
// Any pointer, any length, any seed; one group of G lanes per buffer.
// U rows per step per lane, the next U rows' loads in flight. A buffer runs in
// three parts: geometry + preload (row 0 and the first U rows issued
// together), body (every row: the lane's lagged column partial), finish
// (Q -> P, lane combine, ragged tail).
struct BufGeo {
    const uint8_t* lp;  // this lane's block in row 0
    const uint8_t* a0;  // the aligned start (always a readable 16-byte block when !tiny)
    const uint8_t* eb;  // end of the last whole 16-byte block
    const uint8_t* e;   // end of the buffer
    uint64_t nb;        // 16-byte blocks from the aligned start
    uint64_t full;      // rows where every lane has a block
    uint64_t rows;
    uint32_t rlast;     // blocks in the last row, 1..G
    int s0;             // offset of the data start in block 0
    bool tiny;          // < 64 bytes: byte-serial on the group's first lane
};

template <int G>
__device__ __forceinline__ BufGeo buf_geo(const uint8_t* p, uint64_t n, uint32_t gl) {
    BufGeo g;
    g.tiny = n < 64;
    const uint8_t* a0 = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(15));
    g.e = p + n;
    g.eb = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(g.e) & ~uintptr_t(15));
    g.s0 = (int)(p - a0);
    g.nb = g.tiny ? 0 : (uint64_t)(g.eb - a0) >> 4;  // >= 3 blocks when n >= 64
    g.full = g.nb / G;
    g.rows = (g.nb + G - 1) / G;
    g.rlast = (uint32_t)(g.nb - (g.rows ? g.rows - 1 : 0) * G);
    g.lp = a0 + 16 * gl;
    g.a0 = a0;
    return g;
}

template <int U, bool LEAD = false>
struct BufPre {
    uint4 w0;      // row 0 (the head)
    uint4 cur[U];  // rows 1..U (LEAD: 1+lead..lead+U)
    uint4 wl[LEAD ? U - 1 : 1];  // LEAD: rows 1..lead, lead = (full-1) % U
    uint4 wp;                    // LEAD: the partial last row
};

// Issue row 0 and the first step's U rows (vmcnt counts in order: waiting
// for row 0 does not wait for the others).
// Loads are unconditional inside a non-tiny buffer: a lane with no block in
// row 0, or a buffer too short for a first step, re-reads the aligned start
// (in bounds; the values are discarded), so there is no divergent region
// around the loads and every later wait counts exactly.
// LEAD (long chunks, one buffer per lane group): the lead rows and the
// partial last row are issued here too, so the U-row loop ends exactly at
// the last full row and no row is loaded on its own and waited for (without
// it a 16 KiB chunk ended in three serial load-wait-reduce rows; the CRC-64
// kernels do the same, crc64_kernels.h buffer_reg64).
template <int G, int U, bool LEAD = false>
__device__ __forceinline__ void buf_preload(const BufGeo& g, uint32_t gl, BufPre<U, LEAD>& pre) {
    if (g.tiny) return;
    const uint8_t* p0 = gl < g.nb ? g.lp : g.a0;
    pre.w0 = load16(p0);
    if constexpr (LEAD) {
        const uint32_t lead = g.full >= 1 ? (uint32_t)((g.full - 1) % U) : 0u;
#pragma unroll
        for (int u = 0; u < U - 1; ++u) pre.wl[u] = load16((uint32_t)u < lead ? g.lp + (1 + u) * (16 * G) : p0);
        const bool step = 1 + lead + U <= g.full;
#pragma unroll
        for (int u = 0; u < U; ++u) pre.cur[u] = load16(step ? g.lp + (1 + lead + u) * (16 * G) : p0);
        const bool part = g.full >= 1 && g.full < g.rows && g.full * G + gl < g.nb;
        pre.wp = load16(part ? g.lp + g.full * (16 * G) : p0);
    } else {
        const bool step = 1 + U <= g.full;
#pragma unroll
        for (int u = 0; u < U; ++u) pre.cur[u] = load16(step ? g.lp + (1 + u) * (16 * G) : p0);
    }
}

// The lane's lagged column partial Q over every row (the preloaded ones first).
template <int G, int U, bool LEAD = false>
__device__ __forceinline__ uint32_t buf_body(const uint32_t* lds, const BufGeo& g, const BufPre<U, LEAD>& pre,
                                             uint32_t seed, uint32_t gl, const LaneAddr& la, bool head = true) {
    if (g.tiny) return 0;
    // Row 0 holds the head: masked leading bytes + seed (branch-free; lanes
    // without a block in row 0 feed a zero block, whose lagged CRC is 0).
    // head == false (uniform): an aligned buffer whose seed enters later.
    uint4 w = pre.w0;
    if (head) {
        const int off = (int)gl * 16;
        w.x = head_word_sel(w.x, off, g.s0, seed);
        w.y = head_word_sel(w.y, off + 4, g.s0, seed);
        w.z = head_word_sel(w.z, off + 8, g.s0, seed);
        w.w = head_word_sel(w.w, off + 12, g.s0, seed);
    }
    if (gl >= g.nb) w = make_uint4(0, 0, 0, 0);
    uint32_t pc = lag16(lds, w, la);
    // Full rows 1..full-1: U rows per step, the next U in flight.
    uint64_t row = 1;
    if constexpr (LEAD) {
        const uint32_t lead = g.full >= 1 ? (uint32_t)((g.full - 1) % U) : 0u;
#pragma unroll
        for (int u = 0; u < U - 1; ++u)
            if ((uint32_t)u < lead) pc = sstep(lds, pc, la, lag16(lds, pre.wl[u], la));
        row += lead;
    }
    const uint8_t* lp = g.lp;
    if (row + U <= g.full) {
#if PCRC_BODY == 2
        uint4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = pre.cur[u];
        auto issue = [&](uint4(&w)[U]) {
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the step about to be reduced has landed
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; ++u) w[u] = load16(lp + (row + U + u) * (16 * G));
            __builtin_amdgcn_sched_barrier(0);
        };
        for (;;) {
            if (row + 2 * U > g.full) {
                pc = lag_column_step<U>(lds, pc, a, la);
                row += U;
                break;
            }
            issue(b);
            pc = lag_column_step<U>(lds, pc, a, la);
            row += U;
            if (row + 2 * U > g.full) {
                pc = lag_column_step<U>(lds, pc, b, la);
                row += U;
                break;
            }
            issue(a);
            pc = lag_column_step<U>(lds, pc, b, la);
            row += U;
        }
#else
        if constexpr (PCRC_BODY == 3 || (PCRC_BODY == 0 && U >= 4 && PCRC_BODY_ROLL)) {
        // Rolling reload: row u of the next step is loaded into cur[u] right
        // after row u's lagged block is taken, so the old and new values never
        // live together and the loop edge needs no copies; U rows stay in
        // flight, each issued a little later than at the top of the step.
        uint4 cur[U];
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = pre.cur[u];
        for (; row + 2 * U <= g.full; row += U) {
            uint32_t c[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                c[u] = lag16(lds, cur[u], la);
                cur[u] = load16(lp + (row + U + u) * (16 * G));
            }
#pragma unroll
            for (int u = 0; u < U; ++u) pc = sstep(lds, pc, la, c[u]);
        }
        pc = lag_column_step<U>(lds, pc, cur, la);
        row += U;
        } else {
        uint4 cur[U];
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = pre.cur[u];
#pragma unroll PCRC_BODY + 1
        for (; row + 2 * U <= g.full; row += U) {
            uint4 nxt[U];
#pragma unroll
            for (int u = 0; u < U; ++u) nxt[u] = load16(lp + (row + U + u) * (16 * G));
            pc = lag_column_step<U>(lds, pc, cur, la);
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = nxt[u];
        }
        pc = lag_column_step<U>(lds, pc, cur, la);
        row += U;
        }
#endif
    }
    const bool part = g.full >= 1 && g.full < g.rows && g.full * G + gl < g.nb;
    if constexpr (LEAD) {
        if (part) pc = sstep(lds, pc, la, lag16(lds, pre.wp, la));
    } else {
        for (; row < g.full; ++row) pc = sstep(lds, pc, la, lag16(lds, load16(lp + row * (16 * G)), la));
        // Partial last row.
        if (part) pc = sstep(lds, pc, la, lag16(lds, load16(lp + g.full * (16 * G)), la));
    }
    return pc;
}

// Q * x^(32 + 128 d) (Q -> P and the lane's shift to the end of the blocks,
// d = 16-byte blocks after its last one), XOR-reduced over the group of G
// lanes: the result on every lane of the group.
template <int G>
__device__ __forceinline__ uint32_t finish_group(const uint32_t* lds, uint32_t pc, uint32_t d, const LaneAddr& la) {
    uint32_t crc;
    if constexpr (G <= 8) {
        // Q * x^(32 + 128 d) through F_d: one table step (round 2 used a D step
        // and log2(G) R_k levels, 16 lookups in a dependent chain).
        const uint32_t lane = threadIdx.x & 63u;
        const uint32_t q = (lane >> 3) & 3u;
        const uint32_t dof = G == 8 ? d * 16u : d * 32u + ((lane >> 2) & 1u) * 4u;
        uint32_t f[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t ts = (i + q) & 3u;
            const uint32_t fo = dof + (G == 8 ? ts * 4u : ts * 8u);
            f[i] = lds_word(lds, __builtin_amdgcn_perm(pc, fo, la.sel[i]) + kFBase);
        }
        crc = group_xor<G>(xor3(xor3(f[0], f[1], f[2]), f[3], 0u));
    } else {
        // Q * x^(32 + 128 d): A_(d%8), then B_(d/8) when d >= 8 (every lane
        // runs both levels; a select keeps the wavefront convergent).
        const uint32_t* A = lds + kABase / 4 + (d & 7u) * 1024u;
        uint32_t x = xor3(xor3(A[pc & 0xffu], A[256 + ((pc >> 8) & 0xffu)], A[512 + ((pc >> 16) & 0xffu)]),
                          A[768 + (pc >> 24)], 0u);
        const uint32_t dh = d >> 3;
        const uint32_t* B = lds + kBBase / 4 + (dh ? dh - 1u : 0u) * 1024u;
        const uint32_t y = xor3(xor3(B[x & 0xffu], B[256 + ((x >> 8) & 0xffu)], B[512 + ((x >> 16) & 0xffu)]),
                                B[768 + (x >> 24)], 0u);
        crc = group_xor<G>(dh ? y : x);
    }
    return crc;
}

// Q -> P, shift to the end of the blocks and XOR-reduce over the group, then
// the ragged tail (< 16 bytes); tiny buffers byte-serially. Valid on EVERY
// lane of the group (the byte-serial parts run on all of them: same bytes,
// same loads), so message chains need no broadcast from the first lane.
template <int G>
__device__ __forceinline__ uint32_t buf_finish(const uint32_t* lds, const BufGeo& g, uint32_t pc,
                                               const uint8_t* p, uint64_t n, uint32_t seed, uint32_t gl,
                                               const LaneAddr& la) {
    uint32_t crc;
    if (g.tiny) {
        crc = seed;
        for (uint64_t k = 0; k < n; ++k) crc = bytestep(lds, crc, load8(p + k), la);
        return crc;
    }
    const uint32_t d = (g.rlast + G - 1 - gl) & (G - 1);
    crc = finish_group<G>(lds, pc, d, la);
    for (const uint8_t* q = g.eb; q < g.e; ++q) crc = bytestep(lds, crc, load8(q), la);
    return crc;
}

// CRC-32C of one buffer (seed applied) by a group of G lanes, unpipelined;
// the result is valid on every lane of the group.
template <int G, int U, bool LEAD = false>
__device__ __forceinline__ uint32_t buffer_crc(const uint32_t* lds, const uint8_t* p, uint64_t n, uint32_t seed,
                                               uint32_t gl, const LaneAddr& la, bool head = true) {
    const BufGeo g = buf_geo<G>(p, n, gl);
    BufPre<U, LEAD> pre;
    buf_preload<G, U, LEAD>(g, gl, pre);
    const uint32_t pc = buf_body<G, U, LEAD>(lds, g, pre, seed, gl, la, head);
    return buf_finish<G>(lds, g, pc, p, n, seed, gl, la);
}

// MSG: 0 = buffer batch, 1 = messages chained through the seed, 2 = messages
// with per-segment CRCs + fold (separate instantiations: the two message
// forms in one kernel shared one register allocation, and each is faster
// compiled alone).
// PCRC_BATCH_OVERLAP (buffer batches): the table image's loads, then the
// wave's first buffer's rows, then the LDS writes -- vmcnt counts in issue
// order, so the writes wait for the image only and the first rows stay in
// flight across the barrier ("Table prologue from a per-device
// image").
#ifndef PCRC_BATCH_OVERLAP
#define PCRC_BATCH_OVERLAP 1
#endif
template <int G, int U = 4, int MSG = 0>
__global__ __launch_bounds__(kBlock) void crc32c_batch_kernel(BatchArgs args, LaneConsts kc, PowTable pt) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[lds_bytes_for<G>() / 4];
    // (A/B, repo:profiles/r05t_ab_overlap_c2_c3_c4.jsonl: C2 +0.1 point 3 of 3 rounds,
    // C3 at G = 16 -0.1, C4 +-0; U = 8 spills. At G = 16 the same overlap with
    // the copy as LDS-DMA -- no VGPRs held, a counted vmcnt before the barrier --
    // measured neutral, 4 rounds: repo:profiles/r05z_ab_dma_overlap_c3.jsonl.)
    constexpr bool kOverlap = MSG == 0 && G >= 32 && U <= 4 && PCRC_BATCH_OVERLAP && !PCRC_TABLE_BUILD;
    constexpr bool kLead = PCRC_BATCH_LEAD || (U == 2 && PCRC_BATCH_LEAD2);  // lead rows + partial row preloaded
    constexpr bool kMsgLead = PCRC_MSG_LEAD != 0;  // the same in the message forms
    if constexpr (!kOverlap) load_tables<G>(lds, kc);

    constexpr int GPW = 64 / G;  // buffers per wavefront
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = wave_id();
    const uint32_t gl = lane & (G - 1);
    const uint32_t grp = lane / G;
    const LaneAddr la = lane_addr(lane);

    const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
    if constexpr (MSG) {
        // One group per message: its segments one after the other, either
        // chained through the seed, or each CRC (seed 0) stored and folded:
        // acc = acc*x^(8 len) ^ crc (crc32c_combine, crc.cpp:393-405). No
        // second kernel.
        // Fold basis cache of the per-segment form (see below), kept across
        // the wave's messages: W register bits per lane.
        constexpr int kFoldW = G >= 32 ? 1 : G >= 8 ? 32 / G : 1;
        uint64_t klen = ~0ull;
        uint32_t kb[kFoldW];
        // MSG == 2: segment-CRC stores are held back, up to two per lane,
        // and issued when a third arrives or at the end of the wave's work --
        // in C5 (two rounds per wave) all of them after the wave's last
        // payload load. (Holding the message-CRC stores too: neutral.)
        HeldStores seg_held;
#pragma unroll
        for (int w = 0; w < kFoldW; ++w) kb[w] = 0;
        for (uint64_t wv = (uint64_t)blockIdx.x * kWaves + wave; wv * GPW < args.nmsg; wv += nwaves) {
            const uint64_t m = wv * GPW + grp;
            const bool active = m < args.nmsg;
            uint64_t s0 = 0, s1 = 0;
            uint32_t acc = args.seed0;
            if (active) {
                s0 = args.msg_start[m];
                s1 = args.msg_start[m + 1];
                if (args.seeds) acc = args.seeds[m];
            }
            if constexpr (MSG == 1) {
                // No per-segment CRCs wanted: chain through the seed
                // (crc32c_extend(seg, n, acc), Crc32Hasher::extend_hash).
                photon_crc_iovec nx = {nullptr, 0};
                if (s0 < s1) nx = args.iov[s0];
                for (uint64_t sg = s0; sg < s1; ++sg) {
                    // The next segment's descriptor is loaded before this
                    // segment's rows (unconditionally: the last one re-reads
                    // itself), so it has arrived when the next segment starts.
                    const photon_crc_iovec cur = nx;
                    nx = args.iov[sg + 1 < s1 ? sg + 1 : sg];
                    acc = buffer_crc<G, U, kMsgLead>(lds, static_cast<const uint8_t*>(cur.base), cur.len, acc, gl, la);
                }
            } else {
                // Per-segment CRCs (seed 0) and the fold acc = acc * K ^ c,
                // K = x^(8 len) (crc32c_combine, crc.cpp:393-405). The multiply
                // is spread over the group: lane gl holds the images under K of
                // the register bits gl*W .. gl*W+W-1 (kb, rebuilt only when the
                // length changes -- once per wave for equal segments), so
                // acc * K is W select-XORs per lane plus an XOR reduction over
                // the G lanes, instead of a 32-step bit-serial multiply on one
                // lane while the others wait.
                // Segment CRCs are not stored one by one from the first lane
                // (a 4-byte store per segment sits in the wave's vmcnt queue in
                // front of the next segment's loads): lane j of the group keeps
                // the CRC of segment s0 + j (mod G), and the group stores G
                // consecutive CRCs with one coalesced store.
                // The fold of segment k runs after segment k+1's first loads are
                // issued (its DPP reduction and select-XORs then overlap them
                // instead of delaying them).
                auto fold = [&](uint32_t c, uint64_t n) {
                    if constexpr ((PCRC_ABL & 16) != 0) {
                        acc ^= c;
                        (void)n;
                    } else if constexpr (G >= 8) {
                        if (n != klen) {
#if PCRC_FOLD_COMPACT
                            // Rolled loops (runs once per wave for equal
                            // segments; unrolled, its 4 + log2(n) 32-step
                            // multiplies were 1,800 instructions inside the
                            // segment loop). K = x^(8n); bit b's image is
                            // K * x^(31-b): a chain of single x-steps.
                            uint32_t r = kOne;
                            uint64_t m = n;
#pragma unroll 1
                            for (int i = 0; m; ++i, m >>= 1)
                                if (m & 1) r = mulmod_rolled(r, pt.x8pow2[i]);
#pragma unroll
                            for (int w = 0; w < kFoldW; ++w) kb[w] = 0u;
#pragma unroll 1
                            for (uint32_t j = 0; j < 32; ++j) {  // r = K * x^j, bit 31 - j
#pragma unroll
                                for (int w = 0; w < kFoldW; ++w)
                                    kb[w] = gl * kFoldW + w == 31u - j ? r : kb[w];
                                r = (r >> 1) ^ ((0u - (r & 1u)) & kPoly);
                            }
#else
                            const uint32_t kn = xpow8_tab(n, pt);
#pragma unroll
                            for (int w = 0; w < kFoldW; ++w) {
                                const uint32_t bit = gl * kFoldW + w;
                                kb[w] = bit < 32 ? mulmod(1u << bit, kn) : 0u;
                            }
#endif
                            klen = n;
                        }
                        uint32_t part = 0;
#pragma unroll
                        for (int w = 0; w < kFoldW; ++w) {
                            // bit >= 32 only for 64-lane groups (kb[w] = 0
                            // there): clamp so the shift stays defined
                            const uint32_t bit = gl * kFoldW + w;
                            part ^= (bit < 32 && ((acc >> (bit & 31u)) & 1u)) ? kb[w] : 0u;
                        }
                        acc = group_xor<G>(part) ^ c;  // acc and c are valid on every lane of the group
                    } else {
                        // 4-lane groups (segments < 2 KiB): 8 basis words per
                        // lane would spill; every lane multiplies.
                        if (n != klen) {
                            kb[0] = xpow8_tab(n, pt);
                            klen = n;
                        }
                        acc = mulmod(acc, kb[0]) ^ c;
                    }
                };
                uint32_t pend = 0, cprev = 0;
                uint64_t nprev = 0;
                bool have = false;
                photon_crc_iovec nx = {nullptr, 0};
                if (s0 < s1) nx = args.iov[s0];
                for (uint64_t sg = s0; sg < s1; ++sg) {
                    const photon_crc_iovec cur = nx;  // (prefetched as above)
                    nx = args.iov[sg + 1 < s1 ? sg + 1 : sg];
                    const uint8_t* p = static_cast<const uint8_t*>(cur.base);
                    const uint64_t n = cur.len;
                    const BufGeo g = buf_geo<G>(p, n, gl);
                    BufPre<U, kMsgLead> pre;
                    buf_preload<G, U, kMsgLead>(g, gl, pre);
                    if (have) fold(cprev, nprev);
                    const uint32_t pc = buf_body<G, U, kMsgLead>(lds, g, pre, 0u, gl, la);
                    const uint32_t c = buf_finish<G>(lds, g, pc, p, n, 0u, gl, la);
                    const uint32_t j = (uint32_t)((sg - s0) & (G - 1));
                    if (gl == j) pend = c;
                    if (j == G - 1 || sg + 1 == s1) {
                        const uint64_t first = sg - j;
                        // Held back, two per lane, and written when a third
                        // comes or the wave ends (see HeldStores above).
                        if (gl <= j && !(PCRC_ABL & 8)) seg_held.put(args.out + first + gl, pend);
                    }
                    cprev = c;
                    nprev = n;
                    have = true;
                }
                if (have) fold(cprev, nprev);
            }
            if (active && gl == 0) args.msg_out[m] = acc;
        }
        seg_held.flush();
        return;
    }
    // (Measured and dropped: software-pipelining the wave's buffers -- the
    // next buffer's descriptor and first rows issued before the current
    // buffer's finish -- 127 instead of 106 VGPRs, C2 -1 point, C3 -0.6.)
    auto item = [&](uint64_t wv, const uint8_t** p, uint64_t* n, uint32_t* seed) {
        const uint64_t bi = wv * GPW + grp;
        *p = nullptr;
        *n = 0;
        *seed = args.seed0;
        if (bi < args.count) {
            if (args.iov) {
                *p = static_cast<const uint8_t*>(args.iov[bi].base);
                *n = args.iov[bi].len;
            } else {
                *p = args.base + bi * args.stride;
                *n = args.nbytes;
            }
            if (args.seeds) *seed = args.seeds[bi];
        }
    };
    if constexpr (kOverlap) {
        constexpr uint32_t kVec = lds_bytes_for<G>() / 16, kPer = (kVec + kBlock - 1) / kBlock;
        const uint32_t* img = g_table_image[table_slot<G>()];
        const uint32_t tid = threadIdx.x;
        u32x4 tv[kPer];
        if (img && !(PCRC_ABL & 4)) {
#pragma unroll
            for (uint32_t i = 0; i < kPer; ++i) {
                const uint32_t j = i * kBlock + tid;
                tv[i] = j < kVec ? *((const g_u32x4*)img + j) : u32x4{0, 0, 0, 0};
            }
        }
        uint64_t wv = (uint64_t)blockIdx.x * kWaves + wave;
        const uint8_t* p;
        uint64_t n;
        uint32_t seed;
        item(wv, &p, &n, &seed);
        BufGeo g = buf_geo<G>(p, n, gl);
        BufPre<U, kLead> pre;
        if (wv * GPW < args.count) buf_preload<G, U, kLead>(g, gl, pre);  // wave-uniform
        if (PCRC_ABL & 4) {
            lds_barrier();
        } else if (img) {
#pragma unroll
            for (uint32_t i = 0; i < kPer; ++i) {
                const uint32_t j = i * kBlock + tid;
                if (j < kVec) *reinterpret_cast<u32x4*>(lds + 4 * j) = tv[i];
            }
            lds_barrier();
        } else {
            build_tables<G>(lds, kc);
        }
        for (bool first = true; wv * GPW < args.count; wv += nwaves, first = false) {
            if (!first) {
                item(wv, &p, &n, &seed);
                g = buf_geo<G>(p, n, gl);
                buf_preload<G, U, kLead>(g, gl, pre);
            }
            const uint32_t s = args.shift_init ? 0u : seed;
            const uint32_t pc = buf_body<G, U, kLead>(lds, g, pre, s, gl, la, !args.shift_init);
            const uint32_t crc = buf_finish<G>(lds, g, pc, p, n, s, gl, la);
            const uint64_t bi = wv * GPW + grp;
            if (bi < args.count && gl == 0) args.out[bi] = crc ^ args.init_shift;  // init_shift is 0 unless shift_init
        }
        return;
    }
    for (uint64_t wv = (uint64_t)blockIdx.x * kWaves + wave; wv * GPW < args.count; wv += nwaves) {
        const uint64_t bi = wv * GPW + grp;
        const bool active = bi < args.count;
        const uint8_t* p;
        uint64_t n;
        uint32_t seed;
        item(wv, &p, &n, &seed);
        const uint32_t crc = buffer_crc<G, U, kLead>(lds, p, n, args.shift_init ? 0u : seed, gl, la,
                                                               !args.shift_init);
        if (active && gl == 0) args.out[bi] = crc ^ args.init_shift;  // init_shift is 0 unless shift_init
    }
}

// Per-message fold of per-segment CRCs: acc = seed; acc = acc*x^(8 len)+crc.
// (Crc32Hasher::extend_hash, rpc/serialize.h:244-252, equals this fold.)

__device__ __forceinline__ uint32_t shift_bytes_tab(uint32_t crc, uint64_t n, const PowTable& t) {
    for (int i = 0; n; ++i, n >>= 1)
        if (n & 1) crc = mulmod(crc, t.x8pow2[i]);
    return crc;
}


// One thread per message. The segments' lengths and CRCs are loaded 8 at a
// time before the (dependent) fold, and the shift constant x^(8*len) is
// recomputed only when the length changes (messages of equal-size segments
// pay one mulmod per segment).
__global__ void crc32c_msg_fold_kernel(const photon_crc_iovec* iov, const uint64_t* msg_start, uint64_t nmsg,
                                       const uint32_t* seg_crc, uint32_t seed0, const uint32_t* seeds,
                                       uint32_t* out, PowTable pt) {
    const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= nmsg) return;
    const uint64_t s0 = msg_start[m], s1 = msg_start[m + 1];
    uint32_t acc = seeds ? seeds[m] : seed0;
    uint64_t klen = 0;
    uint32_t k = kOne;  // x^(8*klen)
    for (uint64_t s = s0; s < s1; s += 8) {
        uint64_t len[8];
        uint32_t c[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (s + j < s1) {
                len[j] = iov[s + j].len;
                c[j] = seg_crc[s + j];
            }
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (s + j < s1) {
                if (len[j] != klen) {
                    k = xpow8_tab(len[j], pt);
                    klen = len[j];
                }
                acc = mulmod(acc, k) ^ c[j];
            }
    }
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

// ------------------------------------------------------- one long buffer
// photon_crc32c_extend_device (crc32c_extend, crc32c.h:30-33, over ONE
// device buffer of more than 256 KiB) in ONE launch that fills the chip. The
// cut (long_plan.h): the head [data, A) up to the first 4 KiB boundary A
// carries the seed; the body [A, end) is T chunks of `chunk` bytes (the last
// one L bytes), every one aligned and whole but the last, so no body chunk
// has a masked head. R*S slots (S lane groups, R rounds): slot v belongs to
// group v % S in round v / S; body chunk t sits in slot v = t + D, D = R*S - T
// (empty slots at the FRONT: leading zeros do not change a CRC), the head in
// slot D - 1 (slot -1, a round before group S-1's first, when D = 0).
// By linearity (crc.cpp:393-405), with X = x^(8 chunk) and J = x^-(8 (chunk
// - L)): CRC = J * XOR_v c_v X^(R S - 1 - v) ^ c_last, the last (short) body
// chunk entering with factor 1 (J X^0 x^(8 (chunk - L)) = 1). With v = g +
// r S and g = (16 b + w) GPW + grp (workgroup b, wave w, group grp):
//   X^(R S - 1 - v) = X^(S (R - 1 - r)) X^(GPW - 1 - grp) Z^(15 - w) Y^(grid - 1 - b)
// (Z = X^GPW, Y = Z^16), so the factors are applied in stages, each a
// multiplication by ONE constant per group / wave / workgroup, done
// lane-parallel (lane l of a 32-lane half holds basis word l of the
// constant: a select and a 32-lane XOR, mul_lanes):
//   group: Horner over its rounds, acc <- acc X^S ^ c (basis words of X^S
//          from the host);
//   wave (GPW = 2): acc_0 X ^ acc_1 (basis words of X from the host);
//   wave: * Z^(15 - w) (basis words from the host's constant through the
//          LDS D tables at kernel start, basis_word_lds: 4 lookups per lane);
//   workgroup: XOR of its waves in LDS, * J Y^(grid - 1 - b) (wave 0, basis
//          words computed at kernel start), ^ c_last in the last workgroup;
//   grid: the workgroups' values XORed by long_reduce.
// Round 3 multiplied every group's accumulator by its own J X^(T - 1 - t_last)
// after the chunk loop: three dependent 32-step bit-serial multiplies (1.7
// µs of the 1 GiB launch's tail; CRC-64: two 64-step ones).
constexpr uint32_t kLongMaxFt = 256;  // workgroups of a long launch (the workgroup factors in the arguments)
struct LongArgs {
    const uint8_t* data;
    uint64_t head;      // bytes before A (0..4095): slot D - 1, with the seed
    uint64_t chunk;     // body chunk bytes (a 1 KiB multiple)
    int64_t nchunks;    // T
    uint64_t last;      // L: bytes of the last body chunk
    int64_t lead;       // D = R S - T
    uint64_t stride;    // S: lane groups in the grid
    uint32_t rounds;    // R
    uint32_t seed;
    uint32_t* out;
    uint32_t* acc;      // long_reduce state (8 + 8 * kLongMaxGrid bytes; grid > 1 only)
    uint64_t tbase;     // long_reduce: the state's ticket count before this launch
    uint32_t treset;    // long_reduce: put the ticket back to 0 (a leased state)
    uint32_t xsb[32];   // basis words of X^S
    uint32_t xb[32];    // basis words of X (GPW = 2)
    uint32_t zt[16];    // Z^(15 - w)
    uint32_t ft[kLongMaxFt];  // J Y^(grid - 1 - b)
    uint32_t out_tag;   // routed calls: nonzero = *out is a tagged 8-byte word in pinned memory (long_reduce)
};

// The long kernels' cross-workgroup XOR, called by EVERY thread of wave 0
// with its workgroup's value v (valid on lane 0): lane 0 stores v into the
// workgroup's slot and takes a ticket; the workgroup that takes the last
// ticket loads all slots at once, XORs them, writes fin(total) and puts the
// ticket back to 0 for the next lease. state: ticket, then kLongMaxGrid
// slots (8 + 8 * kLongMaxGrid bytes).
//
// Ordering without fences: every access to the state is a device-scope
// (agent) atomic, the slot store has completed before the ticket is taken,
// and the last workgroup issues its slot loads only after its ticket
// returned. In the LLVM AMDGPU memory model's code sequences for GFX942
// (AMDGPUUsage "Memory Model GFX942"; gfx950 follows it), the rows used are
//   store atomic monotonic, agent, global  -> global_store sc1
//   load atomic monotonic, agent, global   -> global_load sc1
//   atomicrmw monotonic, agent, global     -> global_atomic (sc0: returns)
// and the release sequence a fetch_add(release, agent) would add is
// `buffer_wbl2 sc1; s_waitcnt vmcnt(0)`: the write-back only concerns
// earlier NON-atomic stores cached in this XCD's L2 (there are none: the
// slot store is itself an sc1 agent-scope store), and the `s_waitcnt
// vmcnt(0)` is kept here explicitly -- on GFX9 stores are counted in vmcnt,
// so the slot store is acknowledged at agent scope before the ticket atomic
// issues. The acquire side's `buffer_inv sc1` only matters for later
// non-atomic loads; the slot loads are sc1 atomics issued after the ticket's
// value came back (control dependency through the readfirstlane'd branch).
// Emitted code (hipcc -S, crc32c_long_kernel<32,4>): global_store_dword
// ... sc1; s_waitcnt vmcnt(0); global_atomic_add ... sc0; s_waitcnt
// vmcnt(0); ... global_load_dword ... sc1. The stores-in-vmcnt rule is GFX9's
// (GFX10+ count stores in vscnt), hence the #error for other targets below.
// Measured and not kept (round 4): tagged slots {launch tag, word} stored
// without waiting and a ticket taken at once, the last workgroup reloading
// until every tag is this launch's -- one acknowledgement less on paper,
// ±0 for CRC-32C and 1.9 µs slower for CRC-64 on 1 GiB
// (repo:profiles/r04_ab_tagged_reduce.jsonl).
// FENCED (bench probe, ABL 8) keeps the release/acquire pair: 5.7 µs more
// per 1 GiB launch (repo:profiles/r03b_ab_long_tail_ablations.jsonl). Round
// 3's first form, device-scope atomicXor into one accumulator or eight with
// a second level, was a chain of 4-7 dependent atomics with fences (8 µs
// after the last chunk). tests/test_gpu_fullsize.py runs 1,000 back-to-back
// full-grid launches over alternating data through one state.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "long_reduce's fence-free ordering relies on GFX9's stores-in-vmcnt (s_waitcnt 0x0F70 = vmcnt(0)): gfx942/gfx950 only"
#endif
constexpr uint32_t kLongMaxGrid = 512;
template <typename T, typename F, bool FENCED = false>
__device__ __forceinline__ void long_reduce_slots(T v, T* state, T* out, F fin, uint64_t base, uint32_t reset,
                                                  uint32_t tag = 0) {
    const uint32_t grid = gridDim.x, lane = threadIdx.x & 63u;
    // tag != 0 (routed calls, out in the routed stream's coherent pinned
    // area): 8-byte system-scope stores {tag, 32-bit word} (one, or two for
    // CRC-64); the host spins on the tags instead of waiting for the stream
    auto put = [&](T r) {
        if (tag) {  // one tagged word per 32 bits, low word first
#pragma unroll
            for (uint32_t h = 0; h < sizeof(T) / 4; ++h)
                __hip_atomic_store(reinterpret_cast<uint64_t*>(out) + h,
                                   (uint64_t)tag << 32 | (uint32_t)((uint64_t)r >> (32 * h)), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        *out = r;
    };
    if (grid == 1) {
        if (lane == 0) put(fin(v));
        return;
    }
    // The same layout for both widths: a 64-bit ticket in bytes 0-7, slots
    // from byte 8. The ticket is never reset on a per-stream state: it counts
    // every workgroup of every launch, the host passes the count before this
    // launch (`base`, kept per state and advanced under a lock in launch
    // order), and the workgroup that draws base + grid - 1 is the last. So a
    // launch that overlapped another on the same state (a destroyed stream's
    // last launch still running when a new stream got its handle)
    // can only spoil those two launches' results: the count stays exact for
    // every later launch. A leased state (reset != 0) starts at 0 and is put
    // back to 0 (leases are exclusive, ordered by their event).
    unsigned long long* ticket = reinterpret_cast<unsigned long long*>(state);
    T* slot = reinterpret_cast<T*>(reinterpret_cast<char*>(state) + 8);
    const unsigned long long mine = base + grid - 1;
    uint32_t last = 0;
    if (lane == 0) {
        if constexpr (FENCED) {
            slot[blockIdx.x] = v;
            last = __hip_atomic_fetch_add(ticket, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == mine;
        } else {
            __hip_atomic_store(slot + blockIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);  // compiler order only
            __builtin_amdgcn_s_waitcnt(0x0F70);       // vmcnt(0): the slot store has completed
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            last = __hip_atomic_fetch_add(ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == mine;
        }
    }
    if (!__shfl(last, 0)) return;
    if constexpr (FENCED) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    T x = 0;
    for (uint32_t w = lane; w < grid; w += 64) x ^= __hip_atomic_load(slot + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (sizeof(T) == 8)
        x = ((T)group_xor<64>((uint32_t)(x >> 32)) << 32) | group_xor<64>((uint32_t)x);
    else
        x = group_xor<64>(x);
    if (lane == 0) {
        put(fin(x));
        if (reset) __hip_atomic_store(ticket, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// The same reduce with ONE round trip on the last workgroup's path (round 5;
// the default, PCRC_LONG_REDUCE_WORD): per 32-bit half of the value, one
// 64-bit state word {count (high 32), XOR (low 32)}. Each workgroup XORs its
// half into the word (no return) and then adds 1 << 32 to it (returned),
// back to back, no wait between: two atomics of one thread to ONE location
// are in that location's modification order as issued (write-write coherence,
// C++ [intro.races]; LLVM AMDGPU implements it), every other workgroup's add
// came before the last one's, and each one's XOR before its add, so the add
// that returns count = base + grid - 1 (mod 2^32) returns, in its low half,
// the XOR of every workgroup's half. That workgroup writes fin(half) and puts
// the word to {base + grid, 0} (a leased / captured state: to 0). CRC-64's
// two halves have a word each and may have different last workgroups: each
// writes its half (the routed form already carries one tagged word per half;
// a device *out gets two 32-bit stores). A CRC32C launch's last workgroup also
// sets the second word, so that both words count every launch on the state.
// Saves the slot store's acknowledgement and the last workgroup's slot loads.
#ifndef PCRC_LONG_REDUCE_WORD
#define PCRC_LONG_REDUCE_WORD 1
#endif
template <typename T, typename F>
__device__ __forceinline__ void long_reduce_word(T v, T* state, T* out, F fin, uint64_t base, uint32_t reset,
                                                 uint32_t tag = 0) {
    constexpr uint32_t kHalves = sizeof(T) / 4;
    const uint32_t grid = gridDim.x, lane = threadIdx.x & 63u;
    if (grid == 1) {
        if (lane == 0) {
            const T r = fin(v);
            if (tag) {
#pragma unroll
                for (uint32_t h = 0; h < kHalves; ++h)
                    __hip_atomic_store(reinterpret_cast<uint64_t*>(out) + h,
                                       (uint64_t)tag << 32 | (uint32_t)((uint64_t)r >> (32 * h)), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
                *out = r;
            }
        }
        return;
    }
    const uint64_t v0 = (uint64_t)__shfl((unsigned long long)(uint64_t)v, 0);  // v is valid on lane 0
    if (lane < kHalves) {
        unsigned long long* w = reinterpret_cast<unsigned long long*>(state) + lane;
        const uint32_t half = (uint32_t)(v0 >> (32 * lane));
        (void)__hip_atomic_fetch_xor(w, (unsigned long long)half, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long old = __hip_atomic_fetch_add(w, 1ull << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(old >> 32) == (uint32_t)(base + grid - 1)) {
            // fin is bitwise per half for both CRCs (identity / inversion)
            const uint32_t r = (uint32_t)((uint64_t)fin((T)((uint64_t)(uint32_t)old << (32 * lane))) >> (32 * lane));
            if (tag)
                __hip_atomic_store(reinterpret_cast<uint64_t*>(out) + lane, (uint64_t)tag << 32 | r, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            else
                reinterpret_cast<uint32_t*>(out)[lane] = r;
            const unsigned long long next = reset ? 0ull : (unsigned long long)(uint32_t)(base + grid) << 32;
            __hip_atomic_store(w, next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // a 32-bit CRC's launch advances the second word too: the state's
            // count covers every launch on it, of either CRC
            if (kHalves == 1) __hip_atomic_store(w + 1, next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// The one-round-trip word as a two-level tree (round 5, the default,
// PCRC_LONG_REDUCE_TREE): device-scope atomics on ONE word serialise at the
// memory side, ≈12 ns each, so a flat word costs a launch of G workgroups
// about 2 G x 12 ns -- 10 µs at 512 workgroups, 3-4 µs at 256
// (repo:scripts/probe_atomics.hip, repo:profiles/r05m_probe_atomics.jsonl:
// 512 workgroups 13.3 µs per launch on one word, 3.0 µs spread over 16 words,
// 2.9 µs with no atomic). Workgroup b counts on group word i = (base + b) mod
// 16 (16 words, each on a 128-byte line of its own; the same {count, XOR}
// form); the group's last member (its add returns count_i - 1, count_i = the
// members of i among all workgroups of the state so far, a closed form in
// base + grid) zeroes the group's XOR and adds {m_i, XOR} to the top word
// (m_i = the group's members in this launch), whose count therefore ends at
// base + grid as the flat word's did; the add that reaches it is the last
// group's and writes the result. Both halves' words advance on every launch
// (a CRC32C value's high half is 0), so one state serves both CRCs.
#ifndef PCRC_LONG_REDUCE_TREE
#define PCRC_LONG_REDUCE_TREE 1
#endif
constexpr uint32_t kTreeGroups = 16, kTreeLine = 16;  // group i's words at state + 16 (1 + i) (8-byte words)
template <typename T, typename F>
__device__ __forceinline__ void long_reduce_tree(T v, T* state, T* out, F fin, uint64_t base, uint32_t reset,
                                                 uint32_t tag = 0) {
    constexpr uint32_t kHalves = sizeof(T) / 4;
    const uint32_t grid = gridDim.x, lane = threadIdx.x & 63u;
    if (grid == 1) {
        long_reduce_word(v, state, out, fin, base, reset, tag);
        return;
    }
    const uint64_t v0 = (uint64_t)__shfl((unsigned long long)(uint64_t)v, 0);  // v is valid on lane 0
    if (lane < 2) {
        unsigned long long* words = reinterpret_cast<unsigned long long*>(state);
        const uint64_t end = base + grid;  // the state's workgroups after this launch
        const uint32_t i = (uint32_t)((base + blockIdx.x) % kTreeGroups);
        auto members = [&](uint64_t below) {  // workgroups g < below of the state with g mod 16 = i
            return below > i ? (below - 1 - i) / kTreeGroups + 1 : 0ull;
        };
        const uint64_t ci = members(end), mi = ci - members(base);
        unsigned long long* g = words + kTreeLine * (1 + i) + lane;
        const uint32_t half = lane < kHalves ? (uint32_t)(v0 >> (32 * lane)) : 0u;
        (void)__hip_atomic_fetch_xor(g, (unsigned long long)half, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long old = __hip_atomic_fetch_add(g, 1ull << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(old >> 32) == (uint32_t)(ci - 1)) {  // the group's last member in this launch
            __hip_atomic_store(g, reset ? 0ull : (unsigned long long)(uint32_t)ci << 32, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            unsigned long long* t = words + lane;
            (void)__hip_atomic_fetch_xor(t, (unsigned long long)(uint32_t)old, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long top = __hip_atomic_fetch_add(t, (unsigned long long)mi << 32, __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)(top >> 32) + (uint32_t)mi == (uint32_t)end) {  // the last group: the result
                if (lane < kHalves) {
                    const uint32_t r =
                        (uint32_t)((uint64_t)fin((T)((uint64_t)(uint32_t)top << (32 * lane))) >> (32 * lane));
                    if (tag)
                        __hip_atomic_store(reinterpret_cast<uint64_t*>(out) + lane, (uint64_t)tag << 32 | r,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    else
                        reinterpret_cast<uint32_t*>(out)[lane] = r;
                }
                __hip_atomic_store(t, reset ? 0ull : (unsigned long long)(uint32_t)end << 32, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

template <typename T, typename F, bool FENCED = false>
__device__ __forceinline__ void long_reduce(T v, T* state, T* out, F fin, uint64_t base, uint32_t reset,
                                            uint32_t tag = 0) {
    if constexpr (PCRC_LONG_REDUCE_WORD && PCRC_LONG_REDUCE_TREE && !FENCED)
        long_reduce_tree(v, state, out, fin, base, reset, tag);
    else if constexpr (PCRC_LONG_REDUCE_WORD && !FENCED)
        long_reduce_word(v, state, out, fin, base, reset, tag);
    else
        long_reduce_slots<T, F, FENCED>(v, state, out, fin, base, reset, tag);
}

// v * x mod P (reflected: bit j = coefficient of x^(31-j)).
__device__ __forceinline__ uint32_t mulx(uint32_t v) { return (v >> 1) ^ ((0u - (v & 1u)) & kPoly); }

// Basis word i of a multiplication by c: (1 << i) * c = c * x^(31-i), from
// the D tables in LDS (after build_tables): k = 31 - i = 8a + b; the bit part
// c * x^b = (c >> b) ^ D3[(c << (8 - b)) & 0xff] (D3[v] = v * x^8: the b bits
// shifted out are a byte shifted out 8 - b positions early), the byte part
// c1 * x^(8a) = (c1 >> 8a) ^ XOR_(j < a) D_(4-(a-j))[byte_j(c1)] (slice t holds
// v * x^(32 - 8t)). 4 lookups instead of 31 dependent select steps (crc64:
// basis_word64_lds). Lanes with a <= j look up entry 0 (= 0).
__device__ __forceinline__ uint32_t basis_word_lds(const uint32_t* lds, uint32_t c, uint32_t i, uint32_t r4) {
    const uint32_t k = 31u - i, b = k & 7u, a = k >> 3;
    const uint32_t y = (c << (8u - b)) & 0xffu;
    const uint32_t v = (c >> b) ^ lds_word(lds, (y << 8) + 3u * 32u + r4);
    uint32_t r = v >> (8u * a);
#pragma unroll
    for (uint32_t j = 0; j < 3; ++j) {
        const uint32_t byte = j < a ? (v >> (8u * j)) & 0xffu : 0u;
        r ^= lds_word(lds, (byte << 8) + (((4u + j - a) & 3u) << 5) + r4);
    }
    return r;
}

// v * c for a v held by every lane of a 32-lane half (lane l of the half
// holds bw = basis word l of c): one select per lane and a 32-lane XOR.
__device__ __forceinline__ uint32_t mul_lanes(uint32_t v, uint32_t bw, uint32_t l32) {
    return group_xor<32>(((v >> l32) & 1u) ? bw : 0u);
}

// The bytes of slot v: [*p, *p + *n) (empty slots: 0 bytes); *head: the
// slot carries the head [data, A) and so the seed. With a body
// (PCRC_LONG_MERGE_HEAD), the head is read as the front of body chunk 0's
// slot -- [data, A + chunk) from the unaligned start -- instead of as slot D -
// 1: the same algebra (crc(head | chunk0) = crc(head) X ^ crc(chunk0), and
// the head's slot factor was X times chunk 0's), without round 3-4's extra
// round -1 for group S - 1 when D = 0 (the reference's 1 GiB at buf+1).
template <typename A>
__device__ __forceinline__ void long_slot(const A& a, int64_t v, const uint8_t** p, uint64_t* n, bool* last,
                                          bool* head) {
    const int64_t t = v - a.lead;  // body chunk, or -1 for the head slot
    *last = t == a.nchunks - 1;
    if (PCRC_LONG_MERGE_HEAD && a.nchunks > 0) {
        *head = t == 0;
        if (t < 0) {
            *p = a.data;
            *n = 0;
        } else {
            *p = t == 0 ? a.data : a.data + a.head + (uint64_t)t * a.chunk;
            *n = (t == 0 ? a.head : 0) + (*last ? a.last : a.chunk);
        }
        return;
    }
    *head = t == -1;
    if (t == -1) {
        *p = a.data;
        *n = a.head;
    } else if (t < 0) {
        *p = a.data;
        *n = 0;
    } else {
        *p = a.data + a.head + (uint64_t)t * a.chunk;
        *n = *last ? a.last : a.chunk;
    }
}

// The first round of a launch: -1 when the head has a slot of its own before
// group S - 1's first round (D = 0, head not merged).
template <typename A>
__device__ __forceinline__ int long_first_round(const A& a) {
    return (a.lead == 0 && !(PCRC_LONG_MERGE_HEAD && a.nchunks > 0)) ? -1 : 0;
}

// Every wave: its workgroup's value (after the wave and workgroup factors),
// valid on lane 0 of wave 0 and written through long_reduce. `acc` is the
// group's Horner value (valid on every lane of the group), `lastc` the last
// body chunk's CRC where this group holds it (else 0). STAMP / ABL: as
// long_run. W is the CRC word type (uint32_t here; crc64_kernels.h has its
// own).
template <int G, bool STAMP = false, int ABL = 0>
__device__ __forceinline__ void long_finish(const LongArgs& a, uint32_t acc, uint32_t lastc, uint32_t bw_x,
                                            uint32_t bw_z, uint32_t bw_f, uint32_t* red) {
    const uint32_t lane = threadIdx.x & 63u, wave = wave_id(), l32 = lane & 31u;
    uint32_t v = acc;
    if constexpr (G == 32) {  // acc_0 * X ^ acc_1: the wave's two groups
        const uint32_t m = mul_lanes(acc, bw_x, l32);
        v = lane < 32 ? m : acc;
        v ^= (uint32_t)__shfl_xor((int)v, 32, 64);
        lastc ^= (uint32_t)__shfl_xor((int)lastc, 32, 64);  // the other group's (one of them is 0)
    }
    if constexpr (!(ABL & 32)) v = mul_lanes(v, bw_z, l32);  // * Z^(15 - w)
    if (lane == 0) {
        red[wave] = v;
        red[kWaves + wave] = lastc;
    }
    __syncthreads();
    if (wave == 0) {
        uint32_t u = 0, e = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            u ^= red[w];
            e ^= red[kWaves + w];
        }
        if constexpr (!(ABL & 32)) u = mul_lanes(u, bw_f, l32);  // * J Y^(grid - 1 - b)
        u ^= e;
        if constexpr (ABL & 16) {
            if (lane == 0) *a.out = u;
        } else if constexpr (ABL & 8) {
            long_reduce_slots<uint32_t, uint32_t (*)(uint32_t), true>(u, a.acc, a.out, [](uint32_t x) { return x; }, a.tbase,
                                                                a.treset);
        } else {
            long_reduce(u, a.acc, a.out, [](uint32_t x) { return x; }, a.tbase, a.treset, a.out_tag);
        }
    }
}

// G lanes per chunk (64: one wavefront; 32: two chunks per wavefront), U rows
// per step. STAMP and ABL are for the bench-only probe (probes.hip): STAMP =
// per-wave s_memrealtime stamps into t (8 words per wave); ABL bits = cost
// attribution, results NOT the CRC unless noted: 8 = the reduce WITH the
// agent-scope release/acquire (correct), 16 = no cross-workgroup reduce
// (each workgroup writes its value), 32 = no wave and workgroup factors.
template <int G, int U, bool STAMP = false, int ABL = 0>
__device__ __forceinline__ void long_run(const LongArgs& a, const LaneConsts& kc, uint32_t* lds, uint32_t* red,
                                         uint64_t* t) {
    uint64_t t0 = 0, c0 = 0, t_tab = 0;
    if constexpr (STAMP) {
        t0 = __builtin_amdgcn_s_memrealtime();
        c0 = __builtin_amdgcn_s_memtime();
    }
    // (Measured and dropped: the batch kernel's overlap here -- the first
    // round's rows issued between the image loads and the LDS writes -- took
    // the long kernel from 99 to 128 VGPRs and was slower at every size: 1 GiB
    // 0.1695 vs 0.1654 ms, 256 MiB 0.0549 vs 0.0530,
    // repo:profiles/r05v_ab_long_overlap.jsonl.)
    load_tables<G>(lds, kc);
    if constexpr (STAMP) t_tab = __builtin_amdgcn_s_memrealtime();
    constexpr int GPW = 64 / G;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = wave_id();
    const uint32_t gl = lane & (G - 1), grp = lane / G;
    const LaneAddr la = lane_addr(lane);
    const uint32_t l32 = lane & 31u;
    const int64_t S = (int64_t)a.stride;
    const int64_t g = ((int64_t)blockIdx.x * kWaves + wave) * GPW + grp;
    // Basis words: X^S and X from the host; Z^(15 - w) and (wave 0) the
    // workgroup factor from the LDS tables here, before any chunk.
    const uint32_t bw_xs = a.xsb[l32];
    const uint32_t bw_x = G == 32 ? a.xb[l32] : 0u;
    const uint32_t bw_z = basis_word_lds(lds, a.zt[wave], l32, la.r4);
    const uint32_t bw_f = wave == 0 ? basis_word_lds(lds, a.ft[blockIdx.x], l32, la.r4) : 0u;
    asm volatile("" ::"v"(bw_z), "v"(bw_f));  // done before the chunk loop (crc64_long_run)
    uint32_t acc = 0, lastc = 0;
    // Rounds; a first round -1 when the head is slot -1 (D = 0: group S-1).
    for (int r = long_first_round(a); r < (int)a.rounds; ++r) {
        const int64_t v = g + (int64_t)r * S;
        const uint8_t* p;
        uint64_t n;
        bool last, head;
        long_slot(a, v, &p, &n, &last, &head);
        const uint32_t seed = head ? a.seed : 0u;  // the head carries the seed
        uint32_t crc = 0;
        if (__ballot(n != 0 || seed != 0))  // a wave with only empty slots skips the round's loads
            crc = buffer_crc<G, U, PCRC_LONG_LEAD>(lds, p, n, seed, gl, la);
        // The last chunk stays out of the Horner fold (it enters with factor
        // 1); keeping a general multiply out of this loop keeps the row loop's
        // schedule (round 3: a 32-step multiply here made the compiler reduce
        // the blocks one at a time).
        const uint32_t m = mul_lanes(acc, bw_xs, l32);  // every lane: the halves stay convergent
        acc = last ? m : m ^ crc;
        lastc = last ? crc : lastc;
    }
    uint64_t t_body = 0;
    if constexpr (STAMP) t_body = __builtin_amdgcn_s_memrealtime();
    long_finish<G, STAMP, ABL>(a, acc, lastc, bw_x, bw_z, bw_f, red);
    if constexpr (STAMP) {
        const uint64_t c1 = __builtin_amdgcn_s_memtime();
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            uint64_t* o = t + 8 * ((uint64_t)blockIdx.x * kWaves + wave);
            o[0] = t0;
            o[1] = t_tab;
            o[2] = t_body;
            o[3] = t1;
            o[4] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
            o[5] = __builtin_amdgcn_s_getreg(20 | (3 << 11));
            o[6] = c0;
            o[7] = c1;
        }
    }
}

template <int G, int U>
__global__ __launch_bounds__(kBlock) void crc32c_long_kernel(LongArgs a, LaneConsts kc) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[lds_bytes_for<G>() / 4];
    __shared__ uint32_t red[2 * kWaves];
    long_run<G, U>(a, kc, lds, red, nullptr);
}

// ------------------------------------------------ one small buffer (latency)
// photon_crc32c_extend_device for buffers whose 16-byte block span is at most
// kSmallBlocks (256 KiB): the reference's small perf shape (128 KiB at buf+1,
// test_checksum.cpp:125-168) and the routed drop-in on a device pointer
// (crc32c.h:30-33) are latency, not bandwidth. Up to kSmallWg workgroups of
// 256 threads, no table prologue: each copies 8.5 KiB of nibble tables from
// a device-resident image built once per device, with its payload loads
// issued right behind the copy. (Round 4's first form was ONE workgroup of
// 1024 threads: 12 µs for 128 KiB, all 131 K lookups on one CU's LDS.)
// Geometry: the block grid [a0, a0 + 16 nb) covers the data from its aligned
// start through its end rounded up to 16 bytes (and at least the 4 seed
// bytes). All threads of the kSmallWg x 256 slots form ONE lane group of
// V = 256 kSmallWg virtual lanes walking rows of V blocks anchored at the END: slot
// vt (workgroup b, wave w, lane l: vt = (4 b + w) 64 + l) takes block
// nb - V (rows - r) + vt in row r (a negative block is a leading zero block,
// which does not change a CRC). Every slot's last block is in the last row,
// V - 1 - vt blocks before the end, so every factor is a constant of the
// layout, independent of the buffer: the lane's x^(32 + 128 (63 - l))
// (nibble tables A_dl, B_dh: Q -> P and the shift inside the wave) and the
// wave's x^(8192 (4 kSmallWg - 1 - (4 b + w))) (basis words from the image). Only the
// workgroups that hold data are launched (the last ones). Masking: bytes
// before the data start and at or after its end are zero, the seed is XORed
// into the data's first 4 bytes; the k zero bytes after the end multiply the
// CRC by x^(8k), undone by x^(-8k) (which also makes a seed over fewer than 4
// data bytes exact: crc32c_extend(D, n, s) = crc(D) ^ s x^(8n)).
// Nibble tables (8 positions x 16 values per multiplier, 512 B): the 64
// lanes of a lookup read one position's 16 words, at most 16 distinct
// addresses in 16 consecutive words: conflict-free with one copy.
// Result: each workgroup's value (all factors applied) goes to slots[b]
// when `slots` is set (the routed drop-in: pinned host memory, the host XORs
// them), else to *out through long_reduce (one workgroup: directly).
constexpr uint32_t kSmallBlocks = 16384;                      // 256 KiB of blocks
// 33 workgroups: V = 8448 virtual lanes, so 128 KiB at ANY alignment with the
// seed's cover (the reference's 128 KiB at buf+1 is 8193 blocks) is one row.
constexpr uint32_t kSmallWg = 33, kSmallLanes = kSmallWg * 256;  // V = 8448 virtual lanes
constexpr uint32_t kSmallRows = (kSmallBlocks + 1 + kSmallLanes - 1) / kSmallLanes;  // 2
// The MID layout (photon_crc32c_extend_device and routed calls over 256 KiB
// up to 16 MiB): the same code with kMidWg = 512 workgroups (two per CU), V =
// 131,072 virtual lanes and up to kMidRows rows per thread. Past 16 MiB the
// long kernel (with its table image and 8 KiB chunks) is as fast or faster
// (repo:profiles/r05v_probe_mid.jsonl, µs per call queued: 16 MiB 9.18 vs
// 9.32, 32 MiB 13.33 vs 10.03; CRC-64 16 MiB 10.79 vs 10.74); before the
// image it had ≈17 µs of fixed cost (r05n: 1 MiB 19.1 µs against 5.2).
constexpr uint32_t kMidWg = 512, kMidLanes = kMidWg * 256, kMidRows = 8;
constexpr uint32_t kMidBlocks = kMidRows * kMidLanes;         // 1,048,576 blocks: 16 MiB
constexpr uint32_t kNib = 512;                                // bytes of one nibble-sliced multiplier
// D_j: x^(32 j), j = 1..3 (a block's lagged CRC in ONE table step, not three
// dependent ones), S: one row of the small layout, A_dl, B_dh: the lane's
// finish, S2: one row of the mid layout.
constexpr uint32_t kSmD = 0, kSmS = 3 * kNib, kSmA = 4 * kNib, kSmB = kSmA + 8 * kNib, kSmS2 = kSmB + 7 * kNib;
constexpr uint32_t kSmLds = kSmS2 + kNib;                     // 10,240 B of tables in LDS
// 4 kMidWg x 32 words: basis of x^(8192 d), d = the waves after this one in
// its layout (4 kSmallWg - 1 - wave, or 4 kMidWg - 1 - wave)
constexpr uint32_t kSmWave = kSmLds;
constexpr uint32_t kSmTail = kSmWave + 4u * kMidWg * 32u * 4u;  // 32 x 32 words: basis of x^(-8 k), k < 32
constexpr uint32_t kSmImage = kSmTail + 32u * 32u * 4u;       // bytes of the device image

struct SmallArgs {
    const uint8_t* a0;   // aligned start (data start & ~15)
    const uint32_t* image;
    uint32_t* out;       // the CRC (device), through long_reduce when grid > 1
    uint32_t* slots;     // or: workgroup b's value at slots[b] (mapped host memory), out unused
    uint32_t* acc;       // long_reduce state (grid > 1, slots == nullptr)
    uint64_t tbase;      // long_reduce ticket base
    uint32_t treset;
    uint32_t nb;         // blocks of the grid, <= kSmallBlocks + 1
    uint32_t s0;         // data start - a0 (0..15)
    uint32_t eoff;       // data end - a0: bytes at or past it are zero
    uint32_t k;          // grid end - data end (0..31): the result is multiplied by x^(-8k)
    uint32_t seed;
    uint32_t wg0;        // workgroup index of blockIdx.x == 0 (kSmallWg - grid)
    uint32_t tag;        // slots mode: nonzero = 64-bit slots {tag, value} stored at system scope (the
                         // host spins on the tags instead of waiting for the stream)
};

// p * K through the nibble-sliced tables of K at T (8 conflict-free lookups).
__device__ __forceinline__ uint32_t nib_mul(const uint32_t* T, uint32_t p) {
    uint32_t v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = T[t * 16 + ((p >> (4 * t)) & 15u)];
    return xor3(xor3(v[0], v[1], v[2]), xor3(v[3], v[4], v[5]), v[6] ^ v[7]);
}

// Bytes of the word at `off` (from a0) at or past `eoff` zeroed (branch-free).
__device__ __forceinline__ uint32_t tail_word(uint32_t w, int off, int eoff) {
    const int m = eoff - off;                  // data bytes of this word
    const int mc = m < 0 ? 0 : m > 4 ? 4 : m;
    return mc == 4 ? w : w & (uint32_t)((1ull << (8 * mc)) - 1ull);
}

// One 16-byte block's lagged CRC (block b of the grid, bytes w): masks and
// the seed at the buffer's ends. lag16: D(D(D(w0) ^ w1) ^ w2) ^ w3 = w0 x^96
// ^ w1 x^64 ^ w2 x^32 ^ w3.
__device__ __forceinline__ uint32_t small_lag(const SmallArgs& a, const uint32_t* lds, uint4 v, int b) {
    if (b <= 1 || b >= (int)a.nb - 2) {  // the head's and the tail's blocks: masks + seed
        const int off = b * 16;
        v.x = head_word_sel(tail_word(v.x, off, (int)a.eoff), off, (int)a.s0, a.seed);
        v.y = head_word_sel(tail_word(v.y, off + 4, (int)a.eoff), off + 4, (int)a.s0, a.seed);
        v.z = head_word_sel(tail_word(v.z, off + 8, (int)a.eoff), off + 8, (int)a.s0, a.seed);
        v.w = head_word_sel(tail_word(v.w, off + 12, (int)a.eoff), off + 12, (int)a.s0, a.seed);
        if (b < 0) v = make_uint4(0, 0, 0, 0);
    }
    return xor3(nib_mul(lds + (kSmD + 2 * kNib) / 4, v.x), nib_mul(lds + (kSmD + kNib) / 4, v.y),
                nib_mul(lds + kSmD / 4, v.z)) ^ v.w;
}

// Q -> the wave's value: x^(32 + 128 dl), then x^(1024 dh) (d = 63 - lane:
// Q -> P and the shift to the end of the wave), the 64-lane XOR and the
// wave's factor x^(8192 (V / 64 - 1 - (4 wg + wave))) (bw_wave).
template <typename Stamp>
__device__ __forceinline__ uint32_t small_finish(const uint32_t* lds, uint32_t q, uint32_t bw_wave, Stamp stamp) {
    const uint32_t lane = threadIdx.x & 63u, l32 = lane & 31u;
    const uint32_t d = 63u - lane, dh = d >> 3;
    const uint32_t x = nib_mul(lds + (kSmA + (d & 7u) * kNib) / 4, q);
    const uint32_t y = nib_mul(lds + (kSmB + (dh ? dh - 1u : 0u) * kNib) / 4, x);
    stamp(10, y);
    uint32_t v = group_xor<64>(dh ? y : x);
    stamp(11, v);
    v = mul_lanes(v, bw_wave, l32);
    stamp(12, v);
    return v;
}

// Steps 2-3 of one wave's share (blocks w[] loaded for virtual lane vt, the
// tables at lds): the column, the shift to the end of the wave and the
// wave's factor (bw_wave): the wave's value, on every lane.
template <uint32_t V, int R>
__device__ __forceinline__ uint32_t small_wave_value(const SmallArgs& a, const uint32_t* lds, const uint4 (&w)[R],
                                                     uint32_t vt, uint32_t bw_wave, uint64_t* ts = nullptr) {
    auto stamp = [&](int i, uint32_t dep) {  // bench-only builds (PCRC_SVC_STAMP): time after `dep` is known
        if (PCRC_SVC_STAMP && ts) {
            asm volatile("" ::"v"(dep));
            ts[i] = __builtin_amdgcn_s_memrealtime();
        }
    };
    // uniform (a scalar branch below): rows past the last are not computed
    const uint32_t rows = __builtin_amdgcn_readfirstlane((a.nb + V - 1) / V);
    const int first = (int)a.nb - (int)(rows * V) + (int)vt;  // this thread's block in row 0
    // 2. The column: lagged blocks (independent per row) and the row shift.
    // A wave64 VALU instruction takes 4 cycles on a SIMD16: at 1-3 rows per
    // thread the column is most of a small call's device time, so a row that
    // does not exist costs nothing (PCRC_SVC_STAMP probe: 1.0 µs for 3 rows).
    uint32_t c[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        c[r] = 0;
        if ((uint32_t)r >= rows) continue;
        c[r] = small_lag(a, lds, w[r], first + r * (int)V);
    }
    stamp(8, c[0] ^ c[R - 1]);
    constexpr uint32_t kRow = (V == kSmallLanes ? kSmS : kSmS2) / 4;  // the row shift x^(128 V)
    uint32_t q = c[0];
#pragma unroll
    for (int r = 1; r < R; ++r)
        if ((uint32_t)r < rows) q = nib_mul(lds + kRow, q) ^ c[r];
    stamp(9, q);
    // 3. Q -> P, the shift to the end of the wave, the wave's factor.
    return small_finish(lds, q, bw_wave, stamp);
}

// The workgroup's value (small_wave_value of its 4 waves XORed, times the
// tail factor bw_tail), valid on wave 0 (every lane); one barrier.
template <uint32_t V, int R>
__device__ __forceinline__ uint32_t small_value(const SmallArgs& a, const uint32_t* lds, const uint4 (&w)[R],
                                                uint32_t vt, uint32_t bw_wave, uint32_t bw_tail, uint32_t* red,
                                                uint64_t* ts = nullptr) {
    const uint32_t lane = threadIdx.x & 63u, wave = wave_id(), l32 = lane & 31u;
    const uint32_t v = small_wave_value<V, R>(a, lds, w, vt, bw_wave, ts);
    if (lane == 0) red[wave] = v;
    __syncthreads();
    uint32_t u = 0;
    if (wave == 0) {
        u = red[0] ^ red[1] ^ red[2] ^ red[3];
        u = mul_lanes(u, bw_tail, l32);  // x^(-8k): the zero bytes after the end (linear: per workgroup)
    }
    return u;
}

// 16 bytes with agent-scope loads that skip the CU's L1 (two 8-byte global_
// loads, not flat_).
__device__ __forceinline__ uint4 load16_coherent(const uint8_t* p) {
    typedef __attribute__((address_space(1))) const uint64_t g_u64;
    g_u64* q = (g_u64*)p;
    const uint64_t lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

// The service takes calls of up to kSvcRows rows of its layout (≈2 MiB).
constexpr uint32_t kSvcRows = 16;
constexpr uint32_t kSvcMaxBlocks = kSvcRows * kSmallLanes;  // 135,168 blocks (2.06 MiB)

// This thread's blocks: only blocks that overlap the data are read (a block
// at or past the end -- the seed's cover, n = 0 -- is all masked bytes, and
// may lie on an unmapped page). COHERENT: agent-scope loads that
// skip the CU's L1 (the resident service below reads buffers that other
// launches rewrite between its requests); else nontemporal loads.
template <bool COHERENT, uint32_t V, int R, typename A>
__device__ __forceinline__ void small_load(const A& a, uint32_t vt, uint4 (&w)[R]) {
    const uint32_t rows = __builtin_amdgcn_readfirstlane((a.nb + V - 1) / V);
    const int first = (int)a.nb - (int)(rows * V) + (int)vt;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int b = first + r * (int)V;
        w[r] = make_uint4(0, 0, 0, 0);
        if ((uint32_t)r < rows && b >= 0 && 16u * (uint32_t)b < a.eoff) {
            const uint8_t* p = a.a0 + 16 * (uint32_t)b;
            if constexpr (COHERENT) {
                w[r] = load16_coherent(p);
            } else {
                w[r] = load16(p);
            }
        }
    }
}

// V = kSmallLanes, R = kSmallRows: the small layout; V = kMidLanes, R =
// kMidRows: the mid layout (the same steps; 512 workgroups, a row shift of its
// own, long_reduce over up to 512 workgroup values).
template <uint32_t V, int R>
__global__ __launch_bounds__(256) void crc32c_small_kernel(SmallArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kSmLds / 4];
    __shared__ uint32_t red[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id(), l32 = lane & 31u;
    const uint32_t wg = a.wg0 + blockIdx.x;               // position in the layout
    const uint32_t vt = wg * 256u + tid;                   // virtual lane
    // 1. The table copy first (vmcnt counts in issue order), then the payload
    //    rows, then the basis words this thread needs at the end.
    constexpr uint32_t kVec = kSmLds / 16;  // 640 16-byte pieces
    static_assert(kVec <= 3 * 256, "table copy: 3 pieces per thread");
    u32x4 tv[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const uint32_t j = (uint32_t)i * 256u + tid;
        tv[i] = j < kVec ? *((const g_u32x4*)a.image + j) : u32x4{0, 0, 0, 0};
    }
    uint4 w[R];
    small_load<false, V>(a, vt, w);
    const uint32_t bw_wave = a.image[kSmWave / 4 + (V / 64u - 1u - (wg * 4u + wave)) * 32u + l32];
    const uint32_t bw_tail = a.image[kSmTail / 4 + a.k * 32u + l32];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const uint32_t j = (uint32_t)i * 256u + tid;
        if (j < kVec) *reinterpret_cast<u32x4*>(lds + 4 * j) = tv[i];
    }
    lds_barrier();
    const uint32_t u = small_value<V, R>(a, lds, w, vt, bw_wave, bw_tail, red);
    if (wave == 0) {
        if (a.slots) {
            if (lane == 0) {
                if (a.tag)  // one 8-byte store: the host never sees a tag without its value
                    __hip_atomic_store(reinterpret_cast<uint64_t*>(a.slots) + blockIdx.x,
                                       (uint64_t)a.tag << 32 | u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                else
                    a.slots[blockIdx.x] = u;
            }
        } else {
            long_reduce(u, a.acc, a.out, [](uint32_t x) { return x; }, a.tbase, a.treset, a.tag);
        }
    }
}

// The resident small-buffer service (routed drop-in calls of up to 2 MiB,
// on by default once device dispatch is on, photon_crc_set_small_service;
// CRC-64: crc64_kernels.h crc64_small_service_kernel). A launch of kSmallWg workgroups that stays on
// the chip between calls: the tables and the basis words are loaded ONCE,
// and a call costs no launch -- the host writes the request into the
// doorbell, wave 0 of every workgroup polls it and hands it to its
// workgroup through LDS, the workgroup computes its share of the layout
// exactly as the small kernel (small_value) and stores its tagged value into
// its own slot in pinned host memory; the host XORs the slots. No GPU-side
// ordering across workgroups is needed (the host collects). One slot per
// workgroup, each on a 64-byte line of its own: 8-byte writes of 128 waves
// into 16 shared lines cost ~5 µs more at 128 KiB than 32 workgroup slots
// (the host link serialises partial writes to one line).
//
// The doorbell (64-bit words; DEVICE memory the host writes through the PCIe
// BAR on large-BAR systems -- the device polls it in 0.2-0.4 µs instead of
// 1.2-2.8 µs over the host link, repo:profiles/r05h_doorbell_probe.jsonl --
// else pinned host memory):
//   0-5  the request, each word {seq (high 32), field (low 32)}: a0 low, a0
//        high, nb | s0 << 20 | k << 24, eoff | wg0 << 26, seed low, seed high
//        (CRC-64: the inverted init). A request is taken when all six carry
//        one seq that is not the last one served (the host writes the words
//        in any order; a torn read retries);
//   6    stop (host -> device): nonzero ends the service;
//   7    quit: set by workgroup 0 when it ends the service (idle for `idle`
//        ticks of the 100 MHz clock, or `life` ticks old), here for the other
//        workgroups and in the pinned area's word 7 for the host, which then
//        starts a new launch for later calls.
// Pinned area: word 7 quit (above); 16 + 8 b: slot of workgroup b, {seq,
// value} (CRC-64: {seq, low}, {seq, high}); 16 + 8 b + 3: workgroup b left.
// A poll finds nothing for kSvcNapTicks: wave 0 sleeps ~0.3 µs (s_sleep)
// before each further poll until the next request, so an idle launch neither
// streams doorbell reads nor keeps its SIMD's issue port busy (a request after
// such a pause is seen at most one nap later).
// Every wave exits: workgroup 0 on stop / idle / life, the others on stop,
// quit or 2 x life by their own clock (a workgroup 0 that never became
// resident cannot keep them alive). The decision is per workgroup (wave 0's,
// through LDS): all four waves always take the same path, so a workgroup
// barrier inside the work never misses a wave. The request's bytes are read
// with agent-scope loads (small_load<true>): a buffer rewritten by another
// launch since this one last read it must not come from this CU's L1.
constexpr uint32_t kSvcStop = 6, kSvcQuit = 7, kSvcSlots = 16, kSvcSlotStride = 8;  // one 64-byte line per slot
constexpr uint32_t kSvcExitWord = 3;  // word 3 of a workgroup's slot line: set as the workgroup leaves
constexpr uint32_t kSvcWords = kSvcSlots + kSvcSlotStride * kSmallWg;
constexpr uint32_t kSvcLds = kSmLds + 32u * 32u * 4u;  // the tables, then the tail basis words
constexpr uint64_t kSvcNapTicks = 2000;  // 20 µs of the 100 MHz clock without a request: nap between polls

struct ServiceArgs {
    const void* image;  // the small kernel's image (tables, wave and tail basis words)
    uint64_t* bell;     // the doorbell (device view)
    uint64_t* area;     // the pinned area (device view)
    uint32_t last;      // the seq served last (by an earlier launch): not served again
    uint32_t idle;      // ticks without a request before workgroup 0 ends the service
    uint32_t life;      // ticks after which workgroup 0 ends it
};

// One request as the doorbell carries it.
struct SvcReq {
    const uint8_t* a0;
    uint32_t nb, s0, k, wg0, eoff, seq;
    uint64_t seed;
};

// The poll loop of both services: work(req) for each request whose part of
// the layout has data in this workgroup. st (PCRC_SVC_STAMP builds): stamps
// 0 poll issue, 1 seen (realtime), 6 seen (shader cycles) of the request.
template <typename Work>
__device__ __forceinline__ void service_loop(const ServiceArgs& s, uint32_t (&cmd)[2][8], uint64_t* st, Work work) {
    const uint32_t lane = threadIdx.x & 63u, wave = wave_id(), wg = blockIdx.x;
    uint32_t last = s.last;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t tl = t0;
    bool nap = false;  // wave 0: the last poll found nothing for kSvcNapTicks
    for (uint32_t round = 0;; ++round) {
        uint32_t* c = cmd[round & 1u];
        if (wave == 0) {
            if (nap) __builtin_amdgcn_s_sleep(10);  // 640 cycles
            const uint64_t t_issue = __builtin_amdgcn_s_memrealtime();
            const uint64_t v = lane <= kSvcQuit ? __hip_atomic_load(s.bell + lane, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_SYSTEM)
                                                : 0ull;
            const uint32_t seq = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
            const bool same = lane >= kSvcStop || (uint32_t)(v >> 32) == seq;
            const bool fresh = __ballot(same) == ~0ull && seq != last;
            const bool stop = __shfl(v, kSvcStop) != 0 || __shfl(v, kSvcQuit) != 0;
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            uint32_t cm = fresh ? 1u : 0u;
            if (stop) {
                cm = 2u;
            } else if (!fresh) {
                if (wg == 0 && (now - tl > s.idle || now - t0 > s.life)) {
                    cm = 2u;
                    if (lane == 0) {
                        __hip_atomic_store(s.bell + kSvcQuit, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        __hip_atomic_store(s.area + kSvcQuit, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                } else if (now - t0 > 2ull * s.life) {
                    cm = 2u;
                }
            }
            nap = !fresh && now - tl > kSvcNapTicks;
            if (fresh) {
                last = seq;
                tl = now;
                if (PCRC_SVC_STAMP && st) {
                    st[0] = t_issue;
                    st[1] = now;
                    st[6] = __builtin_amdgcn_s_memtime();
                }
            }
            if (lane < kSvcStop) c[lane] = (uint32_t)v;
            if (lane == 0) {
                c[6] = seq;
                c[7] = cm;
            }
        }
        __syncthreads();
        const uint32_t cm = c[7];
        if (cm == 2u) break;
        if (cm == 0u) continue;
        SvcReq r;
        r.a0 = reinterpret_cast<const uint8_t*>((uint64_t)c[1] << 32 | c[0]);
        r.nb = c[2] & 0xfffffu;
        r.s0 = (c[2] >> 20) & 15u;
        r.k = (c[2] >> 24) & 31u;
        r.eoff = c[3] & 0x3ffffffu;
        r.wg0 = c[3] >> 26;
        r.seed = (uint64_t)c[5] << 32 | c[4];
        r.seq = c[6];
        if (wg < r.wg0) continue;  // no data in this workgroup's part of the layout
        work(r);
    }
    // the host's process-exit path waits for these instead of the stream (no
    // HIP call at exit: a profiler's exit hooks may have run before it)
    if (wave == 0 && lane == 0)
        __hip_atomic_store(s.area + kSvcSlots + kSvcSlotStride * wg + kSvcExitWord, 1ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void crc32c_small_service_kernel(ServiceArgs s) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kSvcLds / 4];
    __shared__ uint32_t cmd[2][8];  // per poll parity: request words 0-5, seq, command
    __shared__ uint32_t red[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id(), l32 = lane & 31u;
    const uint32_t wg = blockIdx.x, vt = wg * 256u + tid;
    const uint32_t* image = static_cast<const uint32_t*>(s.image);
    for (uint32_t j = tid; j < kSmLds / 16; j += 256u)
        *reinterpret_cast<u32x4*>(lds + 4 * j) = *((const g_u32x4*)image + j);
    for (uint32_t j = tid; j < 32u * 32u / 4u; j += 256u)
        *reinterpret_cast<u32x4*>(lds + kSmLds / 4 + 4 * j) = *((const g_u32x4*)(image + kSmTail / 4) + j);
    const uint32_t bw_wave = image[kSmWave / 4 + (4u * kSmallWg - 1u - (wg * 4u + wave)) * 32u + l32];
    __syncthreads();
    uint64_t st[16] = {};  // PCRC_SVC_STAMP builds: 0-7 service_loop / below, 8-12 inside small_wave_value
    service_loop(s, cmd, PCRC_SVC_STAMP ? st : nullptr, [&](const SvcReq& r) {
        SmallArgs a{};
        a.a0 = r.a0;
        a.nb = r.nb;
        a.s0 = r.s0;
        a.k = r.k;
        a.eoff = r.eoff;
        a.seed = (uint32_t)r.seed;
        if (PCRC_SVC_STAMP) st[2] = __builtin_amdgcn_s_memrealtime();
        const uint32_t bw_tail = lds[kSmLds / 4 + a.k * 32u + l32];
        uint32_t u;
        if (a.nb > kSmallRows * kSmallLanes) {  // uniform: a call of up to kSvcRows rows
            uint4 w[kSvcRows];
            small_load<true, kSmallLanes>(a, vt, w);
            u = small_value<kSmallLanes, kSvcRows>(a, lds, w, vt, bw_wave, bw_tail, red);
        } else {
            uint4 w[kSmallRows];
            small_load<true, kSmallLanes>(a, vt, w);
            if (PCRC_SVC_STAMP) {
                __builtin_amdgcn_s_waitcnt(0);
                st[3] = __builtin_amdgcn_s_memrealtime();
            }
            u = small_value<kSmallLanes, kSmallRows>(a, lds, w, vt, bw_wave, bw_tail, red,
                                                     PCRC_SVC_STAMP ? st : nullptr);
        }
        if (PCRC_SVC_STAMP && wave == 0) {
            asm volatile("" ::"v"(u));
            st[4] = st[5] = __builtin_amdgcn_s_memrealtime();
            st[7] = __builtin_amdgcn_s_memtime();
            if (lane < 16) {
                uint64_t x = st[0];
#pragma unroll
                for (int i = 1; i < 16; ++i) x = lane == (uint32_t)i ? st[i] : x;
                __hip_atomic_store(s.area + kSvcWords + 16 * wg + lane, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        if (wave == 0 && lane == 0)
            __hip_atomic_store(s.area + kSvcSlots + kSvcSlotStride * wg, (uint64_t)r.seq << 32 | u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    });
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
// the CRC kernels' own access pattern with the CRC replaced by an XOR --
// persistent 1024-thread workgroups, each wave sweeping contiguous 64 KiB
// pieces in rows of 1 KiB (one 16-byte nontemporal load per lane), 4 rows
// per step with the next 4 in flight. (Round 1-4's grid-stride form, 8 loads
// per thread 8 MiB apart, read at only ~69 % of 8 TB/s, below the CRC
// kernels themselves) Every byte is read once; the XOR keeps the
// loads live.
constexpr uint64_t kStreamPiece = 64u << 10;
__global__ __launch_bounds__(kBlock) void read_stream_kernel(const uint8_t* p, uint64_t nbytes, uint32_t* sink) {
    constexpr int U = 4;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
    const uint64_t pieces = nbytes / kStreamPiece;
    uint32_t acc = 0;
    for (uint64_t w = (uint64_t)blockIdx.x * kWaves + wave_id(); w < pieces; w += nwaves) {
        const uint8_t* q = p + w * kStreamPiece + 16u * lane;
        uint4 cur[U];
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = load16(q + u * 1024u);
        for (uint32_t r = U; r < kStreamPiece / 1024u; r += U) {
            uint4 nxt[U];
#pragma unroll
            for (int u = 0; u < U; ++u) nxt[u] = load16(q + (r + u) * 1024u);
#pragma unroll
            for (int u = 0; u < U; ++u) acc ^= xor3(cur[u].x, cur[u].y, cur[u].z) ^ cur[u].w;
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = nxt[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= xor3(cur[u].x, cur[u].y, cur[u].z) ^ cur[u].w;
    }
    // the bytes past the last whole piece: 16-byte words, grid-stride
    const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    for (uint64_t i = pieces * kStreamPiece / 16 + tid; i < nbytes / 16; i += (uint64_t)gridDim.x * kBlock) {
        const uint4 v = load16(p + 16 * i);
        acc ^= xor3(v.x, v.y, v.z) ^ v.w;
    }
    sink[tid] = acc;
}

}  // namespace pcrc
