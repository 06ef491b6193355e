// probes.hip -- bench-only HBM read probes (libphoton_probes.so, NOT part of
// the product). They bound what the CRC kernels can reach on this chip:
//   probe_read_gridstride: plain streaming read, every 16 B read once;
//   probe_read_rows:       the CRC kernels' exact access pattern (one
//                          wavefront per buffer, 16*G-byte rows, persistent
//                          1024-thread workgroups, D rows in flight) with the
//                          CRC arithmetic replaced by an XOR.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_kernels.h"
#include "crc64_kernels.h"
#include "long_plan.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;

template <bool NT>
__device__ __forceinline__ u32x4 ld(const uint8_t* p) {
    if (NT) return __builtin_nontemporal_load((g_u32x4*)p);
    return *(g_u32x4*)p;
}

template <int UNR, bool NT>
__global__ __launch_bounds__(256) void gridstride(const uint8_t* p, uint64_t nvec, uint32_t* sink) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    uint64_t i = tid;
    for (; i + (UNR - 1) * nth < nvec; i += UNR * nth) {
        u32x4 v[UNR];
#pragma unroll
        for (int k = 0; k < UNR; ++k) v[k] = ld<NT>(p + 16 * (i + k * nth));
#pragma unroll
        for (int k = 0; k < UNR; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    for (; i < nvec; i += nth) {
        const u32x4 v = ld<NT>(p + 16 * i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    sink[tid] = acc;
}

// One wave per buffer of `rows` rows of 1 KiB, U rows per step.
template <int U, bool NT>
__global__ __launch_bounds__(1024) void rows_kernel(const uint8_t* base, uint64_t stride, uint64_t rows,
                                                   uint64_t count, uint32_t* sink) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * 16;
    uint32_t acc = 0;
    for (uint64_t b = blockIdx.x * 16ull + wave; b < count; b += nwaves) {
        const uint8_t* p = base + b * stride + 16 * lane;
        for (uint64_t r = 0; r < rows; r += U) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = ld<NT>(p + (r + u) * 1024);
#pragma unroll
            for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        }
    }
    sink[blockIdx.x * 1024ull + threadIdx.x] = acc;
}

// The CRC kernels' lane-group read pattern with the CRC replaced by an XOR:
// G lanes per buffer, 64/G buffers per wave, rows of 16*G bytes, U rows per
// step with the next U in flight (as buffer_crc), persistent 1024-thread
// workgroups, nt loads. What does a buffer size / lane-group geometry read at?
template <int G, int U>
__global__ __launch_bounds__(1024) void group_rows_kernel(const uint8_t* base, uint64_t stride, uint64_t rows,
                                                         uint64_t count, uint32_t* sink, const uint64_t* slot) {
    constexpr int GPW = 64 / G;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gl = lane & (G - 1), grp = lane / G;
    const uint64_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * 16;
    uint32_t acc = 0;
    for (uint64_t wv = blockIdx.x * 16ull + wave; wv * GPW < count; wv += nwaves) {
        const uint64_t b = wv * GPW + grp;
        if (b >= count) continue;
        const uint8_t* p = base + (slot ? slot[b] : b) * stride + 16 * gl;
        uint64_t r = 0;
        u32x4 cur[U];
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = ld<true>(p + (uint64_t)u * 16 * G);
        for (; r + 2 * U <= rows; r += U) {
            u32x4 nxt[U];
#pragma unroll
            for (int u = 0; u < U; ++u) nxt[u] = ld<true>(p + (r + U + u) * 16 * G);
#pragma unroll
            for (int u = 0; u < U; ++u) acc ^= cur[u].x ^ cur[u].y ^ cur[u].z ^ cur[u].w;
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = nxt[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= cur[u].x ^ cur[u].y ^ cur[u].z ^ cur[u].w;
    }
    sink[blockIdx.x * 1024ull + threadIdx.x] = acc;
}

// The generic strided CRC32C kernel (crc32c_batch_kernel's non-message path,
// same buffer_crc) with per-wave timestamps and a choice of task hand-out:
//   MODE 0: static (wave w takes wave tasks w, w + nwaves, ... as the product);
//   MODE 1: every task from one device-scope ticket counter (next ticket
//           fetched before the current task runs);
//   MODE 2: static for the first `static_rounds` rounds, tickets for the rest;
//   MODE 3: as 2 with 8 per-XCC ticket regions and stealing across them;
//   MODE 4: static with the chunk of workgroup b rotated by the round;
//   MODE 5: static, split by XCD parity (workgroup b on XCD b % 8): the
//           even XCDs' waves take the first ntask/2 * (1 + static_rounds/1000)
//           tasks, the odd XCDs' waves the rest (round-robin within each).
// t[6*gw..6*gw+5] = s_memrealtime (100 MHz) at the wave start / end, HW_ID, XCC_ID,
// s_memtime (shader clock) at the wave start / end: the in-kernel clock of a
// wave is d(memtime) / d(memrealtime) x 100 MHz (MI355X_MICROARCH.md, DVFS item 6).
template <int G, int MODE>
__global__ __launch_bounds__(pcrc::kBlock) void crc_wave_times_kernel(pcrc::BatchArgs args, pcrc::LaneConsts kc,
                                                                     uint64_t* t, uint32_t* ticket,
                                                                     uint32_t static_rounds) {
    using namespace pcrc;
    __shared__ __attribute__((aligned(16))) uint32_t lds[lds_bytes_for<G>() / 4];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    build_tables<G>(lds, kc);
    constexpr int GPW = 64 / G;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = wave_id();
    const uint32_t gl = lane & (G - 1);
    const uint32_t grp = lane / G;
    const LaneAddr la = lane_addr(lane);
    const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
    const uint64_t ntask = (args.count + GPW - 1) / GPW;
    const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wave;
    const uint64_t nstatic = (MODE == 0 || MODE == 4) ? ntask : MODE == 1 ? 0 : std::min<uint64_t>(ntask, static_rounds * nwaves);
    // The ticket's atomic is issued one task ahead and read (readfirstlane)
    // only after that task: its return latency hides behind the task's loads.
    auto take = [&]() -> uint32_t { return lane == 0 ? atomicAdd(ticket, 1u) : 0u; };
    auto take_at = [&](uint32_t* c) -> uint32_t { return lane == 0 ? atomicAdd(c, 1u) : 0u; };
    auto value = [&](uint32_t v) -> uint64_t { return nstatic + (uint64_t)__builtin_amdgcn_readfirstlane(v); };
    auto run = [&](uint64_t wv) {
        const uint64_t bi = wv * GPW + grp;
        const bool active = bi < args.count;
        const uint8_t* p = active ? args.base + bi * args.stride : nullptr;
        const uint64_t n = active ? args.nbytes : 0;
        const uint32_t crc = buffer_crc<G, 4>(lds, p, n, args.seed0, gl, la);
        if (active && gl == 0) args.out[bi] = crc;
    };
    if (MODE == 5) {
        const uint64_t half = nwaves / 2;
        const uint64_t par = blockIdx.x & 1u;
        const uint64_t pidx = (uint64_t)(blockIdx.x >> 1) * kWaves + wave;
        uint64_t e = (uint64_t)((double)ntask * 0.5 * (1000.0 + (double)static_rounds) / 1000.0);
        if (e > ntask) e = ntask;
        const uint64_t lo = par ? e : 0, hi = par ? ntask : e;
        for (uint64_t wv = lo + pidx; wv < hi; wv += half) run(wv);
    } else if (MODE == 4) {
        // Static, but workgroup b takes chunk (b + k) % grid in round k, so
        // every XCC (b % 8 under round-robin placement) cycles through every
        // chunk offset instead of always the same ones.
        for (uint64_t k = 0; k * nwaves < ntask; ++k) {
            const uint64_t wv = k * nwaves + ((blockIdx.x + k) % gridDim.x) * kWaves + wave;
            if (wv < ntask) run(wv);
        }
    } else {
        for (uint64_t wv = gw; wv < nstatic; wv += nwaves) run(wv);
    }
    if (MODE == 3) {
        // Tail tasks j = nstatic + x + 8*i in 8 regions x, one ticket counter
        // each (128 B apart); a wave drains its own XCC's region, then the
        // others in order. A relaxed load skips exhausted regions without an
        // atomic; the next ticket is taken one task ahead.
        const uint64_t tail = ntask - nstatic;
        const uint32_t home = __builtin_amdgcn_s_getreg(20 | (3 << 11)) & 7u;
        for (uint32_t r = 0; r < 8; ++r) {
            const uint32_t x = (home + r) & 7u;
            const uint64_t cnt = tail > x ? (tail - x + 7) / 8 : 0;
            uint32_t* ctr = ticket + 32 * x;
            if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= cnt) continue;
            uint64_t c = __builtin_amdgcn_readfirstlane(take_at(ctr));
            while (c < cnt) {
                const uint32_t nx = take_at(ctr);
                run(nstatic + x + 8 * c);
                c = __builtin_amdgcn_readfirstlane(nx);
            }
        }
    } else if (MODE == 1 || MODE == 2) {
        uint64_t wv = value(take());
        while (wv < ntask) {
            const uint32_t nx = take();
            run(wv);
            wv = value(nx);
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        t[6 * gw] = t0;
        t[6 * gw + 1] = t1;
        t[6 * gw + 2] = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_ID: wave, simd, cu, se
        t[6 * gw + 3] = __builtin_amdgcn_s_getreg(20 | (3 << 11));   // XCC_ID
        t[6 * gw + 4] = c0;
        t[6 * gw + 5] = c1;
    }
}

// Per-wave stamps as crc_wave_times_kernel writes them (6 words per wave).
struct WaveStamp {
    uint64_t t0, c0;
    __device__ __forceinline__ WaveStamp() : t0(__builtin_amdgcn_s_memrealtime()), c0(__builtin_amdgcn_s_memtime()) {}
    __device__ __forceinline__ void store(uint64_t* t, uint64_t gw) const {
        const uint64_t c1 = __builtin_amdgcn_s_memtime();
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        if ((threadIdx.x & 63u) == 0) {
            t[6 * gw] = t0;
            t[6 * gw + 1] = t1;
            t[6 * gw + 2] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
            t[6 * gw + 3] = __builtin_amdgcn_s_getreg(20 | (3 << 11));
            t[6 * gw + 4] = c0;
            t[6 * gw + 5] = c1;
        }
    }
};

// DVFS control: the product's read_stream_kernel
// (crc32c_kernels.h, grid-stride, 8 loads in flight per thread) and the CRC
// kernel's own lane-group row pattern (group_rows_kernel) with the same
// per-wave clock stamps as crc_wave_times_kernel, so the ramp of a read-only
// body can be set beside the CRC body's.
__global__ __launch_bounds__(256) void read_stream_stamped_kernel(const uint8_t* p, uint64_t nvec, uint32_t* sink,
                                                                  uint64_t* t) {
    const WaveStamp ws;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    uint64_t i = tid;
    for (; i + 7 * nth < nvec; i += 8 * nth) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = pcrc::load16(p + 16 * (i + k * nth));
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    for (; i < nvec; i += nth) {
        const uint4 v = pcrc::load16(p + 16 * i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    sink[tid] = acc;
    ws.store(t, tid >> 6);
}

template <int G, int U>
__global__ __launch_bounds__(1024) void group_rows_stamped_kernel(const uint8_t* base, uint64_t stride, uint64_t rows,
                                                                 uint64_t count, uint32_t* sink, uint64_t* t) {
    const WaveStamp ws;
    constexpr int GPW = 64 / G;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gl = lane & (G - 1), grp = lane / G;
    const uint64_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * 16;
    uint32_t acc = 0;
    for (uint64_t wv = blockIdx.x * 16ull + wave; wv * GPW < count; wv += nwaves) {
        const uint64_t b = wv * GPW + grp;
        if (b >= count) continue;
        const uint8_t* p = base + b * stride + 16 * gl;
        uint64_t r = 0;
        u32x4 cur[U];
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = ld<true>(p + (uint64_t)u * 16 * G);
        for (; r + 2 * U <= rows; r += U) {
            u32x4 nxt[U];
#pragma unroll
            for (int u = 0; u < U; ++u) nxt[u] = ld<true>(p + (r + U + u) * 16 * G);
#pragma unroll
            for (int u = 0; u < U; ++u) acc ^= cur[u].x ^ cur[u].y ^ cur[u].z ^ cur[u].w;
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = nxt[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= cur[u].x ^ cur[u].y ^ cur[u].z ^ cur[u].w;
    }
    sink[blockIdx.x * 1024ull + threadIdx.x] = acc;
    ws.store(t, blockIdx.x * 16ull + wave);
}

// The product's CRC-64 long and batch kernels with per-wave stamps
// (crc64_kernels.h crc64_long_run / crc64_batch_run, STAMP = true).
template <int G>
__global__ __launch_bounds__(pcrc::kBlock) void crc64_long_stamped_kernel(pcrc::Long64Args a, pcrc::LaneConsts64 kc,
                                                                           uint64_t* t) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[pcrc::k64FLdsBytes / 4];
    __shared__ uint64_t red[2 * pcrc::kWaves];
    pcrc::crc64_long_run<G, true>(a, kc, lds, red, t);
}

template <int G>
__global__ __launch_bounds__(pcrc::kBlock) void crc64_batch_stamped_kernel(pcrc::Batch64Args a, pcrc::LaneConsts64 kc,
                                                                            uint64_t* t) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[pcrc::k64FLdsBytes / 4];
    pcrc::crc64_batch_run<G, true>(a, kc, lds, t);
}

// The product's crc32c_long_kernel<G, 4> (one long buffer, chunks per lane
// group: the same long_run) with 8 stamps per wave: s_memrealtime at the
// start, after the LDS table prologue, after the wave's chunks and after the
// cross-workgroup reduce; HW_ID, XCC_ID, s_memtime at the start and end.
// Attributes a launch's fixed cost (scripts/probe_long_times.py).
// ABL: long_run's cost-attribution bits (crc32c_kernels.h).
template <int G, int ABL>
__global__ __launch_bounds__(pcrc::kBlock) void long_stamped_kernel(pcrc::LongArgs a, pcrc::LaneConsts kc, uint64_t* t) {
    using namespace pcrc;
    __shared__ __attribute__((aligned(16))) uint32_t lds[lds_bytes_for<G>() / 4];
    __shared__ uint32_t red[2 * kWaves];
    long_run<G, 4, true, ABL>(a, kc, lds, red, t);
}

extern "C" {

// read_stream_stamped_kernel: grid = blocks x 256 threads (the product's
// photon_crc_util_read_stream uses cus * 8); t holds 6 words per wave.
int probe_read_stream_stamped(const void* p, uint64_t nbytes, uint32_t* sink, uint64_t* t, int blocks,
                              void* stream) {
    hipLaunchKernelGGL(read_stream_stamped_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<const uint8_t*>(p), nbytes / 16, sink, t);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// group_rows_stamped_kernel<32, 4> (the C2 CRC kernel's pattern): rows of 512 B.
int probe_group_rows_stamped(const void* base, uint64_t stride, uint64_t rows, uint64_t count, uint32_t* sink,
                             uint64_t* t, int blocks, void* stream) {
    hipLaunchKernelGGL((group_rows_stamped_kernel<32, 4>), dim3(blocks), dim3(1024), 0,
                       static_cast<hipStream_t>(stream), static_cast<const uint8_t*>(base), stride, rows, count, sink,
                       t);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// crc_wave_times_kernel over a strided batch; `t` holds 6 * grid * 16 words,
// `ticket` 256 words (zeroed here on the stream before the launch).
int probe_crc_wave_times(const void* base, uint64_t nbytes, uint64_t count, uint32_t* out, uint64_t* t,
                         uint32_t* ticket, int g, int mode, int static_rounds, int cus, void* stream) {
    using namespace pcrc;
    LaneConsts kc;
    kc.kshift = xpow(8ull * 16ull * (uint64_t)g);
    mul_basis(kc.kshift, kc.sbasis);
    for (int k = 0; k < 6; ++k) mul_basis(xpow(128ull << k), kc.basis[k]);
    BatchArgs a{};
    a.base = static_cast<const uint8_t*>(base);
    a.stride = nbytes;
    a.nbytes = nbytes;
    a.count = count;
    a.out = out;
    const uint64_t waves = (count + 64 / g - 1) / (64 / g);
    uint64_t grid = (waves + kWaves - 1) / kWaves;
    if (grid > (uint64_t)cus) grid = cus;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (hipMemsetAsync(ticket, 0, 1024, s) != hipSuccess) return -5;
    const uint32_t sr = (uint32_t)static_rounds;
#define WT(GG, M) \
    hipLaunchKernelGGL((crc_wave_times_kernel<GG, M>), dim3(grid), dim3(kBlock), 0, s, a, kc, t, ticket, sr)
    if (g == 8) {
        if (mode == 1) WT(8, 1); else if (mode == 2) WT(8, 2); else if (mode == 3) WT(8, 3); else if (mode == 4) WT(8, 4); else WT(8, 0);
    } else {
        if (mode == 1) WT(32, 1); else if (mode == 2) WT(32, 2); else if (mode == 3) WT(32, 3); else if (mode == 4) WT(32, 4);
        else if (mode == 5) WT(32, 5); else WT(32, 0);
    }
#undef WT
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int probe_read_gridstride(const void* p, uint64_t nbytes, uint32_t* sink, int blocks, int unroll, int nt,
                          void* stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint8_t* b = static_cast<const uint8_t*>(p);
#define GS(U, N) hipLaunchKernelGGL((gridstride<U, N>), dim3(blocks), dim3(256), 0, s, b, nbytes / 16, sink)
    if (nt) {
        if (unroll == 4) GS(4, true); else if (unroll == 16) GS(16, true); else GS(8, true);
    } else {
        if (unroll == 4) GS(4, false); else if (unroll == 16) GS(16, false); else GS(8, false);
    }
#undef GS
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// group_rows_kernel<G, U> over count buffers of rows*16*G bytes (rows % U == 0).
// slot (optional, device): buffer i is at base + slot[i] * stride (the C5
// layout: segments in a permuted slot pool).
int probe_group_rows_slots(const void* base, uint64_t stride, uint64_t rows, uint64_t count, uint32_t* sink,
                           int blocks, int g, int u, const uint64_t* slot, void* stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint8_t* b = static_cast<const uint8_t*>(base);
#define GR(GG, UU) \
    hipLaunchKernelGGL((group_rows_kernel<GG, UU>), dim3(blocks), dim3(1024), 0, s, b, stride, rows, count, sink, slot)
    if (u == 2) {
        switch (g) { case 4: GR(4, 2); break; case 8: GR(8, 2); break; case 16: GR(16, 2); break; case 32: GR(32, 2); break; default: GR(64, 2); }
    } else if (u == 8) {
        switch (g) { case 4: GR(4, 8); break; case 8: GR(8, 8); break; case 16: GR(16, 8); break; case 32: GR(32, 8); break; default: GR(64, 8); }
    } else {
        switch (g) { case 4: GR(4, 4); break; case 8: GR(8, 4); break; case 16: GR(16, 4); break; case 32: GR(32, 4); break; default: GR(64, 4); }
    }
#undef GR
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int probe_group_rows(const void* base, uint64_t stride, uint64_t rows, uint64_t count, uint32_t* sink, int blocks,
                     int g, int u, void* stream) {
    return probe_group_rows_slots(base, stride, rows, count, sink, blocks, g, u, nullptr, stream);
}

int probe_read_rows(const void* base, uint64_t stride, uint64_t rows, uint64_t count, uint32_t* sink, int blocks,
                    int u, int nt, void* stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint8_t* b = static_cast<const uint8_t*>(base);
#define RK(U, N) hipLaunchKernelGGL((rows_kernel<U, N>), dim3(blocks), dim3(1024), 0, s, b, stride, rows, count, sink)
    if (nt) {
        if (u == 8) RK(8, true); else if (u == 16) RK(16, true); else RK(4, true);
    } else {
        if (u == 8) RK(8, false); else if (u == 16) RK(16, false); else RK(4, false);
    }
#undef RK
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// long_stamped_kernel<lanes> over [data, data + n), cut as the product cuts it
// for photon_crc_set_long_shape(lanes, rounds) (long_plan.h); `state` = 8 + 8
// * kLongMaxGrid bytes, the first 8 zero (left zero); t = 8 words per wave of
// grid * 16 waves; *grid_out = the grid. force_chunk: a chunk size (a 1 KiB
// multiple) instead of the plan's (0 = the plan's). rounds | ablation << 8
// (long_run's ABL bits: 8, 16, 32 and 16|32).
int probe_long_stamped(const void* data, uint64_t n, uint32_t seed, uint32_t* out, uint32_t* state, uint64_t* t,
                       int cus, int lanes, int rounds, uint64_t force_chunk, int* grid_out, void* stream) {
    using namespace pcrc;
    if ((lanes != 64 && lanes != 32) || (rounds & 255) < 1 || (rounds & 255) > 64) return -22;
    if (force_chunk & 1023) return -22;
    const LongPlan lp = long_plan_for(data, n, cus, (uint32_t)lanes | (uint32_t)(rounds & 255) << 8, force_chunk);
    const LongPowers& pw = long_powers(lp, false);
    LongArgs a{};
    long_args(&a, lp, pw, data, seed, out);
    a.acc = state;
    a.treset = 1;  // the caller's zeroed buffer, put back to 0 by every launch
    LaneConsts kc{};
    kc.kshift = xpow(8ull * 16ull * (uint64_t)lp.lanes);
    mul_basis(kc.kshift, kc.sbasis);
    *grid_out = (int)lp.grid;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int abl = rounds >> 8;  // rounds | ablation bits << 8
#define LSK(G, B) hipLaunchKernelGGL((long_stamped_kernel<G, B>), dim3(lp.grid), dim3(kBlock), 0, s, a, kc, t)
#define LSG(B) if (lp.lanes == 64) LSK(64, B); else LSK(32, B)
    switch (abl) {
        case 8: LSG(8); break;
        case 16: LSG(16); break;
        case 32: LSG(32); break;
        case 48: LSG(48); break;
        default: LSG(0); break;
    }
#undef LSG
#undef LSK
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// crc64_long_stamped_kernel over [data, data + n) with the product's plan for
// lanes x rounds (0 x 0: automatic); `state` 8 + 8 * 512 zeroed bytes, `t`
// 8 words per wave of the grid (<= 256 x 16).
int probe_crc64_long_stamped(const void* data, uint64_t n, uint64_t seed, uint64_t* out, uint64_t* state,
                             uint64_t* t, int cus, int lanes, int rounds, int* grid_out, void* stream) {
    using namespace pcrc;
    const LongPlan lp = long_plan_for(data, n, cus, (uint32_t)lanes | (uint32_t)rounds << 8, 0, true);
    const LongPowers& pw = long_powers(lp, true);
    Long64Args a{};
    long_args64(&a, lp, pw, data, seed, out);
    a.acc = state;
    a.treset = 1;
    LaneConsts64 kc{};
    kc.kshift = xpow64(8ull * 16ull * (uint64_t)lp.lanes);
    for (int i = 0; i < 64; ++i) kc.sbasis[i] = mulmod64(1ull << i, kc.kshift);
    *grid_out = (int)lp.grid;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (lp.lanes == 64)
        hipLaunchKernelGGL((crc64_long_stamped_kernel<64>), dim3(lp.grid), dim3(kBlock), 0, s, a, kc, t);
    else
        hipLaunchKernelGGL((crc64_long_stamped_kernel<32>), dim3(lp.grid), dim3(kBlock), 0, s, a, kc, t);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// crc64_batch_stamped_kernel<g> over count strided buffers (one workgroup per
// CU as the product); `t` 8 words per wave.
int probe_crc64_batch_stamped(const void* base, uint64_t nbytes, uint64_t count, uint64_t* out, uint64_t* t, int g,
                              int cus, void* stream) {
    using namespace pcrc;
    if (g != 32 && g != 64) return -22;
    Batch64Args a{};
    a.base = static_cast<const uint8_t*>(base);
    a.stride = nbytes;
    a.nbytes = nbytes;
    a.count = count;
    a.out = out;
    a.seed0 = 0;
    LaneConsts64 kc{};
    kc.kshift = xpow64(8ull * 16ull * (uint64_t)g);
    for (int i = 0; i < 64; ++i) kc.sbasis[i] = mulmod64(1ull << i, kc.kshift);
    const uint64_t waves = (count + 64 / g - 1) / (64 / g);
    uint64_t grid = (waves + kWaves - 1) / kWaves;
    if (grid > (uint64_t)cus) grid = cus;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (g == 64)
        hipLaunchKernelGGL((crc64_batch_stamped_kernel<64>), dim3(grid), dim3(kBlock), 0, s, a, kc, t);
    else
        hipLaunchKernelGGL((crc64_batch_stamped_kernel<32>), dim3(grid), dim3(kBlock), 0, s, a, kc, t);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // extern "C"
