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

extern "C" {

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

// The uniform CRC kernel (G=32, B=1, U=4, D=3) with parts of the arithmetic
// removed (see crc32c_kernels.h ABL): which resource bounds the kernel?
int probe_crc_ablate(const void* base, uint64_t nbytes, uint64_t count, uint32_t* out, int abl, int cus,
                     void* stream) {
    using namespace pcrc;
    constexpr int G = 32;
    LaneConsts kc;
    kc.kshift = xpow(8ull * 16ull * G);
    for (int k = 0; k < 6; ++k) mul_basis(xpow(128ull << k), kc.basis[k]);
    UniformArgs a{static_cast<const uint8_t*>(base), nbytes, nbytes / (16ull * G), count, out};
    const uint64_t waves = (count + 1) / 2;
    uint64_t grid = (waves + 15) / 16;
    if (grid > (uint64_t)cus) grid = cus;
    hipStream_t s = static_cast<hipStream_t>(stream);
#define AB(X) hipLaunchKernelGGL((crc32c_uniform_kernel<G, 1, 4, 3, X>), dim3(grid), dim3(kBlock), 0, s, a, kc)
    switch (abl) {
        case 1: AB(1); break;
        case 2: AB(2); break;
        case 3: AB(3); break;
        case 4: AB(4); break;
        case 5: AB(5); break;
        default: AB(0); break;
    }
#undef AB
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// The CRC-64 streaming kernel (G=32, U=4, D=3) with parts of the arithmetic
// removed: 1 no S lookups, 2 one D step per block, 4 no lookups (and sums).
int probe_crc64_ablate(const void* base, uint64_t nbytes, uint64_t count, uint64_t* out, int abl, int cus,
                       void* stream) {
    using namespace pcrc;
    constexpr int G = 32;
    LaneConsts64 kc;
    kc.kshift = xpow64(8ull * 16ull * G);
    for (int k = 0; k < 6; ++k)
        for (int i = 0; i < 64; ++i) kc.basis[k][i] = mulmod64(1ull << i, xpow64(128ull << k));
    Uniform64Args a{static_cast<const uint8_t*>(base), nbytes, nbytes / (16ull * G), count, out, 0};
    const uint64_t waves = (count + 1) / 2;
    uint64_t grid = (waves + 15) / 16;
    if (grid > (uint64_t)cus) grid = cus;
    hipStream_t s = static_cast<hipStream_t>(stream);
#define AB64(X) hipLaunchKernelGGL((crc64_uniform_kernel<G, 4, 3, 1, 1, X>), dim3(grid), dim3(kBlock), 0, s, a, kc)
    switch (abl) {
        case 1: AB64(1); break;
        case 2: AB64(2); break;
        case 3: AB64(3); break;
        case 4: AB64(4); break;
        case 5: AB64(5); break;
        default: AB64(0); break;
    }
#undef AB64
    return hipGetLastError() == hipSuccess ? 0 : -5;
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

}  // extern "C"
