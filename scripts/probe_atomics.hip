// Probe (bench-only): what one device-scope atomic per
// workgroup on ONE 64-bit word costs a launch, against no atomic and against
// the same atomics spread over 16 words on separate 128-byte lines. G
// workgroups of 256 threads, each does a little LDS work, then wave 0 lane 0
// does `mode`'s atomics: 0 none, 1 fetch_add (returned) on one word, 2
// fetch_xor + fetch_add (returned) on one word (long_reduce_word), 3 mode 2
// on word (b % 16) of 16, then the word's last workgroup adds to a top word
// (two levels). Kernel time from hipEvents over 200 back-to-back launches.
// Build: hipcc --offload-arch=gfx950 -O3 -o ab/probe_atomics scripts/probe_atomics.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void probe(unsigned long long* w, uint32_t mode, uint32_t per) {
    __shared__ uint32_t s[256];
    s[threadIdx.x] = threadIdx.x * 2654435761u;
    __syncthreads();
    uint32_t v = s[(threadIdx.x * 7) & 255];
    if (threadIdx.x == 0 && mode) {
        if (mode == 1) {
            v += (uint32_t)__hip_atomic_fetch_add(w, 1ull << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const uint32_t i = mode == 3 ? (blockIdx.x & 15u) * 16u : 0u;
            (void)__hip_atomic_fetch_xor(w + i, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long old =
                __hip_atomic_fetch_add(w + i, 1ull << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v += (uint32_t)old;
            if (mode == 3 && ((old >> 32) + 1) % per == 0)
                v += (uint32_t)__hip_atomic_fetch_add(w + 256, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (v == 0x12345678u) w[512] = v;  // keep v live
    }
}

int main() {
    unsigned long long* w = nullptr;
    if (hipMalloc(&w, 8192) != hipSuccess) return 1;
    (void)hipMemset(w, 0, 8192);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int reps = 200;
    for (uint32_t g : {33u, 128u, 256u, 512u, 1024u}) {
        float ms[4] = {};
        for (int pass = 0; pass < 2; ++pass)
            for (uint32_t mode = 0; mode < 4; ++mode) {
                hipLaunchKernelGGL(probe, dim3(g), dim3(256), 0, 0, w, mode, (g + 15) / 16);
                (void)hipEventRecord(e0, 0);
                for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(probe, dim3(g), dim3(256), 0, 0, w, mode, (g + 15) / 16);
                (void)hipEventRecord(e1, 0);
                if (hipEventSynchronize(e1) != hipSuccess) return 2;
                (void)hipEventElapsedTime(&ms[mode], e0, e1);
            }
        printf("{\"workgroups\": %u, \"none_us\": %.2f, \"add_one_word_us\": %.2f, \"xor_add_one_word_us\": %.2f, "
               "\"xor_add_16_words_us\": %.2f}\n",
               g, 1000.0 * ms[0] / reps, 1000.0 * ms[1] / reps, 1000.0 * ms[2] / reps, 1000.0 * ms[3] / reps);
        fflush(stdout);
    }
    return 0;
}
