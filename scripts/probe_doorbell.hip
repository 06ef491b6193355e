// probe_doorbell.hip -- bench-only probe for the resident small-buffer
// service's request path: host -> device -> host ping-pong latency with the
// request word (a) in pinned host memory (the device polls it over the host
// link) and (b) in fine-grained / uncached DEVICE memory that the host writes
// through the BAR (large-BAR systems), the answer always in pinned host
// memory. One workgroup of one wave polls; `pollers` extra workgroups poll
// the same word to show contention. Prints one JSON line per case.
//   hipcc --offload-arch=gfx950 -O2 -o ab/probe_doorbell scripts/probe_doorbell.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

__global__ void pong(const uint64_t* bell, uint64_t* ack, uint32_t rounds, uint32_t lanes) {
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t want = 1;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (want <= rounds) {
        const uint64_t v = lane < lanes ? __hip_atomic_load(bell + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                        : 0ull;
        const uint64_t v0 = __shfl(v, 0);
        if (v0 == want) {
            if (blockIdx.x == 0 && lane == 0)
                __hip_atomic_store(ack, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            ++want;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;  // 2 s: every wave leaves
    }
}

// The service's shape: 256-thread workgroups, wave 0 polls, a workgroup
// barrier every round; the successful poll's issue -> return time stamped.
__global__ __launch_bounds__(256) void pong_wg(const uint64_t* bell, uint64_t* ack, uint32_t rounds, uint32_t lanes,
                                               uint64_t* rt) {
    __shared__ uint32_t cmd[2];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint64_t want = 1;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t round = 0;; ++round) {
        if (wave == 0) {
            const uint64_t ti = __builtin_amdgcn_s_memrealtime();
            const uint64_t v = lane < lanes ? __hip_atomic_load(bell + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                            : 0ull;
            const uint64_t v0 = __shfl(v, 0);
            const uint64_t tn = __builtin_amdgcn_s_memrealtime();
            uint32_t c = 0;
            if (v0 == want) {
                if (blockIdx.x == 0 && lane == 0) {
                    __hip_atomic_store(ack, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    rt[want & 4095] = tn - ti;
                }
                c = 1;
            }
            if (want > rounds || tn - t0 > 200000000ull) c = 2;
            if (lane == 0) cmd[round & 1] = c;
        }
        __syncthreads();
        const uint32_t c = cmd[round & 1];
        if (c == 2) break;
        if (c == 1) ++want;
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int run(const char* name, uint64_t* bell_host, const uint64_t* bell_dev, uint64_t* ack_h, uint64_t* ack_d,
               int blocks, uint32_t lanes, bool wg = false, uint64_t* rt_h = nullptr, uint64_t* rt_d = nullptr) {
    const uint32_t rounds = 2000;
    for (uint32_t i = 0; i < 64; ++i) __atomic_store_n(bell_host + i, 0ull, __ATOMIC_RELEASE);
    __atomic_store_n(ack_h, 0ull, __ATOMIC_RELEASE);
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
    if (wg)
        hipLaunchKernelGGL(pong_wg, dim3(blocks), dim3(256), 0, st, bell_dev, ack_d, rounds, lanes, rt_d);
    else
        hipLaunchKernelGGL(pong, dim3(blocks), dim3(64), 0, st, bell_dev, ack_d, rounds, lanes);
    std::vector<double> lat;
    for (uint32_t r = 1; r <= rounds; ++r) {
        const double t0 = now_us();
        for (uint32_t i = 0; i < lanes; ++i) __atomic_store_n(bell_host + i, (uint64_t)r, __ATOMIC_RELEASE);
        __builtin_ia32_sfence();  // write-combined BAR mappings hold stores until flushed
        const volatile uint64_t* a = ack_h;
        while (*a != r)
            if (now_us() - t0 > 1e6) {
                printf("{\"case\": \"%s\", \"error\": \"no ack at round %u\"}\n", name, r);
                (void)hipStreamSynchronize(st);
                return 1;
            }
        lat.push_back(now_us() - t0);
    }
    (void)hipStreamSynchronize(st);
    (void)hipStreamDestroy(st);
    std::sort(lat.begin(), lat.end());
    double grt = 0;
    if (wg && rt_h) {
        std::vector<uint64_t> v(rt_h + 1, rt_h + 1 + std::min<uint32_t>(rounds, 4095));
        std::sort(v.begin(), v.end());
        grt = v[v.size() / 2] / 100.0;
    }
    printf("{\"case\": \"%s\", \"wg256\": %d, \"blocks\": %d, \"lanes\": %u, \"us_median\": %.2f, \"us_p10\": %.2f, "
           "\"us_p90\": %.2f, \"gpu_poll_rt_us\": %.2f}\n",
           name, (int)wg, blocks, lanes, lat[lat.size() / 2], lat[lat.size() / 10], lat[lat.size() * 9 / 10], grt);
    fflush(stdout);
    return 0;
}

int main() {
    int lb = -1;
    (void)hipDeviceGetAttribute(&lb, hipDeviceAttributeIsLargeBar, 0);
    printf("{\"large_bar\": %d}\n", lb);
    uint64_t *ph = nullptr, *pd = nullptr, *ah = nullptr, *ad = nullptr;
    if (hipHostMalloc((void**)&ah, 4096, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 2;
    (void)hipHostGetDevicePointer((void**)&ad, ah, 0);
    if (hipHostMalloc((void**)&ph, 4096, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 2;
    (void)hipHostGetDevicePointer((void**)&pd, ph, 0);
    uint64_t *rh = nullptr, *rd = nullptr;
    if (hipHostMalloc((void**)&rh, 8 * 4096, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 2;
    (void)hipHostGetDevicePointer((void**)&rd, rh, 0);
    for (int blocks : {1, 32})
        for (uint32_t lanes : {1u, 7u})
            if (run("pinned_host", ph, pd, ah, ad, blocks, lanes)) return 3;
    for (int blocks : {1, 32})
        for (uint32_t lanes : {1u, 7u})
            if (run("pinned_host", ph, pd, ah, ad, blocks, lanes, true, rh, rd)) return 3;
    fflush(stdout);
    for (unsigned flag : {(unsigned)hipDeviceMallocFinegrained, (unsigned)hipDeviceMallocUncached}) {
        uint64_t* dv = nullptr;
        hipError_t e = hipExtMallocWithFlags((void**)&dv, 4096, flag);
        hipPointerAttribute_t at{};
        if (e == hipSuccess) e = hipPointerGetAttributes(&at, dv);
        printf("{\"device_mem_flag\": %u, \"alloc\": \"%s\", \"host_ptr\": \"%p\", \"dev_ptr\": \"%p\"}\n", flag,
               hipGetErrorString(e), at.hostPointer, at.devicePointer);
        fflush(stdout);
        if (e != hipSuccess || lb != 1) continue;
        uint64_t* hv = at.hostPointer ? (uint64_t*)at.hostPointer : dv;
        // a host write and read through the BAR (a crash here = not mapped for the host)
        __atomic_store_n(hv, 0x5eedull, __ATOMIC_RELEASE);
        uint64_t back = 0;
        (void)hipMemcpy(&back, dv, 8, hipMemcpyDeviceToHost);
        printf("{\"device_mem_flag\": %u, \"host_write_seen_by_copy\": %s}\n", flag, back == 0x5eedull ? "true" : "false");
        fflush(stdout);
        if (back != 0x5eedull) continue;
        for (int blocks : {1, 32})
            for (uint32_t lanes : {1u, 7u})
                if (run(flag == hipDeviceMallocFinegrained ? "device_finegrained" : "device_uncached", hv, dv, ah, ad,
                        blocks, lanes, true, rh, rd))
                    return 3;
    }
    return 0;
}
