// routed_latency.cpp -- the reference's latency shape (test_checksum.cpp:
// 125-168: one 128 KiB buffer at buf+1, crc32c_extend in a loop) timed from
// native code, as Photon would call it: the drop-in crc32c_extend on a
// DEVICE pointer (photon_crc_set_device_dispatch), through the launch path
// and through the resident small-buffer service (photon_crc_set_small_service),
// beside the host engine on a host copy of the same bytes. Every routed
// result is checked against the host engine. One JSON line per size.
// Usage: routed_latency [calls]
#include <hip/hip_runtime.h>
#include <photon/common/checksum/crc32c.h>
#include <photon/common/checksum/crc64ecma.h>
#include <photon_crc/crc32c_gpu.h>
#include <photon_crc/tuning.h>

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <vector>

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <typename F>
static double median_us(int calls, F f) {
    std::vector<double> t(calls);
    for (int i = 0; i < calls; ++i) {
        const double t0 = now_us();
        f();
        t[i] = now_us() - t0;
    }
    std::sort(t.begin(), t.end());
    return t[calls / 2];
}

int main(int argc, char** argv) {
    const int calls = argc > 1 ? atoi(argv[1]) : 2000;
    const size_t cap = (16u << 20) + 64;
    std::vector<uint8_t> host(cap);
    uint64_t z = 0x5EED0128;
    for (auto& b : host) {
        z = z * 6364136223846793005ull + 1442695040888963407ull;
        b = (uint8_t)(z >> 56);
    }
    uint8_t* d = nullptr;
    if (hipMalloc((void**)&d, cap) != hipSuccess) return 2;
    if (hipMemcpy(d, host.data(), cap, hipMemcpyHostToDevice) != hipSuccess) return 2;
    int bad = 0;
    for (size_t n : {(size_t)16, (size_t)4096, (size_t)(128u << 10), (size_t)(256u << 10) - 1, (size_t)(1u << 20),
                     (size_t)(4u << 20), (size_t)(16u << 20)}) {
        const uint32_t want = crc32c_extend(host.data() + 1, n, 0);  // host engine (dispatch off)
        photon_crc_set_device_dispatch(1);
        photon_crc_set_small_service(0);
        volatile uint32_t sink = 0;
        const double launch = median_us(calls, [&] { sink = crc32c_extend(d + 1, n, 0); });
        bad += sink != want;
        photon_crc_set_small_service(20000);
        (void)crc32c_extend(d + 1, n, 0);  // starts the service
        uint64_t s0 = 0, s1 = 0;
        photon_crc_small_service_stats(&s0, nullptr, nullptr);
        const double svc = median_us(calls, [&] { sink = crc32c_extend(d + 1, n, 0); });
        photon_crc_small_service_stats(&s1, nullptr, nullptr);
        bad += sink != want;
        photon_crc_set_small_service(0);
        photon_crc_set_device_dispatch(0);
        const double cpu = median_us(calls, [&] { sink = crc32c_extend(host.data() + 1, n, 0); });
        printf("{\"crc\": \"crc32c\", \"bytes\": %zu, \"routed_launch_us\": %.2f, \"routed_service_us\": %.2f, \"service_served\": %llu, "
               "\"host_engine_on_host_copy_us\": %.2f, \"ok\": %s}\n",
               n, launch, svc, (unsigned long long)(s1 - s0), cpu, bad ? "false" : "true");
        fflush(stdout);
    }
    for (size_t n : {(size_t)16, (size_t)(128u << 10)}) {  // crc64ecma_extend (test_checksum.cpp:204-216)
        const uint64_t want = crc64ecma_extend(host.data() + 1, n, 0);
        photon_crc_set_device_dispatch(1);
        photon_crc_set_small_service(0);
        volatile uint64_t sink = 0;
        const double launch = median_us(calls, [&] { sink = crc64ecma_extend(d + 1, n, 0); });
        bad += sink != want;
        photon_crc_set_small_service(20000);
        (void)crc64ecma_extend(d + 1, n, 0);
        const double svc = median_us(calls, [&] { sink = crc64ecma_extend(d + 1, n, 0); });
        bad += sink != want;
        photon_crc_set_small_service(0);
        photon_crc_set_device_dispatch(0);
        const double cpu = median_us(calls, [&] { sink = crc64ecma_extend(host.data() + 1, n, 0); });
        printf("{\"crc\": \"crc64ecma\", \"bytes\": %zu, \"routed_launch_us\": %.2f, \"routed_service_us\": %.2f, "
               "\"host_engine_on_host_copy_us\": %.2f, \"ok\": %s}\n",
               n, launch, svc, cpu, bad ? "false" : "true");
        fflush(stdout);
    }
    photon_crc_set_small_service(200);
    (void)hipFree(d);
    return bad ? 1 : 0;
}
