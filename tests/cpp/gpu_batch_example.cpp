// gpu_batch_example.cpp -- the batched C-ABI from plain C++ with hipMalloc
// (no Python, no torch): fill a C2-shaped batch on the device, checksum it with
// photon_crc32c_batch_strided, compare a sample against the drop-in host
// engine crc32c_hw, and time 20 launches. Exit 0 on bit-exact results.
#include <hip/hip_runtime.h>
#include <photon/common/checksum/crc32c.h>
#include <photon_crc/crc32c_gpu.h>

#include <stdio.h>

#include <chrono>
#include <vector>

int main() {
    const uint64_t n = 65536, count = 8192;
    if (photon_crc_device_count() <= 0) {
        fprintf(stderr, "no device: %s\n", photon_crc_last_error());
        return 2;
    }
    void* d_buf = nullptr;
    uint32_t* d_out = nullptr;
    if (hipMalloc(&d_buf, n * count) != hipSuccess || hipMalloc((void**)&d_out, count * 4) != hipSuccess) return 3;
    if (photon_crc_util_fill_splitmix(d_buf, n, n, count, 0x5EED0001, nullptr)) return 4;
    if (photon_crc32c_batch_strided_sync(d_buf, n, n, count, 0, nullptr, d_out, nullptr)) {
        fprintf(stderr, "batch: %s\n", photon_crc_last_error());
        return 5;
    }
    std::vector<uint32_t> out(count);
    std::vector<uint8_t> host(n);
    if (hipMemcpy(out.data(), d_out, count * 4, hipMemcpyDeviceToHost) != hipSuccess) return 6;
    int bad = 0;
    for (uint64_t i = 0; i < count; i += 97) {
        if (hipMemcpy(host.data(), (char*)d_buf + i * n, n, hipMemcpyDeviceToHost) != hipSuccess) return 7;
        if (crc32c(host.data(), n) != out[i]) ++bad;
    }
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < 20; ++r) photon_crc32c_batch_strided(d_buf, n, n, count, 0, nullptr, d_out, nullptr);
    if (hipDeviceSynchronize() != hipSuccess) return 8;
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("gpu_batch_example: %d mismatches, %.1f GB/s\n", bad, 20.0 * n * count / s / 1e9);
    (void)hipFree(d_buf);
    (void)hipFree(d_out);
    return bad ? 1 : 0;
}
