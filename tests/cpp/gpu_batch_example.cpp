// gpu_batch_example.cpp -- the batched C-ABI from plain C++ built with g++ and
// NO HIP headers, the way Photon code would drive it: device memory, a stream,
// the C2-shaped batch, a completion callback (where Photon would signal a
// photon::semaphore), then a sample compared against the drop-in host engine
// crc32c(), and 20 timed launches. Exit 0 on bit-exact results.
#include <photon/common/checksum/crc32c.h>
#include <photon_crc/crc32c_gpu.h>
#include <photon_crc/tuning.h>  // photon_crc_util_fill_splitmix (test data)

#include <stdio.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

static std::atomic<int> g_done{0};
static void on_done(void*) { g_done.fetch_add(1); }  // Photon: sem->signal(1)

#define TRY(x)                                                                  \
    do {                                                                        \
        int rc_ = (x);                                                          \
        if (rc_) {                                                              \
            fprintf(stderr, "%s: %d %s\n", #x, rc_, photon_crc_last_error());  \
            return 3;                                                           \
        }                                                                       \
    } while (0)

int main() {
    const uint64_t n = 65536, count = 8192;
    if (photon_crc_device_count() <= 0) {
        fprintf(stderr, "no device: %s\n", photon_crc_last_error());
        return 2;
    }
    void *d_buf = nullptr, *d_out = nullptr, *stream = nullptr;
    TRY(photon_crc_stream_create(&stream));
    TRY(photon_crc_device_alloc(&d_buf, n * count));
    TRY(photon_crc_device_alloc(&d_out, count * 4));
    TRY(photon_crc_util_fill_splitmix(d_buf, n, n, count, 0x5EED0001, stream));
    TRY(photon_crc32c_batch_strided(d_buf, n, n, count, 0, nullptr, static_cast<uint32_t*>(d_out), stream));
    std::vector<uint32_t> out(count);
    TRY(photon_crc_memcpy_async(out.data(), d_out, count * 4, stream));
    TRY(photon_crc_stream_on_complete(stream, on_done, nullptr));
    while (g_done.load() == 0) std::this_thread::yield();  // Photon: sem.wait(1) parks the photon thread
    std::vector<uint8_t> host(n);
    int bad = 0;
    for (uint64_t i = 0; i < count; i += 97) {
        TRY(photon_crc_memcpy_async(host.data(), static_cast<char*>(d_buf) + i * n, n, stream));
        TRY(photon_crc_stream_sync(stream));
        if (crc32c(host.data(), n) != out[i]) ++bad;
    }
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < 20; ++r)
        TRY(photon_crc32c_batch_strided(d_buf, n, n, count, 0, nullptr, static_cast<uint32_t*>(d_out), stream));
    TRY(photon_crc_stream_sync(stream));
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("gpu_batch_example: %d mismatches, %.1f GB/s, callback ran %d time(s)\n", bad, 20.0 * n * count / s / 1e9,
           g_done.load());
    TRY(photon_crc_device_free(d_buf));
    TRY(photon_crc_device_free(d_out));
    TRY(photon_crc_stream_destroy(stream));
    return bad ? 1 : 0;
}
