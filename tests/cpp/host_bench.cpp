// host_bench.cpp -- the drop-in host engine timed the way bench.py times
// Photon's own crc32c() (oracle/ref/ref_harness.cpp `bench`): nbuf random
// buffers of len bytes, crc32c() through the crc32c_auto pointer of
// <photon/common/checksum/crc32c.h> (this library's, not Photon's), split
// across threads, best pass of several over at least min_seconds.
// Usage: host_bench <nbuf> <len> <threads> <min_seconds>; one JSON line.
#include <photon/common/checksum/crc32c.h>

#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <thread>
#include <vector>

static void splitmix_fill(uint8_t* p, size_t n, uint64_t seed) {
    uint64_t s = seed;
    for (size_t i = 0; i < n; i += 8) {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        for (size_t k = 0; k < 8 && i + k < n; ++k) p[i + k] = (uint8_t)(z >> (8 * k));
    }
}

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s <nbuf> <len> <threads> <min_seconds>\n", argv[0]);
        return 2;
    }
    const size_t nbuf = strtoull(argv[1], nullptr, 0), len = strtoull(argv[2], nullptr, 0);
    const int threads = atoi(argv[3]);
    const double min_s = atof(argv[4]);
    std::vector<uint8_t> buf(nbuf * len);
    for (size_t i = 0; i < nbuf; ++i) splitmix_fill(buf.data() + i * len, len, 0x5EED0001ull + i);
    std::vector<uint32_t> out(nbuf);
    auto pass = [&]() {
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                for (size_t i = nbuf * t / threads; i < nbuf * (t + 1) / threads; ++i)
                    out[i] = crc32c(buf.data() + i * len, len);
            });
        for (auto& x : th) x.join();
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    double best = 1e30, total = 0;
    int passes = 0;
    while (total < min_s || passes < 3) {
        const double s = pass();
        best = s < best ? s : best;
        total += s;
        ++passes;
    }
    uint32_t x = 0;
    for (uint32_t c : out) x ^= c;
    printf("{\"gib_per_s\": %.4f, \"best_s\": %.6f, \"passes\": %d, \"threads\": %d, \"nbuf\": %zu, \"len\": %zu, "
           "\"xor\": %u}\n",
           (double)nbuf * len / best / (1u << 30), best, passes, threads, nbuf, len, x);
    return 0;
}
