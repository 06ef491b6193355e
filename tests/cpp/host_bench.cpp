// host_bench.cpp -- the drop-in host engine timed the way bench.py times
// Photon's own crc32c() (oracle/ref/ref_harness.cpp `bench`): nbuf random
// buffers of len bytes, crc32c() through the crc32c_auto pointer of
// <photon/common/checksum/crc32c.h> (this library's, not Photon's), split
// across a persistent pool of pinned threads (spin_pool.h), best and median
// pass over at least min_seconds.
// Usage: host_bench <nbuf> <len> <threads> <min_seconds>; one JSON line.
#include <photon/common/checksum/crc32c.h>

#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <thread>
#include <vector>

#include "spin_pool.h"

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
    benchpool::SpinPool pool(threads);
    std::vector<uint8_t> buf(nbuf * len);
    std::vector<uint32_t> out(nbuf);
    benchpool::time_passes(pool, nbuf, 0.0, [&](size_t i) { splitmix_fill(buf.data() + i * len, len, 0x5EED0001ull + i); });
    const benchpool::PassStats st =
        benchpool::time_passes(pool, nbuf, min_s, [&](size_t i) { out[i] = crc32c(buf.data() + i * len, len); });
    uint32_t x = 0;
    for (uint32_t c : out) x ^= c;
    printf("{\"gib_per_s\": %.4f, \"gib_per_s_median\": %.4f, \"best_s\": %.6f, \"passes\": %d, \"threads\": %d, "
           "\"nbuf\": %zu, \"len\": %zu, \"xor\": %u}\n",
           (double)nbuf * len / st.best_s / (1u << 30), (double)nbuf * len / st.median_s / (1u << 30), st.best_s,
           st.passes, threads, nbuf, len, x);
    return 0;
}
