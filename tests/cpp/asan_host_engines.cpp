// asan_host_engines.cpp -- the host drop-in engines (crc32c_cpu.cpp,
// crc64_cpu.cpp) built from source with AddressSanitizer + UBSan
// (tests/test_cpp_consumers.py): hw == sw for every length 0..1499 at every
// start offset 0..15, each buffer its own exactly-sized heap block so any
// over-read of the SSE4.2 / PCLMUL paths is caught.
#include <photon/common/checksum/crc64ecma.h>
#include <photon/common/checksum/crc32c.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
int main() {
    int bad = 0;
    for (size_t n = 0; n < 1500; ++n)
        for (size_t off = 0; off < 16; ++off) {
            unsigned char* b = (unsigned char*)malloc(n + off ? n + off : 1);
            for (size_t i = 0; i < n + off; ++i) b[i] = (unsigned char)(i * 131 + n);
            uint64_t s = n * 0x9E3779B97F4A7C15ull;
            if (crc64ecma_hw(b + off, n, s) != crc64ecma_sw(b + off, n, s)) ++bad;
            if (crc32c_hw(b + off, n, (uint32_t)s) != crc32c_sw(b + off, n, (uint32_t)s)) ++bad;
            free(b);
        }
    printf("asan64: %d mismatches\n", bad);
    return bad != 0;
}
