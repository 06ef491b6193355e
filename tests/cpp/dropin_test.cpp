// dropin_test.cpp -- compiled against the drop-in headers exactly as Photon
// code would be (#include <photon/common/checksum/crc32c.h>, crc64ecma.h) and
// linked with libphoton_checksum.so instead of Photon's crc.cpp/crc_tables.cpp.
// Re-runs the checks of the reference's common/checksum/test/test_checksum.cpp
// (golden file, sw/hw differential 0..3999, combine/series/trim properties)
// without gtest. Usage: dropin_test <checksum.in> <checksum.crc64>
#include <photon/common/checksum/crc32c.h>
#include <photon/common/checksum/crc64ecma.h>

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <fstream>
#include <string>
#include <vector>

static int failures = 0;
#define CHECK(c)                                                   \
    do {                                                           \
        if (!(c)) {                                                \
            ++failures;                                            \
            if (failures < 20) fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
        }                                                          \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    // Golden file (test_checksum.cpp:28-63): "<crc32c> <string>" + crc64 lines.
    std::ifstream in(argv[1]), in2(argv[2]);
    size_t cases = 0;
    while (true) {
        uint32_t c32;
        uint64_t c64;
        std::string s;
        in >> c32 >> s;
        in2 >> c64;
        if (s.empty()) break;
        ++cases;
        CHECK(crc32c(s) == c32);
        CHECK(crc32c_sw((const uint8_t*)s.data(), s.size(), 0) == c32);
        CHECK(crc32c_hw((const uint8_t*)s.data(), s.size(), 0) == c32);
        CHECK(crc32c_hw_portable((const uint8_t*)s.data(), s.size(), 0) == c32);
        CHECK(crc32c_hw_simple((const uint8_t*)s.data(), s.size(), 0) == c32);
        CHECK(crc64ecma(s.data(), s.size(), 0) == c64);
        CHECK(crc64ecma_sw((const uint8_t*)s.data(), s.size(), 0) == c64);
    }
    CHECK(cases == 512);
    // sw vs hw, lengths 0..3999 (test_checksum.cpp:70-84, 121-123).
    std::vector<uint8_t> buf(64 * 1024 + 16);
    for (size_t i = 0; i < 4000; ++i) {
        CHECK(crc32c_sw(buf.data(), i, 0) == crc32c_hw(buf.data(), i, 0));
        CHECK(crc64ecma_sw(buf.data(), i, 0) == crc64ecma_hw(buf.data(), i, 0));
        buf[i] = 'a' + i % 26;
    }
    CHECK(is_crc32c_hw_available());
    // combine / series / combine_series / trim (test_checksum.cpp:231-266).
    const uint32_t N = 10, M = 510;
    unsigned char b[M * N];
    srand(7);
    for (auto& c : b) c = rand();
    auto x = crc32c_sw(b, M * N, 0);
    CHECK(x == crc32c_hw(b, M * N, 0));
    for (int i = 0; i < 10000; ++i) {
        uint32_t L1 = rand() % (sizeof(b) / 2), L2 = sizeof(b) - L1;
        auto c1 = crc32c_hw(b, L1, 0), c2 = crc32c_hw(b + L1, L2, 0);
        CHECK(x == crc32c_combine_hw(c1, c2, L2));
        CHECK(x == crc32c_combine_sw(c1, c2, L2));
        CHECK(x == crc32c_combine(c1, c2, L2));
        CHECK(x == crc32c_extend(b + L1, L2, c1));
    }
    uint32_t crc[N] = {0};
    crc32c_series_sw(b, M, N, crc);
    CHECK(x == crc32c_combine_series_sw(crc, M, N));
    CHECK(x == crc32c_combine_series_hw(crc, M, N));
    memset(crc, 0, sizeof(crc));
    crc32c_series(b, M, N, crc);
    CHECK(x == crc32c_combine_series(crc, M, N));
    for (int i = 0; i < 10000; ++i) {
        uint32_t L1 = 100 + rand() % 64, L3 = 100 + rand() % 64;
        auto c1 = crc32c_hw(b, L1, 0), c2 = crc32c_hw(b + L1, sizeof(b) - L1 - L3, 0);
        auto c3 = crc32c_hw(b + sizeof(b) - L3, L3, 0);
        CHECK(c2 == crc32c_trim_sw({x, sizeof(b)}, {c1, L1}, {c3, L3}));
        CHECK(c2 == crc32c_trim_hw({x, sizeof(b)}, {c1, L1}, {c3, L3}));
        CHECK(c2 == crc32c_trim({x, sizeof(b)}, {c1, L1}, {c3, L3}));
    }
    errno = 0;
    CHECK(crc32c_trim({x, 10}, {1, 6}, {2, 6}) == 0 && errno == EINVAL);
    // CRC64 combine / extend / trim (test_checksum.cpp:268-308).
    auto y = crc64ecma_sw(b, M * N, 0);
    for (int i = 0; i < 2000; ++i) {
        uint32_t L2 = rand() % (sizeof(b) / 2), L1 = sizeof(b) - L2;
        auto c1 = crc64ecma_sw(b, L1, 0), c2 = crc64ecma_sw(b + L1, L2, 0);
        CHECK(y == crc64ecma_combine_sw(c1, c2, L2));
        CHECK(y == crc64ecma_combine_hw(c1, c2, L2));
        CHECK(y == crc64ecma_sw(b + L1, L2, c1));
    }
    for (int i = 0; i < 2000; ++i) {
        uint32_t L1 = 100 + rand() % 64, L3 = 100 + rand() % 64;
        auto c1 = crc64ecma_hw(b, L1, 0), c2 = crc64ecma_hw(b + L1, sizeof(b) - L1 - L3, 0);
        auto c3 = crc64ecma_hw(b + sizeof(b) - L3, L3, 0);
        CHECK(crc64ecma_trim_hw({y, sizeof(b)}, {c1, L1}, {c3, L3}) == c2);
        CHECK(crc64ecma_trim_sw({y, sizeof(b)}, {c1, L1}, {c3, L3}) == c2);
    }
    printf("dropin_test: %zu golden cases, %d failures\n", cases, failures);
    return failures ? 1 : 0;
}
