// multi_device_test.cpp -- the library's one-process, many-GPU plumbing
// (photonlibos_amd/csrc/multi_device.h: the shard plan of
// photon_crc32c_host_batch_strided_multi, the per-slice device switching of
// it and of photon_crc32c_batch_strided_shards / photon_crc32c_extend_spans,
// and the per-device table images) run on the CPU against a SIMULATED
// runtime of 8 devices (on a one-GPU box every shard lands on
// device 0, where a wrong device switch or a resource keyed to the wrong
// device cannot show). Exit status 0 = every check passed.
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <vector>

#include "../../photonlibos_amd/csrc/multi_device.h"

using namespace pcrc;

static int g_fail = 0;
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            if (g_fail++ < 20) fprintf(stderr, "%s:%d: CHECK(%s)\n", __FILE__, __LINE__, #c); \
        }                                                                 \
    } while (0)

// A runtime with kDev devices and a per-thread current device (HIP's rule).
constexpr int kDev = 8;
thread_local int t_cur = 0;
struct FakeRT {
    std::atomic<int> sets{0};
    int get(int* d) {
        *d = t_cur;
        return 0;
    }
    int set(int d) {
        ++sets;
        if (d < 0 || d >= kDev) return -19;  // -ENODEV
        t_cur = d;
        return 0;
    }
};

static void test_plan() {
    const uint64_t counts[] = {0, 1, 2, 3, 7, 8, 9, 100, 4095, 65536, 1048576, (1ull << 40) + 3};
    for (int nd = 1; nd <= kDev; ++nd) {
        std::vector<int> devs;
        for (int d = 0; d < nd; ++d) devs.push_back((d * 3 + 1) % kDev);  // any device ids, in this order
        for (uint64_t count : counts) {
            const std::vector<Slice> p = shard_plan(count, devs);
            CHECK(p.size() == std::min<uint64_t>(nd, count));
            uint64_t next = 0, lo = UINT64_MAX, hi = 0;
            for (size_t k = 0; k < p.size(); ++k) {
                CHECK(p[k].device == devs[k]);      // slice k on device k of the list
                CHECK(p[k].lo == next);             // contiguous and disjoint
                CHECK(p[k].hi > p[k].lo);           // no empty slice
                lo = std::min(lo, p[k].hi - p[k].lo);
                hi = std::max(hi, p[k].hi - p[k].lo);
                next = p[k].hi;
            }
            CHECK(next == count);                   // complete
            if (!p.empty()) CHECK(hi - lo <= 1);    // balanced
        }
    }
    const std::vector<int> all = {0, 1, 2, 3, 4, 5, 6, 7};
    CHECK(first_devices(all, 0).size() == 8 && first_devices(all, -1).size() == 8);
    CHECK(first_devices(all, 3) == std::vector<int>({0, 1, 2}));
    CHECK(first_devices(all, 9).size() == 8);
}

// The host_batch_strided_multi flow: every slice's body runs with ITS device
// current, reads that device's lazily built image, and writes its outputs.
static void test_threaded(uint64_t count, int nd) {
    FakeRT rt;
    PerDevice<int> img;  // "image" of device d = d + 100, built on first use
    std::atomic<int> builds{0};
    std::vector<int> devs;
    for (int d = 0; d < nd; ++d) devs.push_back(kDev - 1 - d);
    const std::vector<Slice> plan = shard_plan(count, devs);
    std::vector<int> out(count, -1);
    std::string err;
    const int rc = run_slices_threaded(
        rt, plan,
        [&](const Slice& sl) {
            int cur = -1;
            rt.get(&cur);
            CHECK(cur == sl.device);
            for (int rep = 0; rep < 3; ++rep) {
                int v = 0;
                CHECK(img.get(cur, &v, [&](int dev, int& slot) {
                    ++builds;
                    slot = dev + 100;
                    return 0;
                }) == 0);
                CHECK(v == sl.device + 100);  // keyed by the slice's device, not device 0
            }
            for (uint64_t i = sl.lo; i < sl.hi; ++i) {
                CHECK(out[i] == -1);  // written once
                out[i] = cur;
            }
            return 0;
        },
        [] { return std::string("no error"); }, &err);
    CHECK(rc == 0);
    CHECK(builds.load() == (int)plan.size());  // one build per device used
    for (const Slice& sl : plan)
        for (uint64_t i = sl.lo; i < sl.hi; ++i) CHECK(out[i] == sl.device);
    for (uint64_t i = 0; i < count; ++i) CHECK(out[i] != -1);
}

static void test_threaded_failure() {
    FakeRT rt;
    std::vector<int> devs = {0, 1, 2, 3, 4, 5, 6, 7};
    const std::vector<Slice> plan = shard_plan(1000, devs);
    std::string err;
    thread_local std::string t_err;
    const int rc = run_slices_threaded(
        rt, plan,
        [&](const Slice& sl) {
            if (sl.device == 5) {
                t_err = "injected on 5";
                return -5;
            }
            return 0;
        },
        [] { return t_err; }, &err);
    CHECK(rc == -5);
    CHECK(err == "device 5: injected on 5");
    // a device the runtime refuses
    std::vector<Slice> bad = {{2, 0, 10}, {9, 10, 20}};
    err.clear();
    CHECK(run_slices_threaded(rt, bad, [](const Slice&) { return 0; }, [] { return std::string(); }, &err) == -19);
    CHECK(err.rfind("device 9:", 0) == 0);
}

// batch_strided_shards / extend_spans: sequential, each body with its
// device current, the caller's device restored (also after a failure).
static void test_sequential() {
    FakeRT rt;
    t_cur = 3;
    const int devs[] = {0, 7, 2, 2, 5, 1};
    std::vector<int> seen;
    int ran = 0;
    int rc = run_on_devices(
        rt, 6, [&](int i) { return devs[i]; },
        [&](int i) {
            int cur = -1;
            rt.get(&cur);
            CHECK(cur == devs[i]);
            seen.push_back(cur);
            return 0;
        },
        &ran);
    CHECK(rc == 0 && ran == 6 && seen == std::vector<int>(devs, devs + 6));
    CHECK(t_cur == 3);
    // a failing body stops the loop; the device is restored
    seen.clear();
    rc = run_on_devices(
        rt, 6, [&](int i) { return devs[i]; },
        [&](int i) {
            seen.push_back(i);
            return i == 2 ? -22 : 0;
        },
        &ran);
    CHECK(rc == -22 && ran == 3 && seen.size() == 3 && t_cur == 3);
    // an invalid device id fails the switch, the body is not run
    seen.clear();
    const int bad[] = {1, 8};
    rc = run_on_devices(
        rt, 2, [&](int i) { return bad[i]; },
        [&](int i) {
            seen.push_back(i);
            return 0;
        },
        &ran);
    CHECK(rc == -19 && seen.size() == 1 && t_cur == 3);
}

// extend_spans' collection pass (run_on_every_device): a device that refuses
// the switch in the middle skips only its own body; every later index still
// runs on its device, the first error is returned, the caller's device is
// restored.
struct FlakyRT : FakeRT {
    int refuse = -1;  // a device id whose next switch fails once
    int set(int d) {
        if (d == refuse) {
            refuse = -1;
            return -5;  // -EIO
        }
        return FakeRT::set(d);
    }
};

static void test_every_device() {
    FlakyRT rt;
    t_cur = 4;
    const int devs[] = {0, 7, 2, 6, 5, 1};
    std::vector<int> freed;
    rt.refuse = 2;  // index 2's switch fails
    int rc = run_on_every_device(
        rt, 6, [&](int i) { return devs[i]; },
        [&](int i) {
            int cur = -1;
            rt.get(&cur);
            CHECK(cur == devs[i]);  // each lease returned on its own device
            freed.push_back(i);
            return 0;
        });
    CHECK(rc == -5 && freed == std::vector<int>({0, 1, 3, 4, 5}) && t_cur == 4);
    // a failing body does not stop the pass either; the first code wins
    freed.clear();
    rc = run_on_every_device(
        rt, 6, [&](int i) { return devs[i]; },
        [&](int i) {
            freed.push_back(i);
            return i == 1 ? -22 : i == 4 ? -12 : 0;
        });
    CHECK(rc == -22 && freed.size() == 6 && t_cur == 4);
    // all good: 0
    CHECK(run_on_every_device(rt, 6, [&](int i) { return devs[i]; }, [](int) { return 0; }) == 0);
}

int main() {
    test_plan();
    for (int nd = 1; nd <= kDev; ++nd)
        for (uint64_t count : {1ull, 5ull, 8ull, 1000ull, 65537ull}) test_threaded(count, nd);
    test_threaded_failure();
    test_sequential();
    test_every_device();
    if (g_fail) {
        fprintf(stderr, "multi_device_test: %d check(s) failed\n", g_fail);
        return 1;
    }
    printf("multi_device_test: ok\n");
    return 0;
}
