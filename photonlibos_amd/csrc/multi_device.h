// multi_device.h -- the one-process, many-GPU plumbing of the C-ABI
// (photon_crc32c_host_batch_strided_multi, photon_crc32c_batch_strided_shards,
// photon_crc32c_extend_spans / photon_crc64ecma_extend_spans), host-only and
// free of HIP so that tests/cpp/multi_device_test.cpp can run it on the CPU
// against a simulated 8-device runtime (these paths had only ever
// run with every shard on device 0 of a one-GPU box, where a wrong
// hipSetDevice or a per-device resource keyed to the wrong device cannot
// show).
//
// Photon runs one process per host: a batch of independent
// buffers is cut into contiguous slices of buffer indices, one per device, no
// collective; one logical buffer spread over devices is folded on the host
// with crc32c_combine's identity (crc.cpp:393-405).
//
// RT is the device runtime: int get(int* dev), int set(int dev) (0 or a
// nonzero error), the HIP one in crc32c_device.hip, a fake in the test.
#pragma once
#include <stdint.h>

#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace pcrc {

struct Slice {
    int device;
    uint64_t lo, hi;  // buffer indices [lo, hi)
};

// Contiguous, disjoint slices covering [0, count) exactly, in device order:
// slice k = [count*k/nd, count*(k+1)/nd) on devs[k], nd = min(#devs, count)
// (a device gets no slice when there are fewer buffers than devices; slice
// sizes differ by at most one buffer).
inline std::vector<Slice> shard_plan(uint64_t count, const std::vector<int>& devs) {
    std::vector<Slice> plan;
    const uint64_t nd = devs.size() < count ? devs.size() : count;
    for (uint64_t k = 0; k < nd; ++k) {
        // (count * k) may exceed 64 bits only for counts beyond 2^61 buffers
        const unsigned __int128 c = count;
        plan.push_back({devs[k], (uint64_t)(c * k / nd), (uint64_t)(c * (k + 1) / nd)});
    }
    return plan;
}

// The first `ndev` usable devices (all when ndev <= 0 or ndev > #usable).
inline std::vector<int> first_devices(const std::vector<int>& usable, int ndev) {
    std::vector<int> d = usable;
    if (ndev > 0 && ndev < (int)d.size()) d.resize(ndev);
    return d;
}

// One lazily built resource per device id (the small kernels' table images):
// the slot of the CALLING thread's current device, which is why every
// multi-device path sets the device before it calls into the engine.
template <typename T>
struct PerDevice {
    std::mutex mu;
    std::vector<T> v;
    // f(dev, T&) builds slot `dev` when it is still value-initialised; returns f's code.
    template <typename F>
    int get(int dev, T* out, F build) {
        std::lock_guard<std::mutex> lk(mu);
        if ((int)v.size() <= dev) v.resize(dev + 1, T{});
        if (v[dev] == T{}) {
            if (int rc = build(dev, v[dev])) return rc;
        }
        *out = v[dev];
        return 0;
    }
    // Slot `dev` as it is (value-initialised when never built).
    T peek(int dev) {
        std::lock_guard<std::mutex> lk(mu);
        return dev >= 0 && dev < (int)v.size() ? v[dev] : T{};
    }
};

// Run body(slice) for every slice of `plan` on a thread of its own whose
// current device is the slice's device (each device driving its own pipeline
// concurrently). Returns 0 or the first failing slice's code, with
// "device D: <its error text>" in *err (errtext() is the failing thread's
// error, read on that thread).
template <typename RT, typename Body, typename ErrText>
int run_slices_threaded(RT& rt, const std::vector<Slice>& plan, Body body, ErrText errtext, std::string* err) {
    std::vector<int> rcs(plan.size(), 0);
    std::vector<std::string> errs(plan.size());
    std::vector<std::thread> th;
    th.reserve(plan.size());
    for (size_t k = 0; k < plan.size(); ++k) {
        th.emplace_back([&, k] {
            const int se = rt.set(plan[k].device);
            rcs[k] = se ? se : body(plan[k]);
            if (rcs[k]) errs[k] = se ? std::string("set device failed") : errtext();
        });
    }
    for (auto& t : th) t.join();
    for (size_t k = 0; k < plan.size(); ++k)
        if (rcs[k]) {
            *err = "device " + std::to_string(plan[k].device) + ": " + errs[k];
            return rcs[k];
        }
    return 0;
}

// Run body(i) for i < n on the calling thread, with device(i) current for
// each call, stopping at the first failure; the caller's current device is
// restored whatever happens. Returns 0 or the first nonzero code (set errors
// included) and the number of bodies run in *ran.
template <typename RT, typename Dev, typename Body>
int run_on_devices(RT& rt, int n, Dev device, Body body, int* ran) {
    int prev = -1;
    if (int rc = rt.get(&prev)) return rc;
    int rc = 0, k = 0;
    for (; k < n && !rc; ++k) {
        rc = rt.set(device(k));
        if (!rc) rc = body(k);
    }
    if (ran) *ran = k;
    (void)rt.set(prev);
    return rc;
}

// The same, but it never stops: body(i) runs for every i whose device could
// be made current (a failed switch skips only that body), so a cleanup pass
// still reaches every later index (extend_spans returns every scratch lease
// on its own device even when one device refuses the switch).
// Returns 0 or the first nonzero code, switch errors included.
template <typename RT, typename Dev, typename Body>
int run_on_every_device(RT& rt, int n, Dev device, Body body) {
    int prev = -1;
    if (int rc = rt.get(&prev)) return rc;
    int first = 0;
    for (int k = 0; k < n; ++k) {
        int rc = rt.set(device(k));
        if (!rc) rc = body(k);
        if (rc && !first) first = rc;
    }
    (void)rt.set(prev);
    return first;
}

}  // namespace pcrc
