// spin_pool.h -- persistent, pinned, spin-waiting thread pool for the CPU
// baseline timings (test/bench infrastructure only; used by
// oracle/ref/ref_harness.cpp for Photon's own crc32c() and by
// tests/cpp/host_bench.cpp for this library's drop-in).
//
// Why not a thread per pass: a 4 MiB pass (config C1) takes ~130 us on one
// core, so spawning threads for every pass measures thread start-up, not
// checksum work. Here the workers are created once, pinned to the CPUs of
// the process's affinity mask, and spin on a generation counter; a pass is
// "publish generation -> every worker runs its slice -> last one arrives",
// which costs ~1 us of hand-off. The calling thread runs slice 0 itself.
#pragma once
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <thread>
#include <vector>

namespace benchpool {

inline void cpu_relax() {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
}

// CPUs of this process's affinity mask, in order.
inline std::vector<int> affinity_cpus() {
    std::vector<int> cpus;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof(set), &set) == 0)
        for (int c = 0; c < CPU_SETSIZE; ++c)
            if (CPU_ISSET(c, &set)) cpus.push_back(c);
    if (cpus.empty()) cpus.push_back(0);
    return cpus;
}

inline void pin_to(int cpu) {
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(cpu, &set);
    (void)sched_setaffinity(0, sizeof(set), &set);
}

class SpinPool {
public:
    // Worker t is pinned to CPU number t * |mask| / n of the affinity mask:
    // spread over the whole mask (on a many-CCD EPYC, packing 16 threads onto
    // CPUs 0-15 would put them on two CCDs and their two memory links).
    explicit SpinPool(int n) : n_(n < 1 ? 1 : n) {
        const std::vector<int> cpus = affinity_cpus();
        auto cpu_of = [&](int t) { return cpus[(size_t)t * cpus.size() / (size_t)n_ % cpus.size()]; };
        pin_to(cpu_of(0));
        for (int t = 1; t < n_; ++t) {
            const int cpu = cpu_of(t);
            workers_.emplace_back([this, t, cpu] {
                pin_to(cpu);
                uint64_t seen = 0;
                for (;;) {
                    uint64_t g;
                    while ((g = gen_.load(std::memory_order_acquire)) == seen) cpu_relax();
                    seen = g;
                    if (stop_.load(std::memory_order_relaxed)) return;
                    (*job_)(t);
                    done_.fetch_add(1, std::memory_order_acq_rel);
                }
            });
        }
    }
    ~SpinPool() {
        stop_.store(true, std::memory_order_relaxed);
        gen_.fetch_add(1, std::memory_order_acq_rel);
        for (auto& w : workers_) w.join();
    }
    int size() const { return n_; }
    // Run f(t) for t in [0, size()) on the pool; returns the wall seconds.
    double run(const std::function<void(int)>& f) {
        job_ = &f;
        done_.store(0, std::memory_order_relaxed);
        const auto t0 = std::chrono::steady_clock::now();
        gen_.fetch_add(1, std::memory_order_acq_rel);
        f(0);
        while (done_.load(std::memory_order_acquire) != n_ - 1) cpu_relax();
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }

private:
    int n_;
    std::vector<std::thread> workers_;
    const std::function<void(int)>* job_ = nullptr;
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> done_{0};
    std::atomic<bool> stop_{false};
};

// Time `per_item(i)` over items [0, nitems) split evenly across the pool:
// best and median pass over at least min_seconds (and at least 5 passes).
struct PassStats {
    double best_s = 0, median_s = 0;
    int passes = 0;
};

inline PassStats time_passes(SpinPool& pool, size_t nitems, double min_seconds,
                             const std::function<void(size_t)>& per_item) {
    const int n = pool.size();
    const std::function<void(int)> slice = [&](int t) {
        const size_t b = nitems * t / n, e = nitems * (t + 1) / n;
        for (size_t i = b; i < e; ++i) per_item(i);
    };
    std::vector<double> ts;
    double total = 0;
    while (total < min_seconds || ts.size() < 5) {
        const double s = pool.run(slice);
        ts.push_back(s);
        total += s;
    }
    std::vector<double> sorted = ts;
    std::sort(sorted.begin(), sorted.end());
    PassStats st;
    st.best_s = sorted.front();
    st.median_s = sorted[sorted.size() / 2];
    st.passes = (int)ts.size();
    return st;
}

}  // namespace benchpool
