// concurrency_test.cpp -- the C-ABI is reentrant (the
// reference contract crc.cpp:126-137: dispatch pointers written once, the
// functions pure, called from any number of photon vCPU threads).
//
// 16 host threads, each on its own stream, submit mixed batches (strided
// CRC-32C of assorted lengths, ragged iovec batches with seeds, messages with
// and without segment CRCs, CRC-64 strided, combine batches) while a 17th
// thread keeps flipping every tuning knob of <photon_crc/tuning.h> (lane-group
// size, generic rows / fused kernel, streaming kernel shapes, message mode,
// CRC-64 streaming shape). Every result is checked against the ORACLE
// (oracle/lib/libcrc_oracle.so, the plain-C restatement pinned to the
// reference). Built with plain g++ (no HIP headers). Exit 0 = all bit-exact.
#include <photon_crc/checked_batch.h>
#include <photon_crc/crc32c_gpu.h>
#include <photon_crc/tuning.h>

#include <stdio.h>
#include <string.h>

#include <unistd.h>

#include <atomic>
#include <chrono>
#include <random>
#include <thread>
#include <vector>

extern "C" {
uint32_t or_crc32c_sw(const uint8_t* p, size_t n, uint32_t crc);
uint32_t or_crc32c_combine(uint32_t crc1, uint32_t crc2, uint32_t len2);
uint64_t or_crc64ecma_sw(const uint8_t* p, size_t n, uint64_t crc);
}

namespace {

constexpr int kThreads = 16;
constexpr int kIters = 40;
constexpr uint64_t kBuf = 8u << 20;
constexpr int kMaxItems = 64;

std::atomic<bool> g_stop{false};
// Watchdog state: what each submitter is doing (iteration, kind, phase).
struct Where {
    std::atomic<int> it{-1}, kind{-1}, phase{0};
};
Where g_where[kThreads];
const char* const kPhase[] = {"setup", "enqueue", "sync", "check", "teardown", "done"};
std::atomic<long> g_checked{0}, g_bad{0}, g_err{0};

#define RET
#define TRY(x)                                                                              \
    do {                                                                                    \
        int rc_ = (x);                                                                      \
        if (rc_) {                                                                          \
            fprintf(stderr, "thread %d: %s: %d %s\n", t, #x, rc_, photon_crc_last_error()); \
            g_err.fetch_add(1);                                                             \
            return RET;                                                                     \
        }                                                                                   \
    } while (0)

// Knob state as set by the flipper (for the mismatch report only).
std::atomic<int> g_k_lanes{0}, g_k_rows{-1}, g_k_msg{0}, g_k_long{0}, g_k_grid{0};

void check_at(bool ok, const char* what, uint64_t a, uint64_t b, uint64_t c) {
    g_checked.fetch_add(1);
    if (!ok && g_bad.fetch_add(1) < 30)
        fprintf(stderr, "MISMATCH %s (%llu, %llu, %llu) knobs now: lanes %d rows %d msg %d long %#x grid %d\n",
                what, (unsigned long long)a, (unsigned long long)b, (unsigned long long)c, g_k_lanes.load(),
                g_k_rows.load(), g_k_msg.load(), g_k_long.load(), g_k_grid.load());
}
#define check(ok) check_at((ok), kind_name, p0, p1, p2)

// Per-thread stream and device memory, set up and torn down by the main
// thread (allocation is not what this test is about: hipMalloc / hipFree are
// device-wide operations; the contract under test is concurrent SUBMISSION).
struct Res {
    void *stream = nullptr, *d_buf = nullptr, *d_iov = nullptr, *d_seeds = nullptr, *d_out = nullptr,
         *d_start = nullptr, *d_seg = nullptr, *d_a = nullptr, *d_b = nullptr, *d_len = nullptr;
};
Res g_res[kThreads];

// A pinned host array from the library's IOAlloc pool (checked_batch.h).
template <typename T>
struct Pinned {
    T* p = nullptr;
    explicit Pinned(size_t n) {
        void* q = nullptr;
        const int bytes = (int)(n * sizeof(T));
        if (photon_crc_pinned_allocate(nullptr, photon_crc_range{bytes, bytes}, &q) >= 0) p = static_cast<T*>(q);
    }
    ~Pinned() {
        if (p) photon_crc_pinned_deallocate(nullptr, p);
    }
    T& operator[](size_t i) { return p[i]; }
};

#undef RET
#define RET -1
int setup(int t) {
    Res& r = g_res[t];
    TRY(photon_crc_stream_create(&r.stream));
    TRY(photon_crc_device_alloc(&r.d_buf, kBuf));
    TRY(photon_crc_device_alloc(&r.d_iov, kMaxItems * 16));
    TRY(photon_crc_device_alloc(&r.d_seeds, kMaxItems * 8));
    TRY(photon_crc_device_alloc(&r.d_out, kMaxItems * 8));
    TRY(photon_crc_device_alloc(&r.d_start, (kMaxItems + 1) * 8));
    TRY(photon_crc_device_alloc(&r.d_seg, kMaxItems * 8));
    TRY(photon_crc_device_alloc(&r.d_a, kMaxItems * 4));
    TRY(photon_crc_device_alloc(&r.d_b, kMaxItems * 4));
    TRY(photon_crc_device_alloc(&r.d_len, kMaxItems * 4));
    return 0;
}

int teardown(int t) {
    Res& r = g_res[t];
    for (void* p : {r.d_buf, r.d_iov, r.d_seeds, r.d_out, r.d_start, r.d_seg, r.d_a, r.d_b, r.d_len})
        TRY(photon_crc_device_free(p));
    TRY(photon_crc_stream_destroy(r.stream));
    return 0;
}

#undef RET
#define RET
void submitter(int t) {
    std::mt19937_64 rng(0xC0FFEEull * (t + 1));
    Res& r = g_res[t];
    void *stream = r.stream, *d_buf = r.d_buf, *d_iov = r.d_iov, *d_seeds = r.d_seeds, *d_out = r.d_out,
         *d_start = r.d_start, *d_seg = r.d_seg, *d_a = r.d_a, *d_b = r.d_b, *d_len = r.d_len;
    Where& w = g_where[t];
    // Host sides of every copy are pinned (IOAlloc pool of the library), as an
    // asynchronous Photon caller's buffers would be.
    Pinned<uint8_t> host(kBuf);
    Pinned<photon_crc_iovec> iov(kMaxItems);
    Pinned<uint32_t> seeds(kMaxItems), out(kMaxItems), segs(kMaxItems), a(kMaxItems), b(kMaxItems), len(kMaxItems);
    Pinned<uint64_t> out64(kMaxItems), start(kMaxItems + 1);
    if (!host.p || !iov.p || !seeds.p || !out.p || !segs.p || !a.p || !b.p || !len.p || !out64.p || !start.p) {
        fprintf(stderr, "thread %d: pinned allocation failed: %s\n", t, photon_crc_last_error());
        g_err.fetch_add(1);
        return;
    }
    TRY(photon_crc_util_fill_splitmix(d_buf, kBuf, kBuf, 1, 0x7000 + t, stream));
    TRY(photon_crc_memcpy_async(host.p, d_buf, kBuf, stream));
    TRY(photon_crc_stream_sync(stream));
    const uint8_t* dbase = static_cast<const uint8_t*>(d_buf);
    const uint64_t lens[] = {0, 1, 15, 100, 4096, 4097, 8192, 65536, 200000};
    for (int it = 0; it < kIters; ++it) {
        const int kind = (int)(rng() % 5);
        w.it = it;
        w.kind = kind;
        w.phase = 1;
        static const char* const kNames[] = {"strided32", "iov32", "msg32", "strided64", "combine"};
        const char* kind_name = kNames[kind];
        uint64_t p0 = 0, p1 = 0, p2 = 0;
        if (kind == 0) {  // strided CRC-32C
            const uint64_t n = lens[rng() % 9], stride = n + (rng() % 3) * 16 + (rng() % 2);
            const uint64_t count = std::min<uint64_t>(kMaxItems, stride ? (kBuf - n) / stride : kMaxItems);
            const uint32_t seed = (uint32_t)rng();
            p0 = n, p1 = stride, p2 = count;
            TRY(photon_crc32c_batch_strided(dbase, stride, n, count, seed, nullptr, static_cast<uint32_t*>(d_out),
                                            stream));
            TRY(photon_crc_memcpy_async(out.p, d_out, count * 4, stream));
            w.phase = 2;
            TRY(photon_crc_stream_sync(stream));
            w.phase = 3;
            for (uint64_t i = 0; i < count; ++i) check(out[i] == or_crc32c_sw(host.p + i * stride, n, seed));
        } else if (kind == 1) {  // ragged iovec batch with per-buffer seeds
            const int count = 1 + (int)(rng() % kMaxItems);
            for (int i = 0; i < count; ++i) {
                const uint64_t n = rng() % 70000, off = rng() % (kBuf - n);
                iov[i] = {dbase + off, n};
                seeds[i] = (uint32_t)rng();
            }
            TRY(photon_crc_memcpy_async(d_iov, iov.p, count * 16, stream));
            TRY(photon_crc_memcpy_async(d_seeds, seeds.p, count * 4, stream));
            TRY(photon_crc32c_batch_iov(static_cast<const photon_crc_iovec*>(d_iov), count, 0,
                                        static_cast<const uint32_t*>(d_seeds), static_cast<uint32_t*>(d_out), stream));
            TRY(photon_crc_memcpy_async(out.p, d_out, count * 4, stream));
            w.phase = 2;
            TRY(photon_crc_stream_sync(stream));
            w.phase = 3;
            for (int i = 0; i < count; ++i) {
                const uint8_t* h = host.p + (static_cast<const uint8_t*>(iov[i].base) - dbase);
                p0 = iov[i].len, p1 = (uintptr_t)iov[i].base & 15, p2 = count;
                check(out[i] == or_crc32c_sw(h, iov[i].len, seeds[i]));
            }
        } else if (kind == 2) {  // messages of segments, chained; optionally with segment CRCs
            const int nmsg = 1 + (int)(rng() % 8);
            uint64_t nseg = 0;
            start[0] = 0;
            for (int m = 0; m < nmsg; ++m) {
                const int k = (int)(rng() % 8);
                for (int j = 0; j < k; ++j) {
                    const uint64_t n = rng() % 20000, off = rng() % (kBuf - n);
                    iov[nseg++] = {dbase + off, n};
                }
                start[m + 1] = nseg;
            }
            const bool seg = rng() & 1;
            const uint32_t seed = (uint32_t)rng();
            if (nseg) TRY(photon_crc_memcpy_async(d_iov, iov.p, nseg * 16, stream));
            TRY(photon_crc_memcpy_async(d_start, start.p, (nmsg + 1) * 8, stream));
            TRY(photon_crc32c_batch_msg_n(static_cast<const photon_crc_iovec*>(d_iov),
                                          static_cast<const uint64_t*>(d_start), nmsg, nseg, seed, nullptr,
                                          seg ? static_cast<uint32_t*>(d_seg) : nullptr,
                                          static_cast<uint32_t*>(d_out), stream));
            TRY(photon_crc_memcpy_async(out.p, d_out, nmsg * 4, stream));
            if (seg && nseg) TRY(photon_crc_memcpy_async(segs.p, d_seg, nseg * 4, stream));
            w.phase = 2;
            TRY(photon_crc_stream_sync(stream));
            w.phase = 3;
            p0 = nmsg, p1 = nseg, p2 = seg;
            for (int m = 0; m < nmsg; ++m) {
                uint32_t acc = seed;
                for (uint64_t j = start[m]; j < start[m + 1]; ++j) {
                    const uint8_t* h = host.p + (static_cast<const uint8_t*>(iov[j].base) - dbase);
                    if (seg) check(segs[j] == or_crc32c_sw(h, iov[j].len, 0));
                    acc = or_crc32c_sw(h, iov[j].len, acc);
                }
                check(out[m] == acc);
            }
        } else if (kind == 3) {  // CRC-64/ECMA strided
            const uint64_t n = lens[1 + rng() % 8], count = std::min<uint64_t>(kMaxItems, (kBuf - n) / n);
            const uint64_t seed = rng();
            p0 = n, p1 = count;
            TRY(photon_crc64ecma_batch_strided(dbase, n, n, count, seed, nullptr, static_cast<uint64_t*>(d_out),
                                               stream));
            TRY(photon_crc_memcpy_async(out64.p, d_out, count * 8, stream));
            w.phase = 2;
            TRY(photon_crc_stream_sync(stream));
            w.phase = 3;
            for (uint64_t i = 0; i < count; ++i) check(out64[i] == or_crc64ecma_sw(host.p + i * n, n, seed));
        } else {  // combine batch (with the reference's shortcuts: crc1 == 0, len2 == 0)
            const int count = kMaxItems;
            for (int i = 0; i < count; ++i) {
                a[i] = i % 7 == 0 ? 0 : (uint32_t)rng();
                b[i] = (uint32_t)rng();
                len[i] = i % 5 == 0 ? 0 : (uint32_t)rng();
            }
            TRY(photon_crc_memcpy_async(d_a, a.p, count * 4, stream));
            TRY(photon_crc_memcpy_async(d_b, b.p, count * 4, stream));
            TRY(photon_crc_memcpy_async(d_len, len.p, count * 4, stream));
            TRY(photon_crc32c_combine_batch(static_cast<const uint32_t*>(d_a), static_cast<const uint32_t*>(d_b),
                                            static_cast<const uint32_t*>(d_len), count, static_cast<uint32_t*>(d_out),
                                            stream));
            TRY(photon_crc_memcpy_async(out.p, d_out, count * 4, stream));
            w.phase = 2;
            TRY(photon_crc_stream_sync(stream));
            w.phase = 3;
            for (int i = 0; i < count; ++i) check(out[i] == or_crc32c_combine(a[i], b[i], len[i]));
        }
    }
    w.phase = 5;
}

// Flips every knob while the submitters run; each launch must see one
// consistent engine shape (any of them is bit-exact).
void knob_flipper() {
    std::mt19937 rng(7);
    const int lanes[] = {0, 4, 8, 16, 32, 64};
    const int rows[] = {-1, 2, 4, 8};
    const int long_lanes[] = {0, 32, 64};
    long flips = 0;
    while (!g_stop.load()) {
        switch (rng() % 5) {
            case 0: { int v = lanes[rng() % 6]; photon_crc_set_lanes_per_buffer(v); g_k_lanes = v; break; }
            case 1: { int v = rows[rng() % 4]; photon_crc_set_generic_rows(v); g_k_rows = v; break; }
            case 2: {
                int v = (int)(rng() % 3);
                photon_crc_set_msg_mode(v);
                photon_crc_set_msg_rows(rng() & 1 ? 2 : 4);
                g_k_msg = v;
                break;
            }
            case 3: {
                int l = long_lanes[rng() % 3], r = l ? (int)(rng() % 4) : 0;
                photon_crc_set_long_shape(l, r);
                g_k_long = l << 8 | r;
                break;
            }
            default: { int v = rng() & 1 ? 0 : 64 + (int)(rng() % 192); photon_crc_set_batch_grid(v); g_k_grid = v; break; }
        }
        ++flips;
        std::this_thread::yield();
    }
    // back to the defaults
    photon_crc_set_lanes_per_buffer(0);
    photon_crc_set_generic_rows(-1);
    photon_crc_set_msg_mode(0);
    photon_crc_set_msg_rows(2);
    photon_crc_set_long_shape(0, 0);
    photon_crc_set_batch_grid(0);
    printf("knob flips: %ld\n", flips);
}

}  // namespace

int main() {
    if (photon_crc_device_count() <= 0) {
        fprintf(stderr, "no device: %s\n", photon_crc_last_error());
        return 2;
    }
    // Watchdog: a hang (a submitter stuck in a HIP call) prints where every
    // thread is and ends the process with status 3 instead of blocking.
    std::thread([] {
        for (int s = 0; s < 60; ++s) {
            std::this_thread::sleep_for(std::chrono::seconds(1));
            if (g_stop.load()) return;
        }
        for (int t = 0; t < kThreads; ++t)
            fprintf(stderr, "WATCHDOG thread %d: iteration %d kind %d phase %s\n", t, g_where[t].it.load(),
                    g_where[t].kind.load(), kPhase[g_where[t].phase.load()]);
        fprintf(stderr, "WATCHDOG knobs: lanes %d rows %d msg %d long %#x grid %d; checked %ld\n",
                g_k_lanes.load(), g_k_rows.load(), g_k_msg.load(), g_k_long.load(), g_k_grid.load(),
                g_checked.load());
        fflush(stderr);
        _exit(3);
    }).detach();
    for (int t = 0; t < kThreads; ++t)
        if (setup(t)) return 1;
    std::thread flipper(knob_flipper);
    std::vector<std::thread> th;
    for (int t = 0; t < kThreads; ++t) th.emplace_back(submitter, t);
    for (auto& x : th) x.join();
    g_stop.store(true);
    flipper.join();
    for (int t = 0; t < kThreads; ++t)
        if (teardown(t)) return 1;
    printf("concurrency_test: %d threads, %ld results checked against the oracle, %ld mismatches, %ld errors\n",
           kThreads, g_checked.load(), g_bad.load(), g_err.load());
    return (g_bad.load() || g_err.load() || g_checked.load() == 0) ? 1 : 0;
}
