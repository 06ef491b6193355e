// file_source.cpp -- the runtime shim (streams, device memory, copies,
// completion callbacks: Photon code needs no HIP headers) and producers of
// checksum input outside device memory
// (include/photon_crc/crc32c_gpu.h):
//   photon_crc_host_register / _unregister: make existing host buffers (e.g.
//       the iovec targets of IFile::preadv, fs/filesystem.h:54-70) readable by
//       the kernels in place (hipHostRegister, mapped);
//   photon_crc32c_file_strided: checksum equal-size records of a file. A
//       reader thread pread()s 4 KiB-aligned chunks (O_DIRECT-compatible) into
//       two pinned chunk buffers while the GPU pipeline
//       (photon_crc32c_host_batch_strided) checksums the previous chunk, so
//       the CPU never touches the payload bytes when the fd is O_DIRECT.
#include <errno.h>
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <string.h>
#include <unistd.h>

#include <condition_variable>
#include <deque>
#include <functional>
#include <vector>
#include <map>
#include <mutex>
#include <string>
#include <thread>

#include <photon_crc/crc32c_gpu.h>

#include "internal.h"

namespace {

using pcrc::report_error;
using pcrc::report_hip_error;

constexpr uint64_t kAlign = 4096;
constexpr uint64_t kChunk = 64ull << 20;  // payload span per chunk
constexpr int kReadPieces = 8;            // parallel preads per chunk (page-cache copies are per-core bound)
constexpr int kReaderThreads = 16;        // persistent reader pool, shared by concurrent callers
constexpr int kKeepPairs = 4;             // chunk-buffer pairs kept pinned between calls

// A pair of pinned chunk buffers, owned by ONE call at a time: concurrent
// callers check out their own pair (pinned allocation is slow, so pairs are
// kept for reuse), so they no longer serialise on one global pair.
struct ChunkPair {
    void* buf[2] = {nullptr, nullptr};
    uint64_t cap = 0;
};

struct PairCache {
    std::mutex mu;
    std::vector<ChunkPair> free;
};

PairCache& pair_cache() {
    static PairCache* c = new PairCache;
    return *c;
}

void free_pair(ChunkPair& p) {
    for (void*& b : p.buf)
        if (b) {
            (void)hipHostFree(b);
            b = nullptr;
        }
    p.cap = 0;
}

int checkout_pair(uint64_t cap, ChunkPair* out) {
    {
        PairCache& c = pair_cache();
        std::lock_guard<std::mutex> lk(c.mu);
        for (size_t i = 0; i < c.free.size(); ++i)
            if (c.free[i].cap >= cap) {
                *out = c.free[i];
                c.free.erase(c.free.begin() + i);
                return 0;
            }
    }
    ChunkPair p;
    for (void*& b : p.buf) {
        hipError_t e = hipHostMalloc(&b, cap, hipHostMallocPortable);
        if (e != hipSuccess) {
            free_pair(p);
            return report_hip_error(e, "hipHostMalloc(chunk)");
        }
    }
    p.cap = cap;
    *out = p;
    return 0;
}

void return_pair(ChunkPair p) {
    PairCache& c = pair_cache();
    std::lock_guard<std::mutex> lk(c.mu);
    c.free.push_back(p);
    if ((int)c.free.size() > kKeepPairs) {  // drop the smallest
        size_t k = 0;
        for (size_t i = 1; i < c.free.size(); ++i)
            if (c.free[i].cap < c.free[k].cap) k = i;
        free_pair(c.free[k]);
        c.free.erase(c.free.begin() + k);
    }
}

// Persistent reader threads (created on first use) running pread pieces for
// every caller: no thread start-up per chunk.
class ReaderPool {
public:
    static ReaderPool& get() {
        static ReaderPool* p = new ReaderPool;  // never destroyed: workers outlive static destruction
        return *p;
    }
    // Run every task on the pool and wait for all of them.
    void run_all(std::vector<std::function<void()>>& tasks) {
        std::mutex done_mu;
        std::condition_variable done_cv;
        size_t left = tasks.size();
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (auto& t : tasks)
                q_.push_back([&t, &done_mu, &done_cv, &left] {
                    t();
                    std::lock_guard<std::mutex> g(done_mu);
                    if (--left == 0) done_cv.notify_all();
                });
        }
        cv_.notify_all();
        std::unique_lock<std::mutex> g(done_mu);
        done_cv.wait(g, [&] { return left == 0; });
    }

private:
    ReaderPool() {
        for (int i = 0; i < kReaderThreads; ++i)
            std::thread([this] {
                for (;;) {
                    std::function<void()> job;
                    {
                        std::unique_lock<std::mutex> lk(mu_);
                        cv_.wait(lk, [&] { return !q_.empty(); });
                        job = std::move(q_.front());
                        q_.pop_front();
                    }
                    job();
                }
            }).detach();
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
};

// Read [off, off+want_max) of fd into dst, accepting a short read at end of
// file once at least want_min bytes are in (the 4 KiB-rounded tail of the
// last chunk may run past EOF). -errno, or -EIO before want_min.
int read_span(int fd, uint8_t* dst, uint64_t want_min, uint64_t want_max, uint64_t off, std::string* err) {
    uint64_t got = 0;
    while (got < want_max) {
        const ssize_t r = pread(fd, dst + got, want_max - got, (off_t)(off + got));
        if (r < 0) {
            if (errno == EINTR) continue;
            *err = std::string("pread: ") + strerror(errno);
            return -errno;
        }
        got += (uint64_t)r;
        if (r == 0 || (got >= want_min && got < want_max)) break;
    }
    if (got < want_min) {
        *err = "pread: end of file before the last record";
        return -EIO;
    }
    return 0;
}

// read_span over kReadPieces 4 KiB-aligned pieces in parallel on the reader
// pool; only the last piece may end short (at EOF).
int read_span_parallel(int fd, uint8_t* dst, uint64_t want_min, uint64_t want_max, uint64_t off, std::string* err) {
    const uint64_t piece = ((want_max / kReadPieces) + kAlign - 1) & ~(kAlign - 1);
    if (want_max < 4 * kAlign * kReadPieces || piece == 0) return read_span(fd, dst, want_min, want_max, off, err);
    int rcs[kReadPieces + 1] = {};
    std::string errs[kReadPieces + 1];
    std::vector<std::function<void()>> tasks;
    int used = 0;
    for (uint64_t lo = 0; lo < want_max; lo += piece, ++used) {
        const uint64_t hi = lo + piece < want_max ? lo + piece : want_max;
        const bool last = hi == want_max;
        const uint64_t need = last ? (want_min > lo ? want_min - lo : 0) : hi - lo;
        const int k = used;
        tasks.push_back([=, &rcs, &errs] { rcs[k] = read_span(fd, dst + lo, need, hi - lo, off + lo, &errs[k]); });
    }
    ReaderPool::get().run_all(tasks);
    for (int i = 0; i < used; ++i)
        if (rcs[i]) {
            *err = errs[i];
            return rcs[i];
        }
    return 0;
}

// Ranges registered through photon_crc_host_register, so the message batch
// can check that a segment [p, p+n) stays inside its registration (file-local:
// no exported symbol a host application could collide with).
std::mutex g_reg_mu;
std::map<uintptr_t, uint64_t> g_reg;

}  // namespace

void pcrc::record_registration(const void* p, uint64_t n) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg[reinterpret_cast<uintptr_t>(p)] = n;
}

void pcrc::forget_registration(const void* p) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg.erase(reinterpret_cast<uintptr_t>(p));
}

int pcrc::registered_range_check(const void* p, uint64_t n) {
    const uintptr_t q = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.upper_bound(q);
    if (it == g_reg.begin()) return -1;
    --it;
    if (q - it->first >= it->second) return -1;  // not inside a known registration
    return n <= it->second - (q - it->first) ? 1 : 0;
}

extern "C" {

int photon_crc_stream_create(void** stream) {
    if (!stream) return report_error(-EINVAL, "null stream pointer");
    if (photon_crc_device_count() <= 0) return -ENODEV;
    hipStream_t s = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e != hipSuccess) return report_hip_error(e, "hipStreamCreateWithFlags");
    *stream = s;
    return 0;
}

int photon_crc_stream_destroy(void* stream) {
    if (!stream) return 0;
    hipError_t e = hipStreamDestroy(static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : report_hip_error(e, "hipStreamDestroy");
}

int photon_crc_stream_sync(void* stream) {
    if (photon_crc_device_count() <= 0) return -ENODEV;
    hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : report_hip_error(e, "hipStreamSynchronize");
}

int photon_crc_stream_on_complete(void* stream, void (*fn)(void* arg), void* arg) {
    if (!fn) return report_error(-EINVAL, "null callback");
    if (photon_crc_device_count() <= 0) return -ENODEV;
    hipError_t e = hipLaunchHostFunc(static_cast<hipStream_t>(stream), fn, arg);
    return e == hipSuccess ? 0 : report_hip_error(e, "hipLaunchHostFunc");
}

int photon_crc_device_alloc(void** ptr, uint64_t nbytes) {
    if (!ptr || !nbytes) return report_error(-EINVAL, "null pointer or zero size");
    if (photon_crc_device_count() <= 0) return -ENODEV;
    hipError_t e = hipMalloc(ptr, nbytes);
    return e == hipSuccess ? 0 : report_hip_error(e, "hipMalloc");
}

int photon_crc_device_free(void* ptr) {
    if (!ptr) return 0;
    pcrc::services_end_before_free();
    hipError_t e = hipFree(ptr);
    return e == hipSuccess ? 0 : report_hip_error(e, "hipFree");
}

int photon_crc_memcpy_async(void* dst, const void* src, uint64_t nbytes, void* stream) {
    if (!nbytes) return 0;
    if (!dst || !src) return report_error(-EINVAL, "null pointer");
    if (photon_crc_device_count() <= 0) return -ENODEV;
    hipError_t e = hipMemcpyAsync(dst, src, nbytes, hipMemcpyDefault, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : report_hip_error(e, "hipMemcpyAsync");
}

int photon_crc_host_register(void* ptr, uint64_t len) {
    if (!ptr || !len) return report_error(-EINVAL, "null or empty range");
    hipError_t e = hipHostRegister(ptr, len, hipHostRegisterMapped | hipHostRegisterPortable);
    if (e != hipSuccess) return report_hip_error(e, "hipHostRegister");
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg[reinterpret_cast<uintptr_t>(ptr)] = len;
    return 0;
}

int photon_crc_host_unregister(void* ptr) {
    hipError_t e = hipHostUnregister(ptr);
    if (e != hipSuccess) return report_hip_error(e, "hipHostUnregister");
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg.erase(reinterpret_cast<uintptr_t>(ptr));
    return 0;
}

int photon_crc32c_file_strided(int fd, uint64_t offset, uint64_t stride, uint64_t nbytes, uint64_t count,
                               uint32_t seed0, uint32_t* h_out) {
    if (!count) return 0;
    if (fd < 0 || !h_out || stride < nbytes || !nbytes) return report_error(-EINVAL, "bad arguments");
    if (photon_crc_device_count() <= 0) return -ENODEV;
    // Records per chunk; a chunk's read span is rounded out to 4 KiB.
    uint64_t per = kChunk / stride;
    if (per == 0) per = 1;
    if (per > count) per = count;
    const uint64_t span_max = (per - 1) * stride + nbytes + 2 * kAlign;
    ChunkPair cb;
    if (int prc = checkout_pair(span_max, &cb)) return prc;
    struct Return {
        ChunkPair& p;
        ~Return() { return_pair(p); }
    } give_back{cb};

    const uint64_t nchunks = (count + per - 1) / per;
    std::mutex mu;
    std::condition_variable cv;
    int ready[2] = {-1, -1};  // chunk index held by each buffer, -1 = free
    int64_t skew[2] = {0, 0};  // record 0 of the chunk sits at buf + skew
    int read_rc = 0;
    std::string read_err;
    bool stop = false;

    std::thread reader([&] {
        for (uint64_t c = 0; c < nchunks; ++c) {
            const int slot = (int)(c & 1);
            {
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return ready[slot] < 0 || stop; });
                if (stop) return;
            }
            const uint64_t first = c * per;
            const uint64_t k = count - first < per ? count - first : per;
            const uint64_t lo = offset + first * stride;
            const uint64_t hi = lo + (k - 1) * stride + nbytes;
            const uint64_t alo = lo & ~(kAlign - 1);
            const uint64_t ahi = (hi + kAlign - 1) & ~(kAlign - 1);
            std::string err;
            int rc = read_span_parallel(fd, static_cast<uint8_t*>(cb.buf[slot]), hi - alo, ahi - alo, alo, &err);
            std::unique_lock<std::mutex> g(mu);
            if (rc) {
                read_rc = rc;
                read_err = err;
                stop = true;
                cv.notify_all();
                return;
            }
            skew[slot] = (int64_t)(lo - alo);
            ready[slot] = (int)c;
            cv.notify_all();
        }
    });

    int rc = 0;
    for (uint64_t c = 0; c < nchunks && !rc; ++c) {
        const int slot = (int)(c & 1);
        {
            std::unique_lock<std::mutex> g(mu);
            cv.wait(g, [&] { return ready[slot] == (int)c || stop; });
            if (ready[slot] != (int)c) {
                rc = read_rc ? read_rc : -EIO;
                break;
            }
        }
        const uint64_t first = c * per;
        const uint64_t k = count - first < per ? count - first : per;
        rc = photon_crc32c_host_batch_strided(static_cast<uint8_t*>(cb.buf[slot]) + skew[slot], stride, nbytes, k,
                                              seed0, nullptr, h_out + first);
        std::unique_lock<std::mutex> g(mu);
        ready[slot] = -1;
        cv.notify_all();
    }
    {
        std::unique_lock<std::mutex> g(mu);
        stop = true;
        cv.notify_all();
    }
    reader.join();
    if (read_rc) return report_error(read_rc, read_err.c_str());
    return rc;
}

}  // extern "C"
