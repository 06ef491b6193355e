// checked_batch.cpp -- pinned IOAlloc pool + batched CheckedMessage checksums
// (include/photon_crc/checked_batch.h).
//
// Reference behaviour mirrored:
//   IOAlloc::allocate / deallocate callbacks   common/io-alloc.h:31-85
//   Crc32Hasher::extend_hash                   rpc/serialize.h:239-252
//   CheckedMessage::validate_checksum          rpc/serialize.h:266-275
// The checksums themselves are computed by photon_crc32c_batch_msg_n (HIP).
#include <photon_crc/checked_batch.h>

#include <errno.h>
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <map>
#include <mutex>
#include <thread>
#include <string>
#include <unordered_map>
#include <vector>

#include "internal.h"

namespace {

using pcrc::report_error;
using pcrc::report_hip_error;
using pcrc::registered_range_check;

// ------------------------------------------------------------------ pool
constexpr int kMinClass = 12;               // 4 KiB blocks
constexpr int kMaxClass = 26;               // 64 MiB blocks
constexpr size_t kSlabBytes = 64ull << 20;  // pinned in 64 MiB slabs

struct Slab {
    size_t size;
    int cls;        // block class, -1 for a dedicated (oversized) slab
    uint32_t used;  // blocks handed out
};

struct Pool {
    std::mutex mu;
    std::map<uintptr_t, Slab> slabs;            // keyed by base address
    std::vector<void*> free_[kMaxClass + 1];
    std::unordered_map<uintptr_t, uintptr_t> live;  // block -> slab base
    uint64_t pinned = 0, in_use = 0;

    // Slab containing [p, p+n), or slabs.end().
    std::map<uintptr_t, Slab>::iterator find(uintptr_t p, uint64_t n) {
        auto it = slabs.upper_bound(p);
        if (it == slabs.begin()) return slabs.end();
        --it;
        if (p + n > it->first + it->second.size || p + n < p) return slabs.end();
        return it;
    }
};

Pool& pool() {
    static Pool* p = new Pool;  // never destroyed: callbacks may run at exit
    return *p;
}

int size_class(uint64_t n) {
    int c = kMinClass;
    while ((1ull << c) < n) ++c;
    return c;
}

void* pin(size_t bytes) {
    void* p = nullptr;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable);
    if (e != hipSuccess) {
        report_hip_error(e, "hipHostMalloc");
        return nullptr;
    }
    return p;
}

// Is [p, p+n) memory the kernels may read? Returns the device address of p
// (same as p for hipHostMalloc'd and device memory), or nullptr; *host says
// whether the bytes live in host memory (read over the host link).
const void* device_address(const void* p, uint64_t n, bool* host) {
    *host = true;
    {
        // Pinned-pool memory: [p, p+n) must lie inside ONE live block
        // (the slab alone let a segment run past its IOAlloc block).
        Pool& P = pool();
        std::lock_guard<std::mutex> lk(P.mu);
        const uintptr_t q = reinterpret_cast<uintptr_t>(p);
        auto it = P.find(q, 1);
        if (it != P.slabs.end()) {
            const uint64_t bsz = it->second.cls < 0 ? it->second.size : 1ull << it->second.cls;
            const uintptr_t blk = it->first + (q - it->first) / bsz * bsz;
            if (!P.live.count(blk) || n > bsz || q - blk > bsz - n) return nullptr;
            return p;
        }
    }
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    // The whole range [p, p+n) must lie inside the one allocation or
    // registration that p belongs to, else the kernels would read past it:
    // device memory is checked against its allocation, host memory against a
    // photon_crc_host_register registration (memory registered by other code
    // keeps the start-pointer check: HIP does not report those ranges).
    if (a.type == hipMemoryTypeDevice) {
        void* lo = nullptr;
        size_t size = 0;
        if (hipMemGetAddressRange(&lo, &size, const_cast<void*>(p)) == hipSuccess && size) {
            const uintptr_t q = reinterpret_cast<uintptr_t>(p), b0 = reinterpret_cast<uintptr_t>(lo);
            if (q < b0 || n > size || q - b0 > size - n) return nullptr;
        } else {
            (void)hipGetLastError();
        }
    } else if (registered_range_check(p, n) == 0) {
        // Host memory registered through photon_crc_host_register or a vDMA
        // target's register_memory: against its registration. (hipHostMalloc
        // memory from other code keeps the start-pointer check: HIP does not
        // report the range of registered host memory reliably --
        // hipMemGetAddressRange refused in-range vDMA registrations.)
        return nullptr;
    }
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) {
        *host = false;
        return p;
    }
    if (a.type == hipMemoryTypeHost && a.devicePointer && a.hostPointer)
        return static_cast<const char*>(a.devicePointer) + (static_cast<const char*>(p) -
                                                             static_cast<const char*>(a.hostPointer));
    return nullptr;
}

// Lane-group size for a batch: segments read over the host link go faster in
// wide groups (1 KiB contiguous per row instead of 128 B: 41.5 -> 52.1 GiB/s
// on the C5 shape, profiles/r01_rpc_lanes.jsonl); device memory keeps the
// automatic choice (8 lanes for 8 KiB segments is the fastest there).
int lanes_for(uint64_t host_bytes, uint64_t total_bytes) { return 2 * host_bytes >= total_bytes ? 64 : 0; }

struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev) {
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && cur != dev && hipSetDevice(dev) == hipSuccess) prev = cur;
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace

// ----------------------------------------------------------- batch object
struct photon_crc_msg_batch {
    int dev = 0;
    uint32_t flags = 0;
    uint32_t max_msg = 0, max_seg = 0;
    // pinned host staging
    photon_crc_iovec* h_iov = nullptr;
    uint64_t* h_start = nullptr;
    uint32_t* h_expect = nullptr;
    uint32_t* h_out = nullptr;
    // device side (zero-copy: device addresses of the pinned staging above)
    bool zero_copy = true;
    photon_crc_iovec* d_iov = nullptr;
    uint64_t* d_start = nullptr;
    uint32_t* d_out = nullptr;
    uint32_t* d_seg = nullptr;  // segment CRCs of the two-kernel form (device memory)
    // 16 zero bytes of device memory: an object body's m_checksum is hashed
    // as this zero word instead of being zeroed in the caller's message
    // (no host memset on a TRUSTED batch's device body, refilled
    // bodies re-masked on every submit, the caller's object left unmodified).
    uint32_t* d_zero = nullptr;
    hipEvent_t done_ev = nullptr;
    uint64_t nmsg = 0, nseg = 0;
    uint64_t nseg_caller = 0;  // segments as the caller counts them (a body = one), against max_seg
    uint64_t host_bytes = 0, total_bytes = 0;  // payload in host memory / all (lane choice)
    bool submitted = false;
    std::atomic<bool> completed{false};    // results on the host and counted
    std::atomic<int64_t> mismatches{0};
    // Completion callback of the latest submit: done_ev fires
    // before the host function runs, so a batch is only free for the next
    // submit / reset / destroy once the callback has RETURNED as well; until
    // then those calls return -EBUSY (destroy waits), so the next run cannot
    // overwrite the verdicts the callback is reading.
    void (*user_done)(void*) = nullptr;
    void* user_arg = nullptr;
    std::atomic<int> cb_running{0};
};

namespace {

void free_batch(photon_crc_msg_batch* b) {
    pcrc::services_end_before_free();
    if (b->done_ev) (void)hipEventDestroy(b->done_ev);
    for (void* p : {(void*)b->h_iov, (void*)b->h_start, (void*)b->h_expect, (void*)b->h_out})
        if (p) (void)hipHostFree(p);
    if (!b->zero_copy)
        for (void* p : {(void*)b->d_iov, (void*)b->d_start, (void*)b->d_out})
            if (p) (void)hipFree(p);
    if (b->d_seg) (void)hipFree(b->d_seg);
    if (b->d_zero) (void)hipFree(b->d_zero);
    delete b;
}

// Count the mismatches of a finished run (results already on the host).
void settle(photon_crc_msg_batch* b) {
    int64_t bad = 0;
    for (uint64_t i = 0; i < b->nmsg; ++i) bad += b->h_out[i] != b->h_expect[i];
    b->mismatches.store(bad, std::memory_order_relaxed);
    b->completed.store(true, std::memory_order_release);
}

// The host function of a submit with a callback: runs after done_ev (stream
// order), so the verdicts are on the host. It settles the batch WITHOUT any
// HIP call (host functions must not call HIP), so result() inside the
// callback needs none either, then runs the user's callback.
void done_trampoline(void* p) {
    auto* b = static_cast<photon_crc_msg_batch*>(p);
    if (!b->completed.load(std::memory_order_acquire)) settle(b);
    b->user_done(b->user_arg);
    b->cb_running.store(0, std::memory_order_release);
}

// Results are on the host: count mismatches once.
int64_t finish(photon_crc_msg_batch* b) {
    if (!b->completed.load(std::memory_order_acquire)) {
        hipError_t e = hipEventSynchronize(b->done_ev);
        if (e != hipSuccess) return report_hip_error(e, "hipEventSynchronize");
        settle(b);
    }
    return b->mismatches.load(std::memory_order_relaxed);
}

}  // namespace

extern "C" {

int photon_crc_pinned_allocate(void*, photon_crc_range size, void** ptr) {
    if (!ptr || size.min <= 0 || size.max < size.min) return report_error(-EINVAL, "bad IOAlloc range");
    Pool& P = pool();
    const uint64_t n = (uint64_t)size.max;
    const int cls = size_class(n);
    std::lock_guard<std::mutex> lk(P.mu);
    void* blk = nullptr;
    uintptr_t slab_base = 0;
    if (cls > kMaxClass) {
        blk = pin(n);
        if (!blk) return -ENOMEM;
        slab_base = reinterpret_cast<uintptr_t>(blk);
        P.slabs[slab_base] = Slab{n, -1, 0};
        P.pinned += n;
    } else {
        auto& fl = P.free_[cls];
        if (fl.empty()) {
            char* s = static_cast<char*>(pin(kSlabBytes));
            if (!s) return -ENOMEM;
            P.slabs[reinterpret_cast<uintptr_t>(s)] = Slab{kSlabBytes, cls, 0};
            P.pinned += kSlabBytes;
            for (size_t off = kSlabBytes; off >= (1ull << cls); off -= 1ull << cls) fl.push_back(s + off - (1ull << cls));
        }
        blk = fl.back();
        fl.pop_back();
        slab_base = P.find(reinterpret_cast<uintptr_t>(blk), 1)->first;
    }
    P.slabs[slab_base].used++;
    P.live[reinterpret_cast<uintptr_t>(blk)] = slab_base;
    P.in_use += cls > kMaxClass ? n : (1ull << cls);
    *ptr = blk;
    return size.max;
}

int photon_crc_pinned_deallocate(void*, void* ptr) {
    Pool& P = pool();
    std::lock_guard<std::mutex> lk(P.mu);
    auto it = P.live.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == P.live.end()) return report_error(-EINVAL, "pointer not from photon_crc_pinned_allocate");
    Slab& s = P.slabs[it->second];
    s.used--;
    if (s.cls < 0) {
        P.in_use -= s.size;
    } else {
        P.in_use -= 1ull << s.cls;
        P.free_[s.cls].push_back(ptr);
    }
    P.live.erase(it);
    return 0;
}

int photon_crc_pinned_stats(uint64_t* slab_bytes, uint64_t* in_use_bytes) {
    Pool& P = pool();
    std::lock_guard<std::mutex> lk(P.mu);
    if (slab_bytes) *slab_bytes = P.pinned;
    if (in_use_bytes) *in_use_bytes = P.in_use;
    return 0;
}

int64_t photon_crc_pinned_release(void) {
    Pool& P = pool();
    std::lock_guard<std::mutex> lk(P.mu);
    int64_t released = 0;
    for (auto it = P.slabs.begin(); it != P.slabs.end();) {
        if (it->second.used) {
            ++it;
            continue;
        }
        const uintptr_t lo = it->first, hi = lo + it->second.size;
        if (it->second.cls >= 0) {
            auto& fl = P.free_[it->second.cls];
            std::vector<void*> keep;
            keep.reserve(fl.size());
            for (void* p : fl)
                if (reinterpret_cast<uintptr_t>(p) < lo || reinterpret_cast<uintptr_t>(p) >= hi) keep.push_back(p);
            fl.swap(keep);
        }
        (void)hipHostFree(reinterpret_cast<void*>(lo));
        P.pinned -= it->second.size;
        released += (int64_t)it->second.size;
        it = P.slabs.erase(it);
    }
    return released;
}

photon_crc_msg_batch* photon_crc_msg_batch_create(uint32_t max_messages, uint32_t max_segments, uint32_t flags) {
    if (!max_messages || !max_segments) {
        report_error(-EINVAL, "empty batch capacity");
        return nullptr;
    }
    if (photon_crc_device_count() <= 0) return nullptr;  // error text set by the probe
    auto* b = new photon_crc_msg_batch;
    b->flags = flags;
    b->max_msg = max_messages;
    b->max_seg = max_segments;
    hipError_t e = hipGetDevice(&b->dev);
    // Descriptor slots: the caller's segments plus, per message, the zero word
    // an object body is hashed with (max_segments keeps its
    // meaning, one segment per body).
    const uint64_t M = max_messages, S = (uint64_t)max_segments + max_messages;
    b->zero_copy = !(flags & PHOTON_CRC_BATCH_STAGED);
    auto hm = [&](void** p, uint64_t n) {
        if (e == hipSuccess) e = hipHostMalloc(p, n, hipHostMallocMapped | hipHostMallocPortable);
    };
    auto dm = [&](void** p, void* host, uint64_t n) {
        if (e != hipSuccess) return;
        // Zero-copy: the kernels read the descriptors from and write the
        // verdicts to the pinned staging directly (no H2D / D2H copies: one
        // launch per submit).
        e = b->zero_copy ? hipHostGetDevicePointer(p, host, 0) : hipMalloc(p, n);
    };
    hm((void**)&b->h_iov, S * sizeof(photon_crc_iovec));
    hm((void**)&b->h_start, (M + 1) * 8);
    hm((void**)&b->h_expect, M * 4);
    hm((void**)&b->h_out, M * 4);
    dm((void**)&b->d_iov, b->h_iov, S * sizeof(photon_crc_iovec));
    dm((void**)&b->d_start, b->h_start, (M + 1) * 8);
    dm((void**)&b->d_out, b->h_out, M * 4);
    if (e == hipSuccess) e = hipMalloc((void**)&b->d_seg, S * 4);
    if (e == hipSuccess) e = hipMalloc((void**)&b->d_zero, 16);
    // complete before any launch on any stream (a plain hipMemset is queued on
    // the null stream, which does not order against non-blocking streams)
    if (e == hipSuccess) e = hipMemsetAsync(b->d_zero, 0, 16, nullptr);
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&b->done_ev, hipEventDisableTiming);
    if (e != hipSuccess) {
        report_hip_error(e, "photon_crc_msg_batch_create");
        free_batch(b);
        return nullptr;
    }
    b->h_start[0] = 0;
    return b;
}

void photon_crc_msg_batch_destroy(photon_crc_msg_batch* b) {
    if (!b) return;
    if (b->submitted && !b->completed) (void)hipEventSynchronize(b->done_ev);
    while (b->cb_running.load(std::memory_order_acquire)) std::this_thread::yield();  // its callback returns first
    free_batch(b);
}

int64_t photon_crc_msg_batch_add(photon_crc_msg_batch* b, const photon_crc_iovec* iov, uint32_t iovcnt,
                                 const void* body, uint64_t body_length, uint32_t expected) {
    if (!b || (iovcnt && !iov)) return report_error(-EINVAL, "null batch or iovector");
    if (b->submitted) return report_error(-EBUSY, "batch already submitted; reset it first");
    const bool has_body = body && body_length;  // serialize.h:271
    // The body is the message object itself (DeserializerIOV::deserialize
    // passes t, serialize.h:462-463) unless the batch is DETACHED_BODY: then
    // Crc32Hasher accumulates the payload's CRC INTO m_checksum, which is the
    // body's first 4 bytes (the CheckedMessage<> base of a Photon message),
    // and hashes the body with it. A CRC whose init equals its first data
    // word is the CRC (init 0) of the data with that word zeroed, so the
    // reference's value is crc32c(body with m_checksum = 0) and the payload
    // does not enter it (tests/golden/ioalloc_binding.json).
    // The batch hashes the body as two segments, the batch's own device zero
    // word in place of m_checksum and then body[4, len): the same CRC, with
    // the caller's object never written (device or host, TRUSTED or not) and
    // the word masked again on every resubmit of refilled bodies.
    const bool object_body = has_body && !(b->flags & PHOTON_CRC_BATCH_DETACHED_BODY);
    if (object_body && body_length < 4) return report_error(-EINVAL, "message body shorter than its m_checksum");
    // The caller's count: one segment for an object body (its payload does
    // not enter the CRC), else the iovector plus the body; the zero word of an
    // object body takes one of the max_messages extra descriptor slots.
    const uint64_t nput = object_body ? 1u : (uint64_t)iovcnt + (has_body ? 1u : 0u);
    if (b->nmsg >= b->max_msg || b->nseg_caller + nput > b->max_seg) return report_error(-ENOSPC, "batch is full");
    const bool trusted = b->flags & PHOTON_CRC_BATCH_TRUSTED;
    uint64_t s = b->nseg;
    uint64_t host = 0, total = 0;
    // The device address of [p, p + n) (checked unless TRUSTED); null if not device-accessible.
    auto resolve = [&](const void* p, uint64_t n, bool* in_host) -> const void* {
        *in_host = true;  // trusted batches: assume RPC payloads in pinned host memory
        return trusted ? p : device_address(p, n, in_host);
    };
    auto put = [&](const void* d, uint64_t n, bool in_host) {
        if (!n) return;  // crc32c_extend over 0 bytes is the identity
        b->h_iov[s++] = photon_crc_iovec{d, n};
        total += n;
        if (in_host) host += n;
    };
    if (object_body) {
        bool in_host = true;
        const void* d = resolve(body, body_length, &in_host);
        if (!d) return report_error(-EFAULT, "body is not device-accessible (pin it: photon_crc_pinned_allocate)");
        put(b->d_zero, 4, false);  // validate_checksum's `m_checksum = Hasher::init_value()` (serialize.h:268)
        put(static_cast<const uint8_t*>(d) + 4, body_length - 4, in_host);
    } else {
        for (uint32_t k = 0; k <= iovcnt; ++k) {
            const void* p = k < iovcnt ? iov[k].base : body;
            const uint64_t n = k < iovcnt ? iov[k].len : (has_body ? body_length : 0);
            if (!n) continue;
            bool in_host = true;
            const void* d = resolve(p, n, &in_host);
            if (!d)
                return report_error(-EFAULT, "segment is not device-accessible (pin it: photon_crc_pinned_allocate)");
            put(d, n, in_host);
        }
    }
    b->nseg = s;
    b->nseg_caller += nput;
    b->host_bytes += host;
    b->total_bytes += total;
    b->h_expect[b->nmsg] = expected;
    b->h_start[++b->nmsg] = s;
    return (int64_t)(b->nmsg - 1);
}

int photon_crc_msg_batch_submit(photon_crc_msg_batch* b, void* stream, void (*done)(void* arg), void* arg) {
    if (!b) return report_error(-EINVAL, "null batch");
    if (b->cb_running.load(std::memory_order_acquire))
        return report_error(-EBUSY, "completion callback of the previous submit still running");
    if (b->submitted && !b->completed) {
        // A caller driven by the `done` callback never called wait(): if the
        // previous submit has finished, settle it and go on; -EBUSY only while
        // it is really still running.
        hipError_t q = hipEventQuery(b->done_ev);
        if (q == hipErrorNotReady) return report_error(-EBUSY, "batch still running");
        if (q != hipSuccess) return report_hip_error(q, "hipEventQuery");
        int64_t frc = finish(b);
        if (frc < 0) return (int)frc;
    }
    b->completed.store(false, std::memory_order_relaxed);  // before anything of this run is enqueued
    DeviceScope scope(b->dev);
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipError_t e = hipSuccess;
    int rc = 0;
    if (b->nmsg) {
        if (!b->zero_copy) {
            if (b->nseg)
                e = hipMemcpyAsync(b->d_iov, b->h_iov, b->nseg * sizeof(photon_crc_iovec), hipMemcpyHostToDevice, st);
            if (e == hipSuccess) e = hipMemcpyAsync(b->d_start, b->h_start, (b->nmsg + 1) * 8, hipMemcpyHostToDevice, st);
            if (e != hipSuccess) return report_hip_error(e, "hipMemcpyAsync(descriptors)");
        }
        rc = pcrc::batch_msg_lanes(b->d_iov, b->d_start, b->nmsg, b->nseg, 0, nullptr, nullptr, b->d_out, stream,
                                   lanes_for(b->host_bytes, b->total_bytes), b->d_seg);
        if (rc) return rc;
        if (!b->zero_copy) {
            e = hipMemcpyAsync(b->h_out, b->d_out, b->nmsg * 4, hipMemcpyDeviceToHost, st);
            if (e != hipSuccess) return report_hip_error(e, "hipMemcpyAsync(results)");
        }
    }
    e = hipEventRecord(b->done_ev, st);
    if (e == hipSuccess && done) {
        b->user_done = done;
        b->user_arg = arg;
        b->cb_running.store(1, std::memory_order_release);
        e = hipLaunchHostFunc(st, done_trampoline, b);
        if (e != hipSuccess) b->cb_running.store(0, std::memory_order_release);
    }
    if (e != hipSuccess) return report_hip_error(e, "completion");
    b->submitted = true;
    return 0;
}

int64_t photon_crc_msg_batch_wait(photon_crc_msg_batch* b) {
    if (!b) return report_error(-EINVAL, "null batch");
    if (!b->submitted) return report_error(-EINVAL, "batch not submitted");
    return finish(b);
}

int photon_crc_msg_batch_result(photon_crc_msg_batch* b, uint64_t i, uint32_t* crc) {
    if (!b || i >= b->nmsg) return report_error(-EINVAL, "bad batch or index");
    if (!b->submitted) return report_error(-EBUSY, "batch not submitted");
    if (!b->completed) {
        hipError_t e = hipEventQuery(b->done_ev);
        if (e == hipErrorNotReady) return report_error(-EBUSY, "batch still running");
        if (e != hipSuccess) return report_hip_error(e, "hipEventQuery");
        int64_t rc = finish(b);
        if (rc < 0) return (int)rc;
    }
    if (crc) *crc = b->h_out[i];
    return b->h_out[i] == b->h_expect[i] ? 1 : 0;
}

uint64_t photon_crc_msg_batch_count(const photon_crc_msg_batch* b) { return b ? b->nmsg : 0; }

int photon_crc_msg_batch_reset(photon_crc_msg_batch* b) {
    if (!b) return report_error(-EINVAL, "null batch");
    if (b->cb_running.load(std::memory_order_acquire))
        return report_error(-EBUSY, "completion callback of the previous submit still running");
    if (b->submitted && !b->completed) {
        int64_t rc = finish(b);
        if (rc < 0) return (int)rc;
    }
    b->nmsg = b->nseg = b->nseg_caller = 0;
    b->host_bytes = b->total_bytes = 0;
    b->submitted = false;
    b->completed.store(false, std::memory_order_relaxed);
    b->mismatches.store(0, std::memory_order_relaxed);
    return 0;
}

}  // extern "C"
