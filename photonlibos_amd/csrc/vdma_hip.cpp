// vdma_hip.cpp -- device-memory vDMA target/initiator (include/photon_crc/vdma_hip.h)
// for PhotonLibOS's vDMA interface (net/vdma.h:13-77). The shared-memory
// implementation net/vdma/shm.cpp:23-312 is the behavioural model: same id
// encoding, same alloc/dealloc/map/unmap rules; HBM + HIP IPC instead of
// shm_open + mmap.
#include <photon_crc/vdma_hip.h>

#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <photon_crc/checked_batch.h>

#include "internal.h"

namespace photon {
namespace {

using pcrc::report_error;
using pcrc::report_hip_error;

constexpr uint32_t kMagic = 0x56444d48;  // "HMDV"
constexpr int kMaxRetry = 10000;         // shm.cpp:223

// What the target publishes in the POSIX shm object `name`.
struct Published {
    uint32_t magic;
    int32_t device;
    uint64_t size;
    uint64_t unit;
    hipIpcMemHandle_t handle;
};

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

// 16-byte id {index, size} (shm.cpp:45-54).
std::string encode_id(uint64_t idx, uint64_t size) {
    uint64_t v[2] = {idx, size};
    return std::string(reinterpret_cast<const char*>(v), sizeof(v));
}

bool decode_id(std::string_view id, uint64_t* idx, uint64_t* size) {
    if (id.size() != 16) return false;
    uint64_t v[2];
    memcpy(v, id.data(), sizeof(v));
    *idx = v[0];
    *size = v[1];
    return true;
}

class HipBuffer final : public vDMABuffer {
public:
    HipBuffer(uint64_t idx, char* addr, size_t size, int type, const void* owner)
        : idx_(idx), addr_(addr), size_(size), type_(type), owner_(owner), id_(encode_id(idx, size)) {}
    // Registered caller memory: the id carries the address instead of an index.
    HipBuffer(char* addr, size_t size, bool host_pinned, const void* owner)
        : idx_(UINT64_MAX), addr_(addr), size_(size), type_(kHipRegisteredMem), owner_(owner),
          host_pinned_(host_pinned), id_(encode_id(reinterpret_cast<uintptr_t>(addr), size)) {}
    ~HipBuffer() override {}

    std::string_view id() const override { return id_; }
    void* address() const override { return addr_; }
    size_t buf_size() const override { return size_; }
    int type_code() const override { return type_; }
    bool is_registered() const override { return true; }
    bool is_valid() const override { return addr_ != nullptr; }

    uint64_t idx() const { return idx_; }
    const void* owner() const { return owner_; }
    bool host_pinned() const { return host_pinned_; }

private:
    uint64_t idx_;
    char* addr_;
    size_t size_;
    int type_;
    const void* owner_;
    bool host_pinned_ = false;
    std::string id_;
};

class HipTarget final : public vDMATarget {
public:
    ~HipTarget() override {
        std::lock_guard<std::mutex> lk(mu_);
        DeviceScope scope(dev_);
        for (auto& kv : registered_)
            if (kv.second->host_pinned()) (void)hipHostUnregister(kv.second->address());
        registered_.clear();
        pcrc::services_end_before_free();
        if (base_) (void)hipFree(base_);
        if (!name_.empty()) shm_unlink(name_.c_str());
    }

    int init(const char* name, size_t size, size_t unit, int device) {
        if (!unit || size < unit) return report_error(-EINVAL, "vdma target: need unit > 0 and size >= unit");
        if (device < 0 && hipGetDevice(&device) != hipSuccess) return report_error(-ENODEV, "vdma target: no device");
        dev_ = device;
        DeviceScope scope(dev_);
        hipError_t e = hipMalloc(&base_, size);
        if (e != hipSuccess) return report_hip_error(e, "vdma target: hipMalloc");
        size_ = size;
        unit_ = unit;
        const size_t n = size / unit;
        buffers_.reserve(n);
        for (size_t i = 0; i < n; ++i)
            buffers_.emplace_back(new HipBuffer(i, static_cast<char*>(base_) + i * unit, unit, kHipDeviceMem, this));
        used_.assign(n, false);
        if (name && *name) {
            Published pub{};
            pub.magic = kMagic;
            pub.device = dev_;
            pub.size = size;
            pub.unit = unit;
            e = hipIpcGetMemHandle(&pub.handle, base_);
            if (e != hipSuccess) return report_hip_error(e, "vdma target: hipIpcGetMemHandle");
            const int fd = shm_open(name, O_RDWR | O_CREAT | O_TRUNC, 0600);
            if (fd < 0) return report_error(-errno, "vdma target: shm_open");
            const bool ok = ::write(fd, &pub, sizeof(pub)) == (ssize_t)sizeof(pub);
            close(fd);
            if (!ok) {
                shm_unlink(name);
                return report_error(-EIO, "vdma target: publishing the IPC handle");
            }
            name_ = name;
        }
        return 0;
    }

    vDMABuffer* alloc(size_t size) override {
        if (size != unit_) {  // shm.cpp:189-191: only whole units
            errno = EINVAL;
            report_error(-EINVAL, "vdma target: alloc size must equal the unit");
            return nullptr;
        }
        for (int retry = 0; retry <= kMaxRetry; ++retry) {
            {
                std::lock_guard<std::mutex> lk(mu_);
                for (size_t i = 0; i < used_.size(); ++i)
                    if (!used_[i]) {
                        used_[i] = true;
                        return buffers_[i].get();
                    }
            }
            std::this_thread::yield();  // shm.cpp:196-201 yields the photon thread
        }
        errno = ENOBUFS;
        return nullptr;
    }

    int dealloc(vDMABuffer* buf) override {
        auto* hb = dynamic_cast<HipBuffer*>(buf);
        if (!hb || hb->owner() != this || hb->type_code() != kHipDeviceMem) {
            errno = EINVAL;
            return -1;
        }
        std::lock_guard<std::mutex> lk(mu_);
        used_[hb->idx()] = false;
        return 0;
    }

    vDMABuffer* register_memory(void* buf, size_t size) override {
        if (!buf || !size) {
            errno = EINVAL;
            return nullptr;
        }
        DeviceScope scope(dev_);
        hipPointerAttribute_t a;
        bool device_mem = false;
        if (hipPointerGetAttributes(&a, buf) == hipSuccess)
            device_mem = a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged ||
                         (a.type == hipMemoryTypeHost && a.devicePointer);
        else
            (void)hipGetLastError();
        if (!device_mem) {
            hipError_t e = hipHostRegister(buf, size, hipHostRegisterMapped | hipHostRegisterPortable);
            if (e != hipSuccess) {
                report_hip_error(e, "vdma target: hipHostRegister");
                errno = EIO;
                return nullptr;
            }
            pcrc::record_registration(buf, size);  // so batches check segments against it
        }
        std::lock_guard<std::mutex> lk(mu_);
        auto hb = std::unique_ptr<HipBuffer>(new HipBuffer(static_cast<char*>(buf), size, !device_mem, this));
        HipBuffer* raw = hb.get();
        registered_[raw] = std::move(hb);
        return raw;
    }

    int unregister_memory(vDMABuffer* vbuf) override {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = registered_.find(vbuf);
        if (it == registered_.end()) {
            errno = EINVAL;
            return -1;
        }
        if (it->second->host_pinned()) {
            DeviceScope scope(dev_);
            pcrc::forget_registration(it->second->address());
            (void)hipHostUnregister(it->second->address());
        }
        registered_.erase(it);
        return 0;
    }

private:
    std::mutex mu_;
    int dev_ = 0;
    void* base_ = nullptr;
    size_t size_ = 0, unit_ = 0;
    std::string name_;
    std::vector<std::unique_ptr<HipBuffer>> buffers_;
    std::vector<bool> used_;
    std::map<vDMABuffer*, std::unique_ptr<HipBuffer>> registered_;
};

class HipInitiator final : public vDMAInitiator {
public:
    ~HipInitiator() override {
        std::lock_guard<std::mutex> lk(mu_);
        mapped_.clear();
        if (base_) {
            DeviceScope scope(dev_);
            (void)hipIpcCloseMemHandle(base_);
        }
    }

    int init(const char* name, size_t size) {
        if (!name || !*name) return report_error(-EINVAL, "vdma initiator: no name");
        const int fd = shm_open(name, O_RDONLY, 0);
        if (fd < 0) return report_error(-errno, "vdma initiator: shm_open (is the target up?)");
        Published pub{};
        const bool ok = ::read(fd, &pub, sizeof(pub)) == (ssize_t)sizeof(pub);
        close(fd);
        if (!ok || pub.magic != kMagic) return report_error(-EINVAL, "vdma initiator: not a HIP vDMA target");
        if (size && size != pub.size) return report_error(-EINVAL, "vdma initiator: size differs from the target's");
        if (hipGetDevice(&dev_) != hipSuccess) return report_error(-ENODEV, "vdma initiator: no device");
        hipError_t e = hipIpcOpenMemHandle(&base_, pub.handle, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            base_ = nullptr;
            return report_hip_error(e, "vdma initiator: hipIpcOpenMemHandle");
        }
        size_ = pub.size;
        return 0;
    }

    vDMABuffer* map(std::string_view id) override {
        uint64_t idx = 0, bsize = 0;
        if (!decode_id(id, &idx, &bsize) || !bsize || idx >= size_ / bsize || (idx + 1) * bsize > size_) {
            errno = EINVAL;
            return nullptr;
        }
        std::lock_guard<std::mutex> lk(mu_);
        std::string key(id);
        if (mapped_.count(key)) {  // shm.cpp:266-273: an id is mapped once
            errno = EBUSY;
            return nullptr;
        }
        auto hb = std::unique_ptr<HipBuffer>(
            new HipBuffer(idx, static_cast<char*>(base_) + idx * bsize, bsize, kHipDeviceMem, this));
        HipBuffer* raw = hb.get();
        mapped_[key] = std::move(hb);
        return raw;
    }

    int unmap(vDMABuffer* buffer) override {
        if (!buffer) {
            errno = EINVAL;
            return -1;
        }
        std::lock_guard<std::mutex> lk(mu_);
        if (!mapped_.erase(std::string(buffer->id()))) {
            errno = EINVAL;
            return -1;
        }
        return 0;
    }

    int write(vDMABuffer* vbuf, size_t size, off_t offset) override { return fence(vbuf, size, offset); }
    int read(vDMABuffer* vbuf, size_t size, off_t offset) override { return fence(vbuf, size, offset); }

private:
    int fence(vDMABuffer* vbuf, size_t size, off_t offset) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (!vbuf || !mapped_.count(std::string(vbuf->id())) || offset < 0 ||
                (size_t)offset > vbuf->buf_size() || size > vbuf->buf_size() - (size_t)offset) {
                errno = EINVAL;
                return -1;
            }
        }
        DeviceScope scope(dev_);
        pcrc::services_end_on(dev_);  // else the device-wide wait below waits for their idle time
        if (hipDeviceSynchronize() != hipSuccess) {
            errno = EIO;
            return -1;
        }
        std::atomic_thread_fence(std::memory_order_seq_cst);
        return 0;
    }

    std::mutex mu_;
    int dev_ = 0;
    void* base_ = nullptr;
    size_t size_ = 0;
    std::map<std::string, std::unique_ptr<HipBuffer>> mapped_;
};

}  // namespace

vDMATarget* new_hip_vdma_target(const char* name, size_t size, size_t unit, int device) {
    auto* t = new HipTarget;
    if (t->init(name, size, unit, device)) {
        delete t;
        return nullptr;
    }
    return t;
}

vDMAInitiator* new_hip_vdma_initiator(const char* name, size_t size) {
    auto* i = new HipInitiator;
    if (i->init(name, size)) {
        delete i;
        return nullptr;
    }
    return i;
}

int crc32c_vdma_batch(vDMABuffer* const* bufs, const uint64_t* lens, size_t n, uint32_t* h_out, void* stream) {
    if (!n) return 0;
    if (!bufs || !h_out) return report_error(-EINVAL, "null buffers or output");
    if (n > UINT32_MAX) return report_error(-EINVAL, "too many buffers");
    // One single-segment message per buffer through the CheckedMessage batch
    // (per-buffer CRC, seed 0); it checks that every buffer is device-accessible.
    photon_crc_msg_batch* b = photon_crc_msg_batch_create((uint32_t)n, (uint32_t)n, 0);
    if (!b) return -ENOMEM;
    int rc = 0;
    for (size_t i = 0; i < n && !rc; ++i) {
        if (!bufs[i]) {
            rc = report_error(-EINVAL, "null buffer");
            break;
        }
        const uint64_t len = lens ? lens[i] : bufs[i]->buf_size();
        if (len > bufs[i]->buf_size()) {
            rc = report_error(-EINVAL, "length exceeds the buffer");
            break;
        }
        photon_crc_iovec seg{bufs[i]->address(), len};
        const int64_t r = photon_crc_msg_batch_add(b, &seg, 1, nullptr, 0, 0);
        if (r < 0) rc = (int)r;
    }
    if (!rc) rc = photon_crc_msg_batch_submit(b, stream, nullptr, nullptr);
    if (!rc) {
        const int64_t w = photon_crc_msg_batch_wait(b);
        if (w < 0) rc = (int)w;
    }
    for (size_t i = 0; i < n && !rc; ++i) {
        const int r = photon_crc_msg_batch_result(b, i, &h_out[i]);
        if (r < 0) rc = r;
    }
    photon_crc_msg_batch_destroy(b);
    return rc;
}

}  // namespace photon
