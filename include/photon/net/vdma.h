/*
 * photon/net/vdma.h -- the vDMA interface of PhotonLibOS (net/vdma.h:13-77),
 * declared with the same classes, virtual methods (order, signatures) and
 * factory functions, so that the HIP implementation in libphoton_checksum.so
 * (photon_crc/vdma_hip.h) compiles unchanged against Photon's own header.
 *
 *   vDMABuffer    -- a transportable buffer: id() is a binary identity both
 *                    sides translate to an address; address(), buf_size().
 *   vDMATarget    -- owns the memory: alloc/dealloc fixed-size units,
 *                    register_memory/unregister_memory for caller memory.
 *   vDMAInitiator -- the peer: map(id) -> the buffer at its own address,
 *                    unmap, write/read to hand data to / take it from the target.
 *
 * Photon's shared-memory implementation (net/vdma/shm.cpp) is declared for
 * completeness; this library does not define it -- it implements the
 * device-memory target and initiator (new_hip_vdma_target/_initiator).
 */
#pragma once

#include <stddef.h>
#include <sys/types.h>

#include <string_view>

#include <photon/common/object.h>

namespace photon {

enum vDMABufferType {
    kSharedMem
};

class vDMABuffer {
public:
    virtual std::string_view id() const = 0;
    virtual void* address() const = 0;
    virtual size_t buf_size() const = 0;
    virtual int type_code() const = 0;
    virtual bool is_registered() const = 0;
    virtual bool is_valid() const = 0;

protected:
    virtual ~vDMABuffer() {}
};

class vDMATarget : public Object {
public:
    virtual vDMABuffer* alloc(size_t size) = 0;
    virtual int dealloc(vDMABuffer* buf) = 0;
    virtual vDMABuffer* register_memory(void* buf, size_t size) = 0;
    virtual int unregister_memory(vDMABuffer* vbuf) = 0;
};

class vDMAInitiator : public Object {
public:
    virtual vDMABuffer* map(std::string_view id) = 0;
    virtual int unmap(vDMABuffer* buffer) = 0;
    virtual int write(vDMABuffer* vbuf, size_t size, off_t offset) = 0;
    virtual int read(vDMABuffer* vbuf, size_t size, off_t offset) = 0;
};

vDMATarget* new_shm_vdma_target(const char* shm_name, size_t shm_size, size_t unit);
vDMAInitiator* new_shm_vdma_initiator(const char* shm_name, size_t shm_size);

}  // namespace photon
