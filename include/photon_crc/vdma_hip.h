/*
 * vdma_hip.h -- a device-memory vDMA target/initiator for PhotonLibOS's
 * vDMA interface (net/vdma.h:13-77), part of libphoton_checksum.so
 * (producers of device-resident checksum input).
 *
 * Behavioural model: Photon's shared-memory implementation
 * (net/vdma/shm.cpp:23-312), with HBM instead of a POSIX shm segment:
 *
 *   new_hip_vdma_target(name, size, unit, device)
 *       hipMalloc's `size` bytes on `device` (-1 = current) and carves them
 *       into size/unit buffers of `unit` bytes. alloc(n) hands out the
 *       lowest free buffer and only accepts n == unit (shm.cpp:188-191);
 *       with every buffer in use it retries (yielding the OS thread) and then
 *       returns nullptr (shm.cpp:196-203). dealloc returns it (0; -1 for a
 *       buffer of another target). id() is 16 bytes {uint64 index, uint64
 *       unit}, the encoding of shm.cpp:45-54. When `name` is non-null the
 *       target publishes the region's HIP IPC handle in the POSIX shm object
 *       `name`, so an initiator in another process can map it; the object is
 *       unlinked when the target is destroyed.
 *       register_memory(buf, n): device memory is wrapped as is; host memory
 *       is pinned and mapped (hipHostRegister) so kernels read it in place.
 *       (The shm target does not implement it, shm.cpp:210-218.)
 *
 *   new_hip_vdma_initiator(name, size)
 *       opens the handle the target `name` published, in another process
 *       (HIP does not open an IPC handle in the process that exported it;
 *       there, use the target's buffers directly; nullptr if the handle
 *       cannot be opened). map(id) returns the buffer at this process's
 *       address of the region; mapping an id twice fails (shm.cpp:265-274);
 *       unmap forgets it. write/read(vbuf, size, offset): initiator and
 *       target address the same HBM, so no bytes move; write makes this
 *       process's preceding device work on the buffer visible to the target
 *       (device synchronise + system fence) and read is the matching acquire.
 *       Both check that [offset, offset+size) lies inside the buffer
 *       (-1, errno = EINVAL otherwise). (The shm initiator returns -1,
 *       shm.cpp:286-294.)
 *
 * Buffers of both are device-accessible: crc32c_vdma_batch checksums any
 * number of them in one launch (raw CRC-32C, seed 0 = crc32c(address(), n)).
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <photon/net/vdma.h>

namespace photon {

// type_code() values of the HIP buffers (vDMABufferType::kSharedMem is 0).
enum vDMAHipBufferType {
    kHipDeviceMem = 0x48495001,      // a unit of a target's HBM region (or an initiator's mapping of it)
    kHipRegisteredMem = 0x48495002,  // caller memory from register_memory
};

vDMATarget* new_hip_vdma_target(const char* name, size_t size, size_t unit, int device = -1);
vDMAInitiator* new_hip_vdma_initiator(const char* name, size_t size);

// CRC-32C (seed 0) of bufs[i]'s first lens[i] bytes (lens == nullptr: the
// whole buf_size()) into h_out[i], on the current device, one batched launch.
// Every buffer must be device-accessible (the HIP buffers above, or any
// device / pinned memory); 0, or a negative errno (-EFAULT for a buffer the
// GPU cannot read, -EINVAL for lens[i] > buf_size()).
int crc32c_vdma_batch(vDMABuffer* const* bufs, const uint64_t* lens, size_t n, uint32_t* h_out,
                      void* stream = nullptr);

}  // namespace photon
