// internal.h -- shared by the translation units of libphoton_checksum.so.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <photon_crc/crc32c_gpu.h>

namespace pcrc {
// Record the text returned by photon_crc_last_error() on this thread and
// return `code` (report_hip_error: -EIO with the HIP error string).
int report_error(int code, const char* what);
int report_hip_error(hipError_t e, const char* what);
// photon_crc32c_batch_msg_n with an explicit lane-group size (0 = automatic;
// 4, 8, 16, 32 or 64).
// seg_scratch (nseg words, optional): where the two-kernel form keeps the
// segment CRCs when d_seg_out is NULL (else stream-ordered scratch is used).
int batch_msg_lanes(const photon_crc_iovec* d_iov, const uint64_t* d_msg_start, uint64_t nmsg, uint64_t nseg,
                    uint32_t seed0, const uint32_t* d_seeds, uint32_t* d_seg_out, uint32_t* d_out, void* stream,
                    int lanes, uint32_t* seg_scratch = nullptr);
// [p, p+n) against the ranges registered with photon_crc_host_register:
// 1 inside one registration, 0 p is registered but the range runs past it,
// -1 p is in no registration made through this library.
int registered_range_check(const void* p, uint64_t n);
// Record / forget a host range registered with hipHostRegister by another part
// of the library (the vDMA target's register_memory), for the check above.
void record_registration(const void* p, uint64_t n);
void forget_registration(const void* p);
// End the resident small-buffer services running on device `dev` (and wait
// for their waves), so that a device-wide synchronise that follows does not
// wait for their idle time (the next routed call starts them again).
void services_end_on(int dev);
// The same on every device that has one running: before the library's own
// hipFree (which waits for the device's streams), so it does not wait for a
// service's idle time or life.
void services_end_before_free();
}  // namespace pcrc
