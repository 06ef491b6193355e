// internal.h -- shared by the translation units of libphoton_checksum.so.
#pragma once
#include <hip/hip_runtime_api.h>

namespace pcrc {
// Record the text returned by photon_crc_last_error() on this thread and
// return `code` (report_hip_error: -EIO with the HIP error string).
int report_error(int code, const char* what);
int report_hip_error(hipError_t e, const char* what);
}  // namespace pcrc
