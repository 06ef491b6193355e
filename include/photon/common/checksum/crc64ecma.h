/*
 * photon/common/checksum/crc64ecma.h -- drop-in interface of the MI355X build
 * for PhotonLibOS's CRC-64/ECMA-182 (reference common/checksum/crc64ecma.h:20-87):
 * reflected polynomial 0xC96C5795D7870F42, init and result inverted
 * (crc.cpp:119-122). Same names, types, linkage and dispatch pointers.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string_view>

uint64_t crc64ecma_sw(const uint8_t* buffer, size_t nbytes, uint64_t crc);
uint64_t crc64ecma_hw(const uint8_t* buffer, size_t nbytes, uint64_t crc);

extern uint64_t (*crc64ecma_auto)(const uint8_t* data, size_t nbytes, uint64_t crc);
extern void (*crc64ecma_series_auto)(const uint8_t* buffer, uint32_t part_size, uint32_t n_parts,
                                     uint64_t* crc_parts);
extern uint64_t (*crc64ecma_combine_auto)(uint64_t crc1, uint64_t crc2, uint32_t len2);
extern uint64_t (*crc64ecma_combine_series_auto)(uint64_t* crc, uint32_t part_size, uint32_t n_parts);

inline uint64_t crc64ecma_extend(const void* data, size_t nbytes, uint64_t crc) {
    return crc64ecma_auto(static_cast<const uint8_t*>(data), nbytes, crc);
}
inline uint64_t crc64ecma_extend(std::string_view text, uint64_t crc) {
    return crc64ecma_extend(text.data(), text.size(), crc);
}
// Returns uint32_t like the reference (crc64ecma.h:32-34 truncates the CRC).
inline uint32_t crc64ecma(std::string_view text) { return crc64ecma_extend(text, 0); }
inline uint64_t crc64ecma(const void* buffer, size_t nbytes, uint64_t crc) {
    return crc64ecma_extend(buffer, nbytes, crc);
}
inline bool is_crc64ecma_hw_available() { return crc64ecma_auto != crc64ecma_sw; }

// Declared (but never defined) by the reference (crc64ecma.h:45-50, 61-66);
// defined here.
void crc64ecma_series_sw(const uint8_t* buffer, uint32_t part_size, uint32_t n_parts, uint64_t* crc_parts);
void crc64ecma_series_hw(const uint8_t* buffer, uint32_t part_size, uint32_t n_parts, uint64_t* crc_parts);
inline void crc64ecma_series(const uint8_t* buffer, uint32_t part_size, uint32_t n_parts, uint64_t* crc_parts) {
    crc64ecma_series_auto(buffer, part_size, n_parts, crc_parts);
}

uint64_t crc64ecma_combine_sw(uint64_t crc1, uint64_t crc2, uint32_t len2);
uint64_t crc64ecma_combine_hw(uint64_t crc1, uint64_t crc2, uint32_t len2);
inline uint64_t crc64ecma_combine(uint64_t crc1, uint64_t crc2, uint32_t len2) {
    return crc64ecma_combine_auto(crc1, crc2, len2);
}

uint64_t crc64ecma_combine_series_sw(uint64_t* crc, uint32_t part_size, uint32_t n_parts);
uint64_t crc64ecma_combine_series_hw(uint64_t* crc, uint32_t part_size, uint32_t n_parts);
inline uint64_t crc64ecma_combine_series(uint64_t* crc, uint32_t part_size, uint32_t n_parts) {
    return crc64ecma_combine_series_auto(crc, part_size, n_parts);
}

struct CRC64ECMA_Component {
    uint64_t crc;
    uint64_t size;
};

uint64_t crc64ecma_trim_hw(CRC64ECMA_Component all, CRC64ECMA_Component prefix, CRC64ECMA_Component suffix);
uint64_t crc64ecma_trim_sw(CRC64ECMA_Component all, CRC64ECMA_Component prefix, CRC64ECMA_Component suffix);
extern uint64_t (*crc64ecma_trim_auto)(CRC64ECMA_Component all, CRC64ECMA_Component prefix,
                                       CRC64ECMA_Component suffix);
inline uint64_t crc64ecma_trim(CRC64ECMA_Component all, CRC64ECMA_Component prefix, CRC64ECMA_Component suffix) {
    return crc64ecma_trim_auto(all, prefix, suffix);
}
