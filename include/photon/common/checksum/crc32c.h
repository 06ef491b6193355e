/*
 * photon/common/checksum/crc32c.h -- drop-in interface of the MI355X build.
 *
 * Declares exactly the entry points of PhotonLibOS's
 * common/checksum/crc32c.h:20-92 (same names, types, linkage and dispatch
 * pointers), so Photon code that includes this header and links
 * libphoton_checksum.so instead of Photon's crc.cpp/crc_tables.cpp objects
 * keeps compiling and behaving identically:
 *   raw CRC-32C, reflected polynomial 0x82F63B78, init = caller's crc,
 *   no final xor; crc32c("123456789") == 0x58E3FA20.
 * The batched device engine is declared in <photon_crc/crc32c_gpu.h>.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string_view>

// Engines (crc32c.h:20-22 of the reference).
uint32_t crc32c_sw(const uint8_t* buffer, size_t nbytes, uint32_t crc);
uint32_t crc32c_hw(const uint8_t* data, size_t nbytes, uint32_t crc);

// Dispatch pointers, chosen once before main() (reference crc.cpp:126-175).
extern uint32_t (*crc32c_auto)(const uint8_t* data, size_t nbytes, uint32_t crc);
extern void (*crc32c_series_auto)(const uint8_t* buffer, uint32_t part_size, uint32_t n_parts,
                                  uint32_t* crc_parts);
extern uint32_t (*crc32c_combine_auto)(uint32_t crc1, uint32_t crc2, uint32_t len2);
extern uint32_t (*crc32c_combine_series_auto)(uint32_t* crc, uint32_t part_size, uint32_t n_parts);

inline uint32_t crc32c_extend(const void* data, size_t nbytes, uint32_t crc) {
    return crc32c_auto(static_cast<const uint8_t*>(data), nbytes, crc);
}
inline uint32_t crc32c(const void* data, size_t nbytes) { return crc32c_extend(data, nbytes, 0); }
inline uint32_t crc32c_extend(std::string_view text, uint32_t crc) {
    return crc32c_extend(text.data(), text.size(), crc);
}
inline uint32_t crc32c(std::string_view text) { return crc32c_extend(text, 0); }

// CRCs of n_parts consecutive parts of part_size bytes (reference
// crc32c.h:47-57). crc32c_series_hw keeps the reference's observable result
// for part_size < 8 (all zeros; crc.cpp:481-500).
void crc32c_series_sw(const uint8_t* buffer, uint32_t part_size, uint32_t n_parts, uint32_t* crc_parts);
void crc32c_series_hw(const uint8_t* buffer, uint32_t part_size, uint32_t n_parts, uint32_t* crc_parts);
inline void crc32c_series(const uint8_t* buffer, uint32_t part_size, uint32_t n_parts, uint32_t* crc_parts) {
    crc32c_series_auto(buffer, part_size, n_parts, crc_parts);
}

// crc(A||B) from crc(A), crc(B) and |B| (reference crc32c.h:59-66).
uint32_t crc32c_combine_sw(uint32_t crc1, uint32_t crc2, uint32_t len2);
uint32_t crc32c_combine_hw(uint32_t crc1, uint32_t crc2, uint32_t len2);
inline uint32_t crc32c_combine(uint32_t crc1, uint32_t crc2, uint32_t len2) {
    return crc32c_combine_auto(crc1, crc2, len2);
}

// Left fold of combine over equal-size parts (reference crc32c.h:68-74).
uint32_t crc32c_combine_series_sw(uint32_t* crc, uint32_t part_size, uint32_t n_parts);
uint32_t crc32c_combine_series_hw(uint32_t* crc, uint32_t part_size, uint32_t n_parts);
inline uint32_t crc32c_combine_series(uint32_t* crc, uint32_t part_size, uint32_t n_parts) {
    return crc32c_combine_series_auto(crc, part_size, n_parts);
}

struct CRC32C_Component {
    uint32_t crc;
    uint32_t size;
};

// Remove known prefix/suffix CRCs from a whole-buffer CRC (reference
// crc32c.h:76-87). all.size < prefix.size + suffix.size: errno = EINVAL, 0.
uint32_t crc32c_trim_sw(CRC32C_Component all, CRC32C_Component prefix, CRC32C_Component suffix);
uint32_t crc32c_trim_hw(CRC32C_Component all, CRC32C_Component prefix, CRC32C_Component suffix);
extern uint32_t (*crc32c_trim_auto)(CRC32C_Component all, CRC32C_Component prefix, CRC32C_Component suffix);
inline uint32_t crc32c_trim(CRC32C_Component all, CRC32C_Component prefix, CRC32C_Component suffix) {
    return crc32c_trim_auto(all, prefix, suffix);
}

inline bool is_crc32c_hw_available() { return crc32c_auto != crc32c_sw; }

// Extra engines the reference exports and its tests call
// (common/checksum/test/test_checksum.cpp:86-87).
uint32_t crc32c_hw_simple(const uint8_t* data, size_t nbytes, uint32_t crc);
uint32_t crc32c_hw_portable(const uint8_t* data, size_t nbytes, uint32_t crc);
