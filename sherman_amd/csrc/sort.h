#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace shm {
namespace dev {
size_t sort_pairs_temp_bytes(uint64_t n);
size_t scan_temp_bytes_max(uint64_t n);
hipError_t sort_pairs(void* temp, size_t bytes, const uint64_t* kin,
                      uint64_t* kout, const uint32_t* vin, uint32_t* vout,
                      uint64_t n, hipStream_t s);
hipError_t sort_pairs_u32(void* temp, size_t bytes, const uint32_t* kin,
                          uint32_t* kout, const uint32_t* vin, uint32_t* vout,
                          uint64_t n, hipStream_t s);
size_t scan_temp_bytes(uint64_t n);
hipError_t exclusive_scan_u64(void* temp, size_t bytes, const uint64_t* in,
                              uint64_t* out, uint64_t n, hipStream_t s);
hipError_t exclusive_scan_u32(void* temp, size_t bytes, const uint32_t* in,
                              uint32_t* out, uint64_t n, hipStream_t s);
}  // namespace dev
}  // namespace shm
