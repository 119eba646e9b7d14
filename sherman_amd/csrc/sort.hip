// sort.hip — device-wide primitives from rocPRIM (library sort / scan, the
// analogue of using hipBLASLt for a plain GEMM): stable LSD radix sort of
// (u64 key, u32 index) pairs and exclusive prefix sums.
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "sort.h"

namespace shm {
namespace dev {

size_t sort_pairs_temp_bytes(uint64_t n) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (const uint64_t*)nullptr,
                            (uint64_t*)nullptr, (const uint32_t*)nullptr,
                            (uint32_t*)nullptr, (size_t)n, 0u, 64u);
  return bytes;
}

hipError_t sort_pairs(void* temp, size_t bytes, const uint64_t* kin,
                      uint64_t* kout, const uint32_t* vin, uint32_t* vout,
                      uint64_t n, unsigned begin_bit, hipStream_t s) {
  return rocprim::radix_sort_pairs(temp, bytes, kin, kout, vin, vout, (size_t)n,
                                   begin_bit, 64u, s);
}

size_t scan_temp_bytes(uint64_t n) {
  size_t b64 = 0, b32 = 0;
  (void)rocprim::exclusive_scan(nullptr, b64, (const uint64_t*)nullptr,
                          (uint64_t*)nullptr, (uint64_t)0, (size_t)n,
                          rocprim::plus<uint64_t>());
  (void)rocprim::exclusive_scan(nullptr, b32, (const uint32_t*)nullptr,
                          (uint32_t*)nullptr, (uint32_t)0, (size_t)n,
                          rocprim::plus<uint32_t>());
  return b64 > b32 ? b64 : b32;
}

hipError_t exclusive_scan_u64(void* temp, size_t bytes, const uint64_t* in,
                              uint64_t* out, uint64_t n, hipStream_t s) {
  return rocprim::exclusive_scan(temp, bytes, in, out, (uint64_t)0, (size_t)n,
                                 rocprim::plus<uint64_t>(), s);
}

hipError_t exclusive_scan_u32(void* temp, size_t bytes, const uint32_t* in,
                              uint32_t* out, uint64_t n, hipStream_t s) {
  return rocprim::exclusive_scan(temp, bytes, in, out, (uint32_t)0, (size_t)n,
                                 rocprim::plus<uint32_t>(), s);
}

}  // namespace dev
}  // namespace shm
