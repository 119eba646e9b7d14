// sort.hip — device-wide primitives from rocPRIM (library sort / scan, the
// analogue of using hipBLASLt for a plain GEMM): stable LSD radix sort of
// (u64 key, u32 index) pairs and exclusive prefix sums.
#include <algorithm>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "sort.h"

namespace shm {
namespace dev {

size_t scan_temp_bytes(uint64_t n);

// rocPRIM's default dispatch (block sort / merge sort below 2^20 items /
// onesweep).  Forcing onesweep at 0.5 Mi pairs was slower (217 us plus 17
// buffer fills per sort) than the merge path (175 us).
using SortCfg = rocprim::default_config;

static size_t sort_bytes_at(uint64_t n, unsigned begin_bit) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs<SortCfg>(nullptr, bytes, (const uint64_t*)nullptr,
                                  (uint64_t*)nullptr, (const uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (size_t)n, begin_bit, 64u);
  return bytes;
}

static size_t sort32_bytes_at(uint64_t n) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs<SortCfg>(nullptr, bytes, (const uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (size_t)n, 0u, 32u);
  return bytes;
}

// rocPRIM picks block sort / merge sort / onesweep by size, each with its own
// temporary-storage need, so the workspace is the max over every size up to
// n (not just the need at n).  Only full-width sorts are used: partial bit
// ranges (begin_bit > 0) on 64-bit keys returned non-permutations on gfx950
// / ROCm 7.2 in our probe (tools/debug_sorted_walk.py).
size_t sort_pairs_temp_bytes(uint64_t n) {
  size_t best = 0;
  for (uint64_t s = 1; s < n; s = s + 1 > s + s / 32 ? s + 1 : s + s / 32)
    best = std::max(best, std::max(sort_bytes_at(s, 0), sort32_bytes_at(s)));
  return std::max(best, std::max(sort_bytes_at(n, 0), sort32_bytes_at(n)));
}

hipError_t sort_pairs(void* temp, size_t bytes, const uint64_t* kin,
                      uint64_t* kout, const uint32_t* vin, uint32_t* vout,
                      uint64_t n, hipStream_t s) {
  if (sort_bytes_at(n, 0) > bytes) return hipErrorInvalidValue;
  return rocprim::radix_sort_pairs<SortCfg>(temp, bytes, kin, kout, vin, vout, (size_t)n,
                                            0u, 64u, s);
}

hipError_t sort_pairs_u32(void* temp, size_t bytes, const uint32_t* kin,
                          uint32_t* kout, const uint32_t* vin, uint32_t* vout,
                          uint64_t n, hipStream_t s) {
  if (sort32_bytes_at(n) > bytes) return hipErrorInvalidValue;
  return rocprim::radix_sort_pairs<SortCfg>(temp, bytes, kin, kout, vin, vout, (size_t)n,
                                            0u, 32u, s);
}

size_t scan_temp_bytes_max(uint64_t n) {
  size_t best = 0;
  for (uint64_t s = 1; s < n; s = s + 1 > s + s / 32 ? s + 1 : s + s / 32)
    best = std::max(best, scan_temp_bytes(s));
  return std::max(best, scan_temp_bytes(n));
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
  if (scan_temp_bytes(n) > bytes) return hipErrorInvalidValue;
  return rocprim::exclusive_scan(temp, bytes, in, out, (uint64_t)0, (size_t)n,
                                 rocprim::plus<uint64_t>(), s);
}

hipError_t exclusive_scan_u32(void* temp, size_t bytes, const uint32_t* in,
                              uint32_t* out, uint64_t n, hipStream_t s) {
  if (scan_temp_bytes(n) > bytes) return hipErrorInvalidValue;
  return rocprim::exclusive_scan(temp, bytes, in, out, (uint32_t)0, (size_t)n,
                                 rocprim::plus<uint32_t>(), s);
}

}  // namespace dev
}  // namespace shm
