// lds_dma.h — LDS-DMA page staging shared by the walk kernels.
#pragma once
#include "device_common.h"

// m0 is set by the LDS-DMA asm below; nothing else in these kernels uses it
#pragma clang diagnostic ignored "-Winline-asm"

namespace shm {
namespace dev {

// One page -> one LDS slot: global_load_lds_dwordx4, lane l's 16 bytes land
// at lds_addr + 16 l.  Issued from inline asm on purpose: hipcc treats a
// visible LDS-DMA as a pending LDS write and puts s_waitcnt vmcnt(0) in front
// of every later ds_read, which would drain the whole ring; the ring's waits
// are counted by hand instead (wait_vm below).
__device__ __forceinline__ void glds16(const uint8_t* page, uint32_t lds_addr) {
  const uint64_t ga = (uint64_t)(page + 16 * lane_id());
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "global_load_lds_dwordx4 %0, off"
      :
      : "v"(ga), "s"(lds_addr)
      : "memory", "m0");
}

// the same with the non-temporal policy: a leaf read once per batch should
// not displace the lines that are reused (directory, upper levels)
__device__ __forceinline__ void glds16_nt(const uint8_t* page, uint32_t lds_addr) {
  const uint64_t ga = (uint64_t)(page + 16 * lane_id());
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "global_load_lds_dwordx4 %0, off nt"
      :
      : "v"(ga), "s"(lds_addr)
      : "memory", "m0");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ uint32_t rfl(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// LDS byte address of a __shared__ object (for m0)
template <class T>
__device__ __forceinline__ uint32_t lds_addr_of(const T* p) {
  return rfl((uint32_t)(uintptr_t)((__attribute__((address_space(3))) const T*)p));
}

}  // namespace dev
}  // namespace shm
