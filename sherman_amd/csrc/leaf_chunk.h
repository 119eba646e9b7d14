// leaf_chunk.h — leaf entries of a lane's dword-aligned page chunk.
//
// Kernels that spread a staged leaf page over a lane group (L lanes, E = 54/L
// consecutive 18 B entries each) read one 18E-byte chunk per lane and unpack
// its entries with compile-time byte offsets (LeafEntry layout, Tree.h:174-187:
// f_version nibble @0, key @1, value @9, r_version nibble @17).
#pragma once
#include "device_common.h"

namespace shm {
namespace dev {

// the 4 bytes starting at byte offset O (compile time) of a dword array
template <int O, int N>
__device__ __forceinline__ uint32_t chunk_bytes4(const uint32_t (&D)[N]) {
  static_assert((O >> 2) + 1 < N || (O & 3) == 0, "chunk bound");
  if constexpr ((O & 3) == 0) {
    return D[O >> 2];
  } else {
    return __builtin_amdgcn_alignbyte(D[(O >> 2) + 1], D[O >> 2], O & 3);
  }
}
template <int O, int N>
__device__ __forceinline__ uint32_t chunk_byte(const uint32_t (&D)[N]) {
  return (D[O >> 2] >> (8 * (O & 3))) & 0xFF;
}

// entry J of the chunk: key, value and the raw version bytes
template <int J, int N>
__device__ __forceinline__ void chunk_entry(const uint32_t (&D)[N], uint64_t& key, uint64_t& val,
                                            uint32_t& fraw, uint32_t& rraw) {
  constexpr int O = kLeafEntry * J;
  key = (uint64_t)chunk_bytes4<O + 1>(D) | ((uint64_t)chunk_bytes4<O + 5>(D) << 32);
  val = (uint64_t)chunk_bytes4<O + 9>(D) | ((uint64_t)chunk_bytes4<O + 13>(D) << 32);
  fraw = chunk_byte<O>(D);
  rraw = chunk_byte<O + 17>(D);
}

// unpack all E entries (E = 2 or 4)
template <int E, int N>
__device__ __forceinline__ void chunk_entries(const uint32_t (&D)[N], uint64_t (&key)[E],
                                              uint64_t (&val)[E], uint32_t (&fraw)[E],
                                              uint32_t (&rraw)[E]) {
  static_assert(E == 2 || E == 4, "entry unpack covers E = 2 and 4");
  chunk_entry<0>(D, key[0], val[0], fraw[0], rraw[0]);
  chunk_entry<1>(D, key[1], val[1], fraw[1], rraw[1]);
  if constexpr (E > 2) {
    chunk_entry<2>(D, key[2], val[2], fraw[2], rraw[2]);
    chunk_entry<3>(D, key[3], val[3], fraw[3], rraw[3]);
  }
}

// first entry of lane chunk li.  Chunks stay inside the page: the last
// lane's chunk is shifted down to end at entry 53, and entries it shares with
// its left neighbour belong to the neighbour (owned iff base + j >= E * li;
// lanes past 54 / E own nothing).
template <int E>
__device__ __forceinline__ int chunk_base(int li) {
  static_assert((kLeafCardinality - E) % 2 == 0, "chunk starts must be dword aligned");
  return E * li < kLeafCardinality - E ? E * li : kLeafCardinality - E;
}

}  // namespace dev
}  // namespace shm
