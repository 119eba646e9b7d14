// isort.hip — ordering of an insert batch: sorted by key, one op per key
// (the last writer in batch order), as Tree::insert applied op after op
// leaves it (src/Tree.cpp:353-403, 878-889: a later insert of a key
// overwrites the earlier one).
//
//   1. k_tile_dedup   every 4096-op tile: an LDS hash table keeps each key's
//                     last op (atomic max of the op index), and the tile's
//                     survivors are compacted to its front (gcount).  Heavy
//                     hitters (zipf) shrink to one op per tile here.
//   2. coarse pass    partition.hip: 256 bins by the top 8 bits of the key's
//                     offset in the shard range, carrying the op index.
//   3. k_bin_sort     every bin (<= 8192 ops) fully sorted by (key, index)
//                     in LDS, in place.  A larger bin (skewed keys) sets
//                     kErrSortOverflow and the host re-sorts the batch with
//                     rocPRIM instead.
// The result is what the stable radix sort of (key, index) produced before:
// sorted keys, equal keys adjacent in index order, so mark_unique /
// compact_unique keep working unchanged.
#include "device_common.h"
#include "kernels.h"

namespace shm {
namespace dev {

namespace {

constexpr int kIT = 1024;  // threads per block

__device__ __forceinline__ bool pair_gt(uint64_t ka, uint32_t ia, uint64_t kb, uint32_t ib) {
  return ka > kb || (ka == kb && ia > ib);
}

// ascending bitonic sort of size `m` (power of two, <= capacity) in LDS
template <int PER>
__device__ __forceinline__ void lds_bitonic(uint64_t* key, uint32_t* idx, uint32_t m) {
  const int t = threadIdx.x;
  for (uint32_t k = 2; k <= m; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int r = 0; r < PER / 2; ++r) {
        const uint32_t p = (uint32_t)(r * kIT + t);  // pair index
        if (p < (m >> 1)) {
          const uint32_t i = 2 * j * (p / j) + (p % j);
          const uint32_t l = i + j;
          const bool up = (i & k) == 0;
          const uint64_t a = key[i], b = key[l];
          const uint32_t x = idx[i], y = idx[l];
          if (pair_gt(a, x, b, y) == up) {
            key[i] = b;
            key[l] = a;
            idx[i] = y;
            idx[l] = x;
          }
        }
      }
      __syncthreads();
    }
  }
}

// exclusive block scan of one u32 per thread (kIT threads)
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int t = threadIdx.x, l = lane_id(), w = t >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, off);
    if (l >= off) incl += y;
  }
  if (l == kWave - 1) wsum[w] = incl;
  __syncthreads();
  uint32_t base = 0, all = 0;
  for (int x = 0; x < kIT / kWave; ++x) {
    base += x < w ? wsum[x] : 0;
    all += wsum[x];
  }
  *total = all;
  __syncthreads();
  return base + incl - v;
}

}  // namespace

__global__ __launch_bounds__(kIT) void k_tile_dedup(const uint64_t* __restrict__ keys, uint64_t n,
                                                   uint64_t* __restrict__ keys_out,
                                                   uint32_t* __restrict__ idx_out,
                                                   uint32_t* __restrict__ gcount,
                                                   uint32_t* err) {
  // LDS hash table of the tile's distinct keys: slot -> (key, 1 + last index)
  constexpr int kSlots = 2 * kIsortTile;
  constexpr int PER = kIsortTile / kIT;
  constexpr int SPT = kSlots / kIT;  // slots per thread in the compaction
  __shared__ unsigned long long hkey[kSlots];
  __shared__ uint32_t hidx[kSlots];
  __shared__ uint32_t wsum[kIT / kWave];
  const int t = threadIdx.x;
  const uint64_t base = (uint64_t)blockIdx.x * kIsortTile;
#pragma unroll
  for (int r = 0; r < SPT; ++r) {
    hkey[r * kIT + t] = kKeyMax;  // empty (kKeyMax is never a stored key)
    hidx[r * kIT + t] = 0;
  }
  __syncthreads();
  bool bad = false;
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const uint64_t i = base + (uint64_t)(r * kIT + t);
    if (i >= n) continue;
    const uint64_t k = keys[i];
    if (k == kKeyMax) {
      bad = true;  // kKeyMax cannot be stored (root highest is exclusive, Tree.h:150)
      continue;
    }
    uint32_t h = (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> 50) & (kSlots - 1);
    for (int probe = 0; probe < kSlots; ++probe) {
      const unsigned long long o = atomicCAS(&hkey[h], (unsigned long long)kKeyMax,
                                             (unsigned long long)k);
      if (o == kKeyMax || o == k) {
        atomicMax(&hidx[h], (uint32_t)i + 1u);  // the last writer in batch order
        break;
      }
      h = (h + 1) & (kSlots - 1);
    }
  }
  if (bad) atomicOr(err, kErrKeyMax);
  __syncthreads();
  uint32_t keep = 0;
#pragma unroll
  for (int r = 0; r < SPT; ++r) keep += hkey[SPT * t + r] != kKeyMax ? 1u : 0u;
  uint32_t total;
  uint32_t pos = block_scan(keep, wsum, &total);
#pragma unroll
  for (int r = 0; r < SPT; ++r) {
    const uint64_t k = hkey[SPT * t + r];
    if (k != kKeyMax) {
      keys_out[base + pos] = k;
      idx_out[base + pos] = hidx[SPT * t + r] - 1u;
      ++pos;
    }
  }
  if (t == 0) gcount[blockIdx.x] = total;
}

__global__ __launch_bounds__(kIT) void k_bin_sort(uint64_t* __restrict__ keys1,
                                                 uint32_t* __restrict__ pay1,
                                                 const uint32_t* __restrict__ bins,
                                                 uint32_t* __restrict__ S, uint32_t* err) {
  constexpr int kCap = kFineCap;  // 8192 keys = 96 KB of LDS
  constexpr int PER = kCap / kIT;
  __shared__ uint64_t skey[kCap];
  __shared__ uint32_t sidx[kCap];
  const int t = threadIdx.x;
  // the coarse pass is complete: clear its group sums for the next batch
  if (blockIdx.x == 0)
    for (int j = t; j < kPartGroupWords; j += kIT) S[j] = 0;
  const uint32_t start = bins[2 * blockIdx.x], cnt = bins[2 * blockIdx.x + 1];
  if (cnt <= 1) return;  // block-uniform
  if (cnt > (uint32_t)kCap) {
    if (t == 0) atomicOr(err, kErrSortOverflow);
    return;
  }
  uint32_t m = 2;
  while (m < cnt) m <<= 1;
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const uint32_t o = (uint32_t)(r * kIT + t);
    if (o < m) {
      skey[o] = o < cnt ? keys1[start + o] : kKeyMax;
      sidx[o] = o < cnt ? pay1[start + o] : ~0u;
    }
  }
  __syncthreads();
  lds_bitonic<PER>(skey, sidx, m);
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const uint32_t o = (uint32_t)(r * kIT + t);
    if (o < cnt) {
      keys1[start + o] = skey[o];
      pay1[start + o] = sidx[o];
    }
  }
}

void launch_tile_dedup(const uint64_t* keys, uint64_t n, uint64_t* keys_out, uint32_t* idx_out,
                       uint32_t* gcount, uint32_t* err, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_tile_dedup, dim3((unsigned)((n + kIsortTile - 1) / kIsortTile)),
                     dim3(kIT), 0, s, keys, n, keys_out, idx_out, gcount, err);
}

void launch_bin_sort(uint64_t* keys1, uint32_t* pay1, const uint32_t* bins, uint32_t* S,
                     uint32_t* err, hipStream_t s) {
  hipLaunchKernelGGL(k_bin_sort, dim3(kCoarse), dim3(kIT), 0, s, keys1, pay1, bins, S, err);
}

}  // namespace dev
}  // namespace shm
