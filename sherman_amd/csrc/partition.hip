// partition.hip — bucket a get batch by the top kPartBits key bits, so the
// queries a wave walks together share their internal pages and (for
// same-leaf queries) their leaf read.  Hand-written MSD counting partition:
//   hist    : 1024-thread blocks, one kPartTile-key tile each; keys are loaded
//             up front (16 per thread, full memory-level parallelism), then
//             counted with LDS atomics into a 16 Ki-bin histogram row
//   colscan : per bucket, exclusive prefix of the tile rows (tile-major)
//   scatter : every block scans the 16 Ki bucket totals itself (cheaper than a
//             separate launch), adds its tile's prefix, and places its keys
//             with LDS-atomic cursors; it also records where each input went
//             (pos_of) so results can be gathered back contiguously.
// Order inside a bucket is unspecified (results do not depend on it).
#include "device_common.h"
#include "kernels.h"

namespace shm {
namespace dev {

namespace {
constexpr int kPT = 1024;                     // threads per block
constexpr int kPer = kPartTile / kPT;         // keys per thread (16)
constexpr int kBinsPer = kPartBuckets / kPT;  // bins per thread (16)
static_assert(kPer * kPT == kPartTile, "tile");
static_assert(kBinsPer * kPT == kPartBuckets, "bins");
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
}  // namespace

__global__ __launch_bounds__(kPT) void k_part_hist(const uint64_t* __restrict__ keys,
                                                   uint64_t n, uint32_t* __restrict__ gh) {
  __shared__ __attribute__((aligned(16))) uint32_t h[kPartBuckets];
  const int t = threadIdx.x;
#pragma unroll
  for (int j = 0; j < kBinsPer / 4; ++j)
    reinterpret_cast<u4*>(h)[t + j * kPT] = u4{0, 0, 0, 0};
  const uint64_t base = (uint64_t)blockIdx.x * kPartTile;
  uint32_t d[kPer];
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const uint64_t i = base + (uint64_t)r * kPT + t;
    d[r] = i < n ? (uint32_t)(keys[i] >> (64 - kPartBits)) : ~0u;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kPer; ++r)
    if (d[r] != ~0u) atomicAdd(&h[d[r]], 1u);
  __syncthreads();
  u4* g = reinterpret_cast<u4*>(gh + (uint64_t)blockIdx.x * kPartBuckets);
#pragma unroll
  for (int j = 0; j < kBinsPer / 4; ++j)
    g[t + j * kPT] = reinterpret_cast<const u4*>(h)[t + j * kPT];
}

__global__ __launch_bounds__(256) void k_part_colscan(uint32_t* __restrict__ gh,
                                                      uint32_t tiles,
                                                      uint32_t* __restrict__ tot) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= (uint32_t)kPartBuckets) return;
  uint32_t acc = 0;
  uint32_t t = 0;
  for (; t + 8 <= tiles; t += 8) {
    uint32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = gh[(uint64_t)(t + u) * kPartBuckets + b];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      gh[(uint64_t)(t + u) * kPartBuckets + b] = acc;
      acc += v[u];
    }
  }
  for (; t < tiles; ++t) {
    const uint64_t o = (uint64_t)t * kPartBuckets + b;
    const uint32_t v = gh[o];
    gh[o] = acc;
    acc += v;
  }
  tot[b] = acc;
}

__global__ __launch_bounds__(kPT) void k_part_scatter(const uint64_t* __restrict__ keys,
                                                      uint64_t n,
                                                      const uint32_t* __restrict__ gh,
                                                      const uint32_t* __restrict__ tot,
                                                      uint64_t* __restrict__ out_keys,
                                                      uint32_t* __restrict__ pos_of) {
  __shared__ __attribute__((aligned(16))) uint32_t c[kPartBuckets];
  __shared__ uint32_t wsum[kPT / kWave];
  const int t = threadIdx.x;
  const uint64_t base = (uint64_t)blockIdx.x * kPartTile;
  // issue the key loads first; they land while the bucket scan runs
  uint64_t k[kPer];
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const uint64_t i = base + (uint64_t)r * kPT + t;
    k[r] = i < n ? keys[i] : 0;
  }
  // exclusive scan of the bucket totals: thread t owns bins [16t, 16t+16)
  uint32_t v[kBinsPer];
  uint32_t sum = 0;
#pragma unroll
  for (int j = 0; j < kBinsPer / 4; ++j) {
    const u4 x = reinterpret_cast<const u4*>(tot)[t * (kBinsPer / 4) + j];
    v[4 * j] = x.x; v[4 * j + 1] = x.y; v[4 * j + 2] = x.z; v[4 * j + 3] = x.w;
    sum += x.x + x.y + x.z + x.w;
  }
  uint32_t incl = sum;  // inclusive wave scan (Hillis-Steele over 64 lanes)
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, off);
    if (lane_id() >= off) incl += y;
  }
  if (lane_id() == kWave - 1) wsum[t >> 6] = incl;
  __syncthreads();
  uint32_t wbase = 0;
  for (int w = 0; w < (t >> 6); ++w) wbase += wsum[w];
  uint32_t run = wbase + incl - sum;
  const uint32_t* g = gh + (uint64_t)blockIdx.x * kPartBuckets + t * kBinsPer;
#pragma unroll
  for (int j = 0; j < kBinsPer; ++j) {
    c[t * kBinsPer + j] = run + g[j];
    run += v[j];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const uint64_t i = base + (uint64_t)r * kPT + t;
    if (i < n) {
      const uint32_t p = atomicAdd(&c[k[r] >> (64 - kPartBits)], 1u);
      out_keys[p] = k[r];
      pos_of[i] = p;
    }
  }
}

// vals_out[i] = res[pos_of[i]]; found_out[i] = (value != kValueNull), which is
// exactly the reference's search() result (Tree.cpp:445-448)
__global__ void k_gather_results(const uint64_t* __restrict__ res,
                                 const uint32_t* __restrict__ pos_of, uint64_t n,
                                 uint64_t* __restrict__ vals_out,
                                 uint8_t* __restrict__ found_out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t v = res[pos_of[i]];
  vals_out[i] = v;
  if (found_out) found_out[i] = v != kValueNull ? 1 : 0;
}

void launch_partition(const uint64_t* keys, uint64_t n, uint32_t* gh,
                      uint32_t* tot, uint64_t* out_keys, uint32_t* pos_of,
                      hipStream_t s) {
  if (!n) return;
  const uint32_t tiles = (uint32_t)((n + kPartTile - 1) / kPartTile);
  hipLaunchKernelGGL(k_part_hist, dim3(tiles), dim3(kPT), 0, s, keys, n, gh);
  hipLaunchKernelGGL(k_part_colscan, dim3(kPartBuckets / 256), dim3(256), 0, s, gh,
                     tiles, tot);
  hipLaunchKernelGGL(k_part_scatter, dim3(tiles), dim3(kPT), 0, s, keys, n, gh, tot,
                     out_keys, pos_of);
}

void launch_gather_results(const uint64_t* res, const uint32_t* pos_of,
                           uint64_t n, uint64_t* vals_out, uint8_t* found_out,
                           hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_gather_results, dim3((unsigned)((n + 255) / 256)), dim3(256),
                       0, s, res, pos_of, n, vals_out, found_out);
}

}  // namespace dev
}  // namespace shm
