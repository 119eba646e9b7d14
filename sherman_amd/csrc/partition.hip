// partition.hip — order a get batch by its top 16 key bits so the queries a
// wave walks together share their internal pages (one page read per group,
// not per query), and put the results back in input order afterwards.
//
// Two-level MSD counting partition.  Every kernel spans the whole chip and
// every global store is a contiguous run: scatters are staged through LDS
// (a random 8-byte store per element costs a whole line transaction; the
// staged form writes ~16-element runs in the coarse pass and fully
// contiguous ranges in the fine pass).
//   coarse_hist    : input tiles (<= kMaxTiles), 256-bin LDS histogram of the
//                    top 8 bits per tile -> M[tile][bin]; the counts are also
//                    added into S[tile / kTileGroup][bin] (group sums)
//   coarse_scatter : per tile, its offset inside every bin from <= 15 M rows
//                    + <= 16 S rows (no separate scan pass), rank keys in LDS,
//                    stage them bin-major, store the runs to keys1;
//                    pos1[i] = slot of input i (coalesced).  Block 0 writes
//                    the fine-pass chunk table.
//   fine           : one block per <= kFineCap-key chunk of a coarse bin:
//                    counting sort on the next 8 bits inside the chunk's own
//                    range -> keys_out[p], src[p] = keys1 slot it came from
//   (walk)         : result of slot p stored at vals1[src[p]] — a scatter
//                    confined to the chunk's range, which stays in L2
//   unpartition    : out[i] = vals1[pos1[i]], found[i] = out[i] != 0
// Order inside a 16-bit bucket is unspecified; results do not depend on it.
#include "device_common.h"
#include "kernels.h"

namespace shm {
namespace dev {

namespace {
constexpr int kPT = 1024;                 // threads per block
constexpr int kGrp = 2;                   // keys per thread per group
constexpr int kGrpKeys = kPT * kGrp;      // 2048 keys per group
constexpr int kFinePer = kFineCap / kPT;  // keys per thread in the fine pass
constexpr int kTileGroup = 16;            // tiles per S row
constexpr int kGroups = kMaxTiles / kTileGroup;
static_assert(kGroups * kCoarse == kPartGroupWords, "S layout");
static_assert(kFinePer * kPT == kFineCap, "fine cap");
static_assert(kGrpKeys == kIsortTile, "insert tiles are the coarse pass's groups");
static_assert(kCoarse == 256 && kFine == 256, "bin code assumes 256 bins");

// Exclusive scan of v over threads 0..255 of the block (others pass 0 and get
// garbage).  Every thread of the block calls it; it ends with a barrier, so
// `wsum` may be reused by the next call.
__device__ __forceinline__ uint32_t scan256(uint32_t v, uint32_t* wsum) {
  const int t = threadIdx.x;
  uint32_t incl = t < 256 ? v : 0;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, off);
    if (lane_id() >= off) incl += y;
  }
  if (t < 256 && lane_id() == kWave - 1) wsum[t >> 6] = incl;
  __syncthreads();
  uint32_t wbase = 0;
  for (int w = 0; w < (t >> 6) && w < 4; ++w) wbase += wsum[w];
  __syncthreads();
  return wbase + incl - (t < 256 ? v : 0);
}

}  // namespace

// gcount (nullable): group gi (kGrpKeys keys from gi * kGrpKeys) holds only
// its first gcount[gi] keys (the insert path's per-tile de-duplicated runs)
__device__ __forceinline__ bool part_valid(uint64_t i, uint64_t n, const uint32_t* gcount) {
  return i < n && (!gcount || (uint32_t)(i % kGrpKeys) < gcount[i / kGrpKeys]);
}

__global__ __launch_bounds__(kPT) void k_part_coarse_hist(const uint64_t* __restrict__ keys,
                                                          uint64_t n, KeyRange kr,
                                                          const uint32_t* __restrict__ gcount,
                                                          uint32_t groups,
                                                          uint32_t* __restrict__ M,
                                                          uint32_t* __restrict__ S) {
  __shared__ uint32_t h[kCoarse];
  const int t = threadIdx.x;
  if (t < kCoarse) h[t] = 0;
  const uint64_t base = (uint64_t)blockIdx.x * groups * kGrpKeys;
  __syncthreads();
  for (uint32_t g = 0; g < groups; ++g) {
    uint32_t d[kGrp];
#pragma unroll
    for (int r = 0; r < kGrp; ++r) {
      const uint64_t i = base + (uint64_t)g * kGrpKeys + (uint64_t)r * kPT + t;
      d[r] = part_valid(i, n, gcount) ? coarse_of(keys[i], kr) : ~0u;
    }
#pragma unroll
    for (int r = 0; r < kGrp; ++r)
      if (d[r] != ~0u) atomicAdd(&h[d[r]], 1u);
  }
  __syncthreads();
  if (t < kCoarse) {
    const uint32_t c = h[t];
    M[(uint64_t)blockIdx.x * kCoarse + t] = c;
    if (c) atomicAdd(&S[(blockIdx.x / kTileGroup) * kCoarse + t], c);
  }
}

__global__ __launch_bounds__(kPT) void k_part_coarse_scatter(
    const uint64_t* __restrict__ keys, uint64_t n, KeyRange kr,
    const uint32_t* __restrict__ gcount, const uint32_t* __restrict__ pay_in,
    uint32_t groups, uint32_t tiles,
    const uint32_t* __restrict__ M, const uint32_t* __restrict__ S,
    uint64_t* __restrict__ keys1, uint32_t* __restrict__ pay1, uint32_t* __restrict__ pos1,
    uint32_t* __restrict__ chunks, uint32_t nchunk_slots, uint32_t* __restrict__ bins) {
  __shared__ uint64_t stage[kGrpKeys];
  __shared__ uint32_t pstage[kGrpKeys];
  __shared__ uint32_t cnt[kCoarse], lex[kCoarse], gbase[kCoarse];
  __shared__ uint32_t part[6][kCoarse];
  __shared__ uint32_t wsum[4];
  const int t = threadIdx.x;
  const uint32_t tile = blockIdx.x;
  const uint64_t tbase = (uint64_t)tile * groups * kGrpKeys;
  // first group of keys in flight while the bin offsets are summed
  uint64_t k[kGrp];
#pragma unroll
  for (int r = 0; r < kGrp; ++r) {
    const uint64_t i = tbase + (uint64_t)r * kPT + t;
    k[r] = part_valid(i, n, gcount) ? keys[i] : 0;
  }
  {
    // thread (bin b, quarter q): q 0/1 sum S rows [SR q, SR q + SR) -> both
    // the bin total and (rows before this tile's group) the group prefix;
    // q 2/3 sum this group's M rows before this tile (8 each).  All loads
    // issue at once.
    constexpr int SR = kGroups / 2;
    static_assert(SR >= 8 && kTileGroup == 16, "quarter layout");
    const int b = t & (kCoarse - 1), q = t >> 8;
    const uint32_t g = tile / kTileGroup;
    const uint32_t u0 = q < 2 ? SR * q : g * kTileGroup + 8 * (q - 2);
    const uint32_t* src = q < 2 ? S : M;
    const int rows = q < 2 ? SR : 8;
    uint32_t v[SR];
#pragma unroll
    for (int x = 0; x < SR; ++x)
      v[x] = (x < rows && (q < 2 || u0 + x < tile)) ? src[(uint64_t)(u0 + x) * kCoarse + b] : 0;
    uint32_t all = 0, pre = 0;
#pragma unroll
    for (int x = 0; x < SR; ++x) {
      all += v[x];
      pre += (u0 + x) < g ? v[x] : 0;
    }
    if (q < 2) {
      part[q][b] = all;
      part[2 + q][b] = pre;
    } else {
      part[2 + q][b] = all;
    }
    __syncthreads();
  }
  const uint32_t tot = t < kCoarse ? part[0][t] + part[1][t] : 0;
  const uint32_t toff =
      t < kCoarse ? part[2][t] + part[3][t] + part[4][t] + part[5][t] : 0;
  const uint32_t cex = scan256(tot, wsum);
  if (t < kCoarse) gbase[t] = cex + toff;
  if (tile == 0 && bins && t < kCoarse) {
    bins[2 * t] = cex;  // bin table: (start, count) per coarse bin
    bins[2 * t + 1] = tot;
  }
  if (tile == 0 && chunks) {
    // fine-pass chunk table: slot j -> (start, len); len 0 = no chunk
    const uint32_t nch = t < kCoarse ? (tot + kFineCap - 1) / kFineCap : 0;
    const uint32_t cpre = scan256(nch, wsum);
    for (uint32_t j = t; j < nchunk_slots; j += kPT) chunks[2 * j + 1] = 0;
    __syncthreads();
    if (t < kCoarse)
      for (uint32_t c = 0; c < nch; ++c) {
        chunks[2 * (cpre + c)] = cex + c * (uint32_t)kFineCap;
        chunks[2 * (cpre + c) + 1] = min((uint32_t)kFineCap, tot - c * (uint32_t)kFineCap);
      }
  }
  for (uint32_t g = 0; g < groups; ++g) {
    const uint64_t gb = tbase + (uint64_t)g * kGrpKeys;
    uint32_t rank[kGrp];
    if (g) {
#pragma unroll
      for (int r = 0; r < kGrp; ++r) {
        const uint64_t i = gb + (uint64_t)r * kPT + t;
        k[r] = part_valid(i, n, gcount) ? keys[i] : 0;
      }
    }
    if (t < kCoarse) cnt[t] = 0;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kGrp; ++r) {
      const uint64_t i = gb + (uint64_t)r * kPT + t;
      rank[r] = part_valid(i, n, gcount) ? atomicAdd(&cnt[coarse_of(k[r], kr)], 1u) : 0;
    }
    __syncthreads();
    const uint32_t c = t < kCoarse ? cnt[t] : 0;
    const uint32_t lx = scan256(c, wsum);
    if (t < kCoarse) lex[t] = lx;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kGrp; ++r) {
      const uint64_t i = gb + (uint64_t)r * kPT + t;
      if (part_valid(i, n, gcount)) {
        const uint32_t b = coarse_of(k[r], kr);
        stage[lex[b] + rank[r]] = k[r];
        if (pay1) pstage[lex[b] + rank[r]] = pay_in ? pay_in[i] : (uint32_t)i;
        if (pos1) pos1[i] = gbase[b] + rank[r];  // coalesced in i
      }
    }
    __syncthreads();
    // bin-major runs out to keys1
    uint32_t valid = (uint32_t)min((uint64_t)kGrpKeys, n > gb ? n - gb : 0);
    if (gcount && valid) valid = min(valid, gcount[gb / kGrpKeys]);
#pragma unroll
    for (int r = 0; r < kGrp; ++r) {
      const uint32_t j = (uint32_t)(r * kPT + t);
      if (j < valid) {
        const uint64_t key = stage[j];
        const uint32_t b = coarse_of(key, kr);
        keys1[gbase[b] + (j - lex[b])] = key;
        if (pay1) pay1[gbase[b] + (j - lex[b])] = pstage[j];
      }
    }
    __syncthreads();
    if (t < kCoarse) gbase[t] += cnt[t];
  }
}

__global__ __launch_bounds__(kPT) void k_part_fine(const uint64_t* __restrict__ keys1,
                                                   const uint32_t* __restrict__ pay1, KeyRange kr,
                                                   const uint32_t* __restrict__ chunks,
                                                   uint32_t* __restrict__ S,
                                                   uint64_t* __restrict__ keys_out,
                                                   uint32_t* __restrict__ src) {
  __shared__ uint64_t stage[kFineCap];
  __shared__ uint32_t sq[kFineCap];
  __shared__ uint32_t h[kFine];
  __shared__ uint32_t wsum[4];
  const int t = threadIdx.x;
  // the scatter pass is complete: clear the group sums for the next batch
  if (blockIdx.x == 0)
    for (int j = t; j < kPartGroupWords; j += kPT) S[j] = 0;
  struct {
    uint64_t start;
    uint32_t len;
  } ch;
  ch.start = chunks[2 * blockIdx.x];
  ch.len = chunks[2 * blockIdx.x + 1];
  if (ch.len == 0) return;  // block-uniform: grid sized for the worst case
  if (t < kFine) h[t] = 0;
  uint64_t k[kFinePer];
  uint32_t pl[kFinePer];
#pragma unroll
  for (int r = 0; r < kFinePer; ++r) {
    const uint32_t o = (uint32_t)(r * kPT + t);
    k[r] = o < ch.len ? keys1[ch.start + o] : 0;
    pl[r] = (uint32_t)ch.start + o;
    if (pay1 && o < ch.len) pl[r] = pay1[ch.start + o];
  }
  __syncthreads();
  uint32_t rank[kFinePer];
#pragma unroll
  for (int r = 0; r < kFinePer; ++r)
    rank[r] = (uint32_t)(r * kPT + t) < ch.len ? atomicAdd(&h[fine_of(k[r], kr)], 1u) : 0;
  __syncthreads();
  const uint32_t ex = scan256(t < kFine ? h[t] : 0, wsum);
  if (t < kFine) h[t] = ex;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kFinePer; ++r) {
    const uint32_t o = (uint32_t)(r * kPT + t);
    if (o < ch.len) {
      const uint32_t lp = h[fine_of(k[r], kr)] + rank[r];
      stage[lp] = k[r];
      sq[lp] = pl[r];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kFinePer; ++r) {
    const uint32_t o = (uint32_t)(r * kPT + t);
    if (o < ch.len) {
      keys_out[ch.start + o] = stage[o];
      src[ch.start + o] = sq[o];
    }
  }
}

// out[i] = vals1[pos1[i]]; found[i] = (value != kValueNull), exactly the
// reference's search() result (Tree.cpp:445-448)
__global__ __launch_bounds__(256) void k_unpartition(const uint64_t* __restrict__ vals1,
                                                     const uint32_t* __restrict__ pos1,
                                                     uint64_t n, uint64_t* __restrict__ out,
                                                     uint8_t* __restrict__ found) {
  constexpr int kPer = 4;
  const uint64_t base = (uint64_t)blockIdx.x * (256 * kPer) + threadIdx.x;
  uint32_t p[kPer];
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const uint64_t i = base + 256 * r;
    p[r] = i < n ? pos1[i] : 0;
  }
  uint64_t v[kPer];
#pragma unroll
  for (int r = 0; r < kPer; ++r) v[r] = base + 256 * r < n ? vals1[p[r]] : 0;
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const uint64_t i = base + 256 * r;
    if (i < n) {
      out[i] = v[r];
      if (found) found[i] = v[r] != kValueNull ? 1 : 0;
    }
  }
}

uint32_t partition_chunk_slots(uint64_t n) {
  return (uint32_t)((n + kFineCap - 1) / kFineCap + kCoarse);
}

void launch_partition(const uint64_t* keys, uint64_t n, uint64_t key_lo, uint32_t key_bits,
                      uint32_t* M, uint32_t* S, uint32_t* chunks, uint64_t* keys1,
                      uint32_t* pos1, uint64_t* keys_out, uint32_t* src, hipStream_t s) {
  if (!n) return;
  const KeyRange kr{key_lo, key_bits};
  const uint64_t all_groups = (n + kGrpKeys - 1) / kGrpKeys;
  const uint32_t groups = (uint32_t)((all_groups + kMaxTiles - 1) / kMaxTiles);
  const uint32_t tiles = (uint32_t)((all_groups + groups - 1) / groups);
  const uint32_t slots = partition_chunk_slots(n);
  hipLaunchKernelGGL(k_part_coarse_hist, dim3(tiles), dim3(kPT), 0, s, keys, n, kr,
                     (const uint32_t*)nullptr, groups, M, S);
  hipLaunchKernelGGL(k_part_coarse_scatter, dim3(tiles), dim3(kPT), 0, s, keys, n, kr,
                     (const uint32_t*)nullptr, (const uint32_t*)nullptr, groups, tiles,
                     (const uint32_t*)M, (const uint32_t*)S, keys1, (uint32_t*)nullptr, pos1,
                     chunks, slots, (uint32_t*)nullptr);
  hipLaunchKernelGGL(k_part_fine, dim3(slots), dim3(kPT), 0, s, (const uint64_t*)keys1,
                     (const uint32_t*)nullptr, kr, (const uint32_t*)chunks, S, keys_out, src);
}

void launch_partition_coarse(const uint64_t* keys, uint64_t n, const uint32_t* gcount,
                             const uint32_t* pay_in, uint64_t key_lo, uint32_t key_bits,
                             uint32_t* M, uint32_t* S, uint64_t* keys1, uint32_t* pay1,
                             uint32_t* bins, hipStream_t s) {
  if (!n) return;
  const KeyRange kr{key_lo, key_bits};
  const uint64_t all_groups = (n + kGrpKeys - 1) / kGrpKeys;
  const uint32_t groups = (uint32_t)((all_groups + kMaxTiles - 1) / kMaxTiles);
  const uint32_t tiles = (uint32_t)((all_groups + groups - 1) / groups);
  // one group per tile: k_tile_dedup already wrote the histograms
  if (groups > 1)
    hipLaunchKernelGGL(k_part_coarse_hist, dim3(tiles), dim3(kPT), 0, s, keys, n, kr, gcount,
                       groups, M, S);
  hipLaunchKernelGGL(k_part_coarse_scatter, dim3(tiles), dim3(kPT), 0, s, keys, n, kr, gcount,
                     pay_in, groups, tiles, (const uint32_t*)M, (const uint32_t*)S, keys1, pay1,
                     (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, bins);
}

void launch_unpartition(const uint64_t* vals1, const uint32_t* pos1, uint64_t n,
                        uint64_t* out, uint8_t* found, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_unpartition, dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, s,
                       vals1, pos1, n, out, found);
}

}  // namespace dev
}  // namespace shm
