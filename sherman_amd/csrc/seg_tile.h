// seg_tile.h — one 1024-op tile of the insert segmentation (the staged
// segments: runs of ops on one page that gets a new key): k_seg_fill's body
// (util.hip, one tile per block).
// (Round 5 measured a one-wave tile, 16 ops per lane at 32 VGPRs: 23.6
// against 13.5 us alone in C5's profile window, and no better beside the
// ordering, 32-33 us either way; the 256-thread tile stays.  Holding the
// pages in registers and loading the look-back words together took C5's
// step 196.9 -> 191.4 us; one copy of the late-word path (not one per
// batched word) took the kernel 74 -> 61 VGPRs, so its blocks fit beside
// k_bin_unique's (112 VGPRs x 4 waves per SIMD): 190.6 -> 188.5 us.  The tile inside the upsert kernel, round 5's
// second attempt at the fusion, lost 17 % on C5: DESIGN §8.)
#pragma once
#include "device_common.h"
#include "kernels.h"

namespace shm {
namespace dev {
namespace segt {

constexpr int kT = 256;                       // threads per block
constexpr int kPer = (int)kSegTile / kT;      // consecutive ops per thread
static_assert(kPer * kT == (int)kSegTile, "tile shape");

// exclusive scan of v over the block's 256 threads; *total = the block sum
template <class T>
__device__ __forceinline__ T block_scan(T v, T* total) {
  __shared__ T ws[kT / kWave];
  T incl = v;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const T y = __shfl_up(incl, off);
    if (lane_id() >= off) incl += y;
  }
  const int w = threadIdx.x / kWave;
  if (lane_id() == kWave - 1) ws[w] = incl;
  __syncthreads();
  T base = 0, sum = 0;
#pragma unroll
  for (int i = 0; i < kT / kWave; ++i) {
    base += i < w ? ws[i] : T(0);
    sum += ws[i];
  }
  __syncthreads();
  *total = sum;
  return base + incl - v;
}

__device__ __forceinline__ uint32_t seg_head(const uint64_t* page, uint64_t i, uint64_t nv) {
  return i < nv && (i == 0 || page[i] != page[i - 1]) ? 1u : 0u;
}

// Only segments whose page gets a new key (pnew[page] == new_mark(tag), set by
// k_locate) need the upsert and split kernels: the others were applied in
// place by k_locate.
__device__ __forceinline__ bool page_new(const uint8_t* pnew, uint64_t pg, uint32_t tag) {
  return pnew[ga_offset(pg) >> 10] == new_mark(tag);
}

// The staged heads of tile x, counted by one thread (seg_tile's fallback):
// the same count tile x publishes, from the same ops and page marks.  A
// plain loop: an unrolled or non-inlined form cost the tile kernel 20 VGPRs.
__device__ __forceinline__ uint32_t tile_heads(const uint64_t* page, uint64_t nv, uint64_t x,
                                               const uint8_t* pnew, uint32_t tag) {
  const uint64_t s0 = x * kSegTile;
  const uint64_t e = s0 + kSegTile < nv ? s0 + kSegTile : nv;
  uint32_t c = 0;
  uint64_t prev = s0 ? page[s0 - 1] : ~0ull;
#pragma unroll 1
  for (uint64_t i = s0; i < e; ++i) {
    const uint64_t cur = page[i];
    if ((i == 0 || cur != prev) && page_new(pnew, cur, tag)) ++c;
    prev = cur;
  }
  return c;
}

// Tile b (whole block): count its staged heads, publish the count in its
// tagged word (chunk tag << 32 | count), sum the words of the tiles before it,
// and fill its segments: seg_start / seg_page at each staged head, seg_end at
// its run's last op + 1 (the run may end in the next tile: read, not waited
// for), and the total at the thread holding the last op.
// Forward progress: a tile waits for an earlier
// tile's word at most `self_after` polls and then counts that tile's staged
// heads itself (tile_heads), so a tile whose block is not placed -- other
// grids holding every slot -- delays the list but never blocks or corrupts
// it, and no wait bound can leave a guessed prefix behind.  In the common
// case the word is there within a few polls and nothing is recounted.
__device__ __forceinline__ void seg_tile(const uint64_t* page, uint64_t nv, uint64_t b,
                                         uint64_t* lbw, uint32_t* seg_start, uint32_t* seg_end,
                                         uint64_t* seg_page, uint32_t* num_seg,
                                         const uint8_t* pnew, uint32_t tag, uint32_t self_after) {
  __shared__ uint32_t s_pre[kT / kWave];
  const uint64_t i0 = b * kSegTile + (uint64_t)threadIdx.x * kPer;
  // the thread's ops' pages, the one before and the one after, held for the
  // fill below (one round of independent loads), then every op's page mark
  // (a second round): the fill re-reads nothing
  uint64_t pg[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) pg[j] = i0 + j < nv ? page[i0 + j] : ~0ull;
  const uint64_t before = i0 > 0 && i0 - 1 < nv ? page[i0 - 1] : ~0ull;
  const uint64_t after = i0 + kPer < nv ? page[i0 + kPer] : ~0ull;
  // page marks and staged heads as bit masks (bit j: op i0 + j)
  uint32_t pn = 0, h = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) pn |= (i0 + j < nv && page_new(pnew, pg[j], tag) ? 1u : 0u) << j;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const uint64_t prv = j ? pg[j - 1] : before;
    h |= (i0 + j < nv && (i0 + j == 0 || pg[j] != prv) ? (pn >> j) & 1u : 0u) << j;
  }
  const uint32_t c = __builtin_popcount(h);
  uint32_t total;
  const uint32_t local = block_scan<uint32_t>(c, &total);
  const uint64_t tg = (uint64_t)tag << 32;
  if (threadIdx.x == 0)
    __hip_atomic_store(lbw + b, tg | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the counts of the tiles before this one: the first kLb words of each
  // thread loaded together (2^20 ops = 1024 tiles: one round), a word not yet
  // published polled after
  constexpr int kLb = 4;
  uint32_t v = 0;
  for (uint64_t x0 = threadIdx.x; x0 < b; x0 += (uint64_t)kLb * kT) {
    uint64_t w[kLb];
#pragma unroll
    for (int k = 0; k < kLb; ++k) {
      const uint64_t x = x0 + (uint64_t)k * kT;
      w[k] = x < b ? __hip_atomic_load(lbw + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : tg;
    }
    // bit k: tile x0 + k kT (< b) not yet published, or the forced recount;
    // a slot past b adds nothing (w = tg | 0)
    uint32_t late = 0;
#pragma unroll
    for (int k = 0; k < kLb; ++k) {
      const bool past = x0 + (uint64_t)k * kT >= b;
      if (past || ((w[k] & ~0xFFFFFFFFull) == tg && self_after))
        v += (uint32_t)w[k];
      else
        late |= 1u << k;
    }
    // the rare path, one copy: poll each late word, then count it ourselves
#pragma unroll 1
    for (; late; late &= late - 1) {
      const uint64_t x = x0 + (uint64_t)__builtin_ctz(late) * kT;
      uint64_t y = 0;
      for (uint32_t spin = 0;; ++spin) {
        if (spin >= self_after) {  // self_after 0: forced (tests)
          y = tile_heads(page, nv, x, pnew, tag);
          break;
        }
        y = __hip_atomic_load(lbw + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((y & ~0xFFFFFFFFull) == tg) break;
        __builtin_amdgcn_s_sleep(1);
      }
      v += (uint32_t)y;
    }
  }
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
  if (lane_id() == 0) s_pre[threadIdx.x / kWave] = v;
  __syncthreads();
  uint32_t pos = local;
#pragma unroll
  for (int w = 0; w < kT / kWave; ++w) pos += s_pre[w];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const uint64_t i = i0 + j;
    if (i >= nv) break;
    const uint32_t hj = (h >> j) & 1u;
    if (hj) {
      seg_start[pos] = (uint32_t)i;
      seg_page[pos] = pg[j];
    }
    pos += hj;
    const uint64_t nxt = j + 1 < kPer ? pg[j + 1] : after;  // ~0 past nv
    if (nxt != pg[j] && ((pn >> j) & 1u)) seg_end[pos - 1] = (uint32_t)(i + 1);
    if (i + 1 == nv) *num_seg = pos;
  }
  __syncthreads();  // s_pre and the scan's words are reused by the next tile
}

}  // namespace segt
}  // namespace dev
}  // namespace shm
