// seg_tile.h — one 1024-op tile of the insert segmentation (the staged
// segments: runs of ops on one page that gets a new key): k_seg_fill's body
// (util.hip, one tile per block), kept apart for a kernel that lists its own
// segments (fusing the segmentation into the upsert kernel).
#pragma once
#include "device_common.h"
#include "kernels.h"

namespace shm {
namespace dev {
namespace segt {

// One tile = one wave (round 5): 1024 ops, 16 consecutive ops per lane,
// streamed in two passes at 32 VGPRs.  A 256-thread block per tile made
// k_seg_fill 4096 waves per C5 chunk; beside the next chunk's k_bin_unique
// (one 16-wave block per CU, 152 KB of LDS, 111 VGPRs: 448 of a SIMD's 512
// VGPRs) one 40-VGPR wave per SIMD fit, so the tiles ran in four rounds
// (30 us in the timed steps against 13.5 alone).  1024 one-wave tiles of 32
// VGPRs fit two per SIMD beside it, and a wave needs no block barrier.
constexpr int kT = kWave;                     // threads per block: one wave
constexpr int kPer = (int)kSegTile / kT;      // consecutive ops per lane
static_assert(kPer * kT == (int)kSegTile, "tile shape");

// Only segments whose page gets a new key (pnew[page] == new_mark(tag), set by
// k_locate) need the upsert and split kernels: the others were applied in
// place by k_locate.
__device__ __forceinline__ bool page_new(const uint8_t* pnew, uint64_t pg, uint32_t tag) {
  return pnew[ga_offset(pg) >> 10] == new_mark(tag);
}

// The staged heads of tile x, counted by one lane (seg_tile's fallback):
// the same count tile x publishes, from the same ops and page marks.
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

// Tile b (one wave): count its staged heads (a staged head is an op whose
// page differs from the previous op's and is marked new), publish the count
// in its tagged word (chunk tag << 32 | count), sum the words of the tiles
// before it, and fill its segments: seg_start / seg_page at each staged
// head, seg_end at its run's last op + 1 (the run may end in the next tile:
// read, not waited for), and the total at the lane holding the last op.
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
  const int lane = lane_id();
  const uint64_t t0 = b * kSegTile;
  const uint64_t i0 = t0 + (uint64_t)lane * kPer;
  // pass 1: this lane's 16 ops, streamed (few registers: the tile must fit
  // beside the ordering's blocks, see kT): staged heads as bits of hm
  uint64_t prev = i0 > 0 && i0 - 1 < nv ? page[i0 - 1] : ~0ull;
  uint32_t hm = 0, c = 0;
#pragma unroll 2
  for (int j = 0; j < kPer; ++j) {
    const uint64_t i = i0 + j;
    const uint64_t cur = i < nv ? page[i] : ~0ull;
    if (i < nv && (i == 0 || cur != prev) && page_new(pnew, cur, tag)) {
      hm |= 1u << j;
      ++c;
    }
    prev = cur;
  }
  // the wave's exclusive scan of the lanes' counts
  uint32_t incl = c;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, off);
    if (lane >= off) incl += y;
  }
  const uint32_t total = (uint32_t)__shfl((int)incl, kWave - 1);
  const uint64_t tg = (uint64_t)tag << 32;
  if (lane == 0) __hip_atomic_store(lbw + b, tg | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the counts of the tiles before this one
  uint32_t v = 0;
  for (uint64_t x = (uint64_t)lane; x < b; x += kWave) {
    uint64_t w = 0;
    for (uint32_t spin = 0;; ++spin) {
      if (spin >= self_after) {
        w = tg | tile_heads(page, nv, x, pnew, tag);
        break;
      }
      w = __hip_atomic_load(lbw + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((w & ~0xFFFFFFFFull) == tg) break;
      __builtin_amdgcn_s_sleep(1);
    }
    v += (uint32_t)w;
  }
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
  // pass 2: the lane's segments (its pages again, from the cache): seg_start
  // / seg_page at each staged head, seg_end at each run end whose page is new
  uint32_t pos = v + incl - c;
  uint64_t cur = i0 < nv ? page[i0] : ~0ull;
#pragma unroll 2
  for (int j = 0; j < kPer; ++j) {
    const uint64_t i = i0 + j;
    if (i >= nv) break;
    const uint64_t nx = i + 1 < nv ? page[i + 1] : ~0ull;
    const bool h = (hm >> j) & 1u;
    if (h) {
      seg_start[pos] = (uint32_t)i;
      seg_page[pos] = cur;
    }
    pos += h ? 1u : 0u;
    const bool tail = i + 1 == nv || nx != cur;
    if (tail && (h || page_new(pnew, cur, tag))) seg_end[pos - 1] = (uint32_t)(i + 1);
    if (i + 1 == nv) *num_seg = pos;
    cur = nx;
  }
}

}  // namespace segt
}  // namespace dev
}  // namespace shm
