// dir_upkeep.h — the leaf directory kept current by the insert chunk's leaf
// writers (tree.cpp dir_maint_enabled has the policy).
//
// The directory (leafdir.hip) maps key prefixes to leaves, the role of the
// reference's IndexCache (include/IndexCache.h:59-259, kept current there by
// the cache's own inserts and invalidated per entry).  Two writers keep it:
//   * a new key in an empty slot (upsert.hip, the no-split branch of
//     leaf_page_store, Tree.cpp:878-912) adds its (fingerprint, slot) pair
//     to its prefix's pair-form entry, or its fingerprint byte to a
//     fingerprint-form entry of its leaf (dir_note_new);
//   * every page a split writes (split_wave.h build_leaf_page, Tree.cpp:
//     914-950) rewrites the entries of the prefixes holding its keys that lie
//     wholly inside its fences -- one leaf, its keys' slots -- and hands the
//     one or two prefixes it shares with a neighbour to the summary walk
//     (kDirPairsBad, or kDirFp cleared) (dir_note_split_page).
// Every entry a get trusts still only names slots to read: a get that does
// not find its key there walks the summary path (get.hip), so the upkeep is
// about cost, never about results.  Prefixes of a split page without keys
// are left as they were: their stale entries can only send a miss on a
// B-link right move.
#pragma once
#include "device_common.h"
#include "kernels.h"

namespace shm {
namespace dev {

__device__ __forceinline__ uint32_t* dir_entry_w(uint64_t* dir, uint64_t lo, uint32_t shift,
                                                 uint64_t n, uint64_t k) {
  if (k < lo || k == kKeyMax) return nullptr;
  const uint64_t p = (k - lo) >> shift;
  return p < n ? reinterpret_cast<uint32_t*>(dir + kDirWords * p) : nullptr;
}

// the entry byte of slot s's fingerprint in the fingerprint form
// (dir_fp_cand's placement: 24 at bytes 4..27, 30 at 32..61)
__device__ __forceinline__ int dir_fp_byte(int s) { return s < 24 ? 4 + s : 8 + s; }

// key k was stored in the empty slot s of leaf page index pg (one lane)
__device__ __forceinline__ void dir_note_new(const UpperArgs& u, uint64_t k, uint32_t pg, int s) {
  uint32_t* w = u.dir_w ? dir_entry_w(u.dir_w, u.dir_lo, u.dir_shift, u.dir_n, k) : nullptr;
  if (!w) return;
  // a plain load: this chunk's other writers only add pairs or flags
  const uint32_t cw = w[7];
  if (u.dir_form == kDirFormPairs) {
    if (!(cw & kDirPairs) || (cw & kDirPairsBad)) return;
    const uint32_t nl = cw & 0xFFu;
    int j = -1;
    for (uint32_t x = 0; x < nl && x < 4; ++x)
      if (w[x] == pg) j = (int)x;
    if (j < 0) {  // a leaf the list does not name (k_dir_pairs' rule)
      atomicOr(w + 7, kDirPairsBad);
      return;
    }
    const uint32_t pos = (atomicAdd(w + 7, 1u << 16) >> 16) & 0xFFu;
    if (pos < kDirPairMax)
      reinterpret_cast<uint16_t*>(w + 8)[pos] =
          (uint16_t)(key_fp(k) | (((uint32_t)s | ((uint32_t)j << 6)) << 8));
    else
      atomicOr(w + 7, kDirPairsBad);  // past the list: unusable for good
  } else if (u.dir_form == kDirFormFp && (cw & kDirFp)) {
    if (w[0] == pg)
      reinterpret_cast<uint8_t*>(w)[dir_fp_byte(s)] = (uint8_t)key_fp(k);
    else
      atomicAnd(w + 7, ~kDirFp);  // the prefix reached another leaf
  }
}

// a prefix shared with a neighbour page: left to the summary walk
__device__ __forceinline__ void dir_note_shared(const UpperArgs& u, uint32_t* w) {
  const uint32_t cw = w[7];
  if (cw & kDirPairs) {
    if (!(cw & kDirPairsBad)) atomicOr(w + 7, kDirPairsBad);
  } else if (cw & kDirFp) {
    atomicAnd(w + 7, ~kDirFp);
  }
}

// One wave: the split wrote leaf page index pg with fences [lowest, highest)
// and c keys, key (sorted) in lane = slot < c.  Rewrites every entry of a
// prefix that holds some of these keys and lies inside the fences, marks
// the shared ones.
__device__ __forceinline__ void dir_note_split_page(const UpperArgs& u, uint32_t pg,
                                                    uint64_t lowest, uint64_t highest,
                                                    uint64_t key, uint32_t c) {
  if (!u.dir_w || u.dir_form == kDirFormNone) return;
  const int lane = lane_id();
  const uint64_t lo = u.dir_lo;
  const uint32_t sh = u.dir_shift;
  const uint64_t span = (1ull << sh) - 1;
  const bool mine = (uint32_t)lane < c && key >= lo && key != kKeyMax &&
                    ((key - lo) >> sh) < u.dir_n;
  const uint64_t pk = mine ? (key - lo) >> sh : 0;
  const uint32_t fp = (uint32_t)lane < c ? key_fp(key) : 0u;
  uint64_t todo = ballot(mine);
  // the fingerprint form's entry body: every slot's fingerprint (the same
  // for every inside prefix of the page); word x of 16 in lane x
  uint32_t fpw = 0;
  if (u.dir_form == kDirFormFp) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int byte = 4 * (lane & 15) + b;
      const int s = byte >= 4 && byte < 28 ? byte - 4 : byte >= 32 && byte < 62 ? byte - 8 : -1;
      const uint32_t f = shfl32(fp, s >= 0 ? s : 0);
      if (s >= 0) fpw |= (f & 0xFFu) << (8 * b);
    }
  }
  while (todo) {  // one prefix per round, in key order
    const int first = ctz64(todo);
    const uint64_t p = rl64(pk, first);
    const uint64_t m = ballot(mine && pk == p);
    todo &= ~m;
    uint32_t* w = reinterpret_cast<uint32_t*>(u.dir_w + kDirWords * p);
    const uint64_t a = lo + (p << sh);
    const bool inside = lowest <= a && highest - 1 >= a + span;
    if (!inside) {
      if (lane == 0) dir_note_shared(u, w);
      continue;
    }
    const uint32_t cnt = (uint32_t)popc64(m);
    uint32_t v = 0;
    if (u.dir_form == kDirFormPairs) {
      // words 0..7: {pg, 0 x 6, 1 leaf | kDirPairs | pairs << 16}; words
      // 8..15: pairs 2x and 2x + 1 = the prefix's keys in slot order
      // (the exchanges run in every lane: uniform control flow)
      const uint32_t q0 = 2u * (uint32_t)(lane & 7);
      const int s0 = first + (int)q0;
      const uint32_t f0 = shfl32(fp, s0 < 63 ? s0 : 62);
      const uint32_t f1 = shfl32(fp, s0 + 1 < 64 ? s0 + 1 : 63);
      if (lane == 0) v = pg;
      if (lane == 7) v = 1u | kDirPairs | ((cnt < 255u ? cnt : 255u) << 16);
      if (lane >= 8 && lane < 16) {
        if (q0 < cnt && q0 < kDirPairMax) v |= (f0 & 0xFFu) | ((uint32_t)s0 << 8);
        if (q0 + 1 < cnt && q0 + 1 < kDirPairMax)
          v |= ((f1 & 0xFFu) | ((uint32_t)(s0 + 1) << 8)) << 16;
      }
    } else {
      v = fpw;
      if (lane == 0) v = pg;
      if (lane == 7) v = 1u | kDirFp;
    }
    if (lane < 16) w[lane] = v;
  }
}

}  // namespace dev
}  // namespace shm
