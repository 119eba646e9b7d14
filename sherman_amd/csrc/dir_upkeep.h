// dir_upkeep.h — the leaf directory kept current after each insert chunk
// (tree.cpp insert_apply has the policy: which chunks keep
// it).
//
// The directory (leafdir.hip) maps key prefixes to leaves, the role of the
// reference's IndexCache (include/IndexCache.h:59-259, kept current there by
// the cache's own inserts and invalidated per entry).  After each kept
// chunk's k_upper, k_dir_upkeep (leafdir.hip: a lane per op for the new
// keys, a wave per split segment; the tree is final then, and the upsert's
// and k_upper's dependent chains pay nothing -- done inline in them the same
// work cost C5 +70 us per chunk) applies these rules:
//   * a new key in an empty slot (the no-split branch of leaf_page_store,
//     Tree.cpp:878-912, applied by upsert.hip) adds its (fingerprint, slot) pair
//     to its prefix's pair-form entry, or its fingerprint byte to a
//     fingerprint-form entry of its leaf (dir_note_new);
//   * every page a split wrote (split_wave.h build_leaf_page, Tree.cpp:
//     914-950) rewrites the entries of the prefixes holding its keys that lie
//     wholly inside its fences -- one leaf, its keys' slots -- and hands the
//     one or two prefixes it shares with a neighbour to the summary walk
//     (kDirPairsBad, or kDirFp cleared) (dir_note_split_page);
//   * an entry neither rule keeps exact (a shared prefix, a new key whose
//     leaf its list does not name) is marked kDirFix and listed, and after
//     the chunk k_dir_repair (leafdir.hip) rebuilds it from the tree.
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

// prefix p for k_dir_repair after the chunk (once: the caller saw kDirFix
// clear in the count word its atomic returned)
__device__ __forceinline__ void dir_fix_later(const UpperArgs& u, uint64_t p) {
  if (!u.dir_fix) return;
  const uint32_t i = atomicAdd(u.dir_fix_n + u.par, 1u);
  if (i < u.dir_fix_cap) u.dir_fix[i] = (uint32_t)p;
}

// an entry this chunk cannot keep exact: left to the summary walk until the
// repair after the chunk rewrites it (bad pairs, fingerprints off, listed)
__device__ __forceinline__ void dir_note_stale(const UpperArgs& u, uint32_t* w, uint64_t p) {
  const uint32_t cw = w[7];
  if (cw & kDirFix) return;  // listed already
  const uint32_t old = atomicOr(w + 7, kDirFix | ((cw & kDirPairs) ? kDirPairsBad : 0u));
  if (old & kDirFp) atomicAnd(w + 7, ~kDirFp);
  if (!(old & kDirFix)) dir_fix_later(u, p);
}

__device__ __forceinline__ uint64_t dir_prefix(const UpperArgs& u, const uint32_t* w) {
  return (uint64_t)(reinterpret_cast<const uint64_t*>(w) - u.dir_w) / kDirWords;
}

// dir_note_stale for a wave's set of prefixes at once (lanes with `want`
// hold one prefix each): one round of atomics, one list reservation
__device__ __forceinline__ void dir_note_stale_lanes(const UpperArgs& u, bool want, uint64_t p) {
  uint32_t* w = want ? reinterpret_cast<uint32_t*>(u.dir_w + kDirWords * p) : nullptr;
  bool add = false;
  if (want) {
    const uint32_t old = atomicOr(w + 7, kDirFix | kDirPairsBad);  // (bad: pair form only)
    if (old & kDirFp) atomicAnd(w + 7, ~kDirFp);
    add = !(old & kDirFix);  // the first to mark it lists it
  }
  const uint64_t m = ballot(add);
  if (!m || !u.dir_fix) return;
  uint32_t base = 0;
  if (lane_id() == ctz64(m)) base = atomicAdd(u.dir_fix_n + u.par, (uint32_t)popc64(m));
  base = rl32(base, ctz64(m));
  if (add) {
    const uint32_t i = base + (uint32_t)popc64(m & lanemask_lt());
    if (i < u.dir_fix_cap) u.dir_fix[i] = (uint32_t)p;
  }
}

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
    if (j < 0) {  // a leaf the list does not name (k_dir_pairs' rule): repair
      dir_note_stale(u, w, dir_prefix(u, w));
      return;
    }
    const uint32_t pos = (atomicAdd(w + 7, 1u << 16) >> 16) & 0xFFu;
    if (pos < kDirPairMax)
      reinterpret_cast<uint16_t*>(w + 8)[pos] =
          (uint16_t)(key_fp(k) | (((uint32_t)s | ((uint32_t)j << 6)) << 8));
    else
      atomicOr(w + 7, kDirPairsBad);  // more keys than pairs: unusable (as a build leaves it)
  } else if (u.dir_form == kDirFormFp && (cw & kDirFp)) {
    if (w[0] == pg)
      reinterpret_cast<uint8_t*>(w)[dir_fp_byte(s)] = (uint8_t)key_fp(k);
    else
      dir_note_stale(u, w, dir_prefix(u, w));  // the prefix reached another leaf
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
  // the prefixes it shares with a neighbour (lanes < nst), marked together
  uint64_t stp = 0;
  uint32_t nst = 0;
  while (todo) {  // one prefix per round, in key order
    const int first = ctz64(todo);
    const uint64_t p = rl64(pk, first);
    const uint64_t m = ballot(mine && pk == p);
    todo &= ~m;
    uint32_t* w = reinterpret_cast<uint32_t*>(u.dir_w + kDirWords * p);
    const uint64_t a = lo + (p << sh);
    const bool inside = lowest <= a && highest - 1 >= a + span;
    if (!inside) {  // shared with a neighbour: repaired after the chunk
      if ((uint32_t)lane == nst) stp = p;
      if (nst < (uint32_t)kWave) ++nst;
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
  // the prefixes inside the fences that hold none of the page's keys: their
  // entries may still name the page the split took them from, so they are
  // written too (one leaf, no pairs / the page's fingerprints), one prefix
  // per lane -- an exact entry must never place a new key in the wrong leaf
  // (locate.hip's exact shortcut)
  const uint64_t lo_k = lowest > lo ? lowest : lo;
  if (highest - 1 < lo || ((lo_k - lo) >> sh) >= u.dir_n) {
    dir_note_stale_lanes(u, (uint32_t)lane < nst, stp);
    return;
  }
  const uint64_t pf = (lo_k - lo) >> sh;
  uint64_t pe = ((highest - 1) - lo) >> sh;
  if (pe >= u.dir_n) pe = u.dir_n - 1;
  // the two prefixes at the fences, when they reach past them, even without
  // a key of the page: their leaf lists may name the page the split took
  // the range from (the last page's right end was the old page's), and an
  // exact entry's list must name the leaf of every key of its prefix
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const uint64_t q = e == 0 ? pf : pe;
    const uint64_t a = lo + (q << sh);
    if (!(lowest <= a && highest - 1 >= a + span) && nst < (uint32_t)kWave) {
      if ((uint32_t)lane == nst) stp = q;
      ++nst;
    }
  }
  dir_note_stale_lanes(u, (uint32_t)lane < nst, stp);
  // the keys inside the directory's range: lanes [k0, k0 + nk), sorted
  const uint64_t km = ballot(mine);
  const uint32_t nk = (uint32_t)popc64(km);
  const uint32_t k0 = km ? (uint32_t)ctz64(km) : 0u;
  // the entry body every such prefix gets, words 0..15 from lanes 0..15
  uint32_t body[16];
#pragma unroll
  for (int x = 0; x < 16; ++x) body[x] = shfl32(fpw, x);
  body[0] = pg;
  if (u.dir_form == kDirFormPairs) {
#pragma unroll
    for (int x = 1; x < 16; ++x) body[x] = 0u;
    body[7] = 1u | kDirPairs;
  } else {
    body[7] = 1u | kDirFp;
  }
  for (uint64_t base = pf; base <= pe; base += kWave) {
    const uint64_t p = base + (uint64_t)lane;
    bool todo_p = p <= pe;
    if (todo_p) {
      const uint64_t a = lo + (p << sh);
      todo_p = lowest <= a && highest - 1 >= a + span;
    }
    // does a key of the page lie in prefix p?  (binary search over the
    // sorted prefixes of lanes [k0, k0 + nk); every lane takes part in the
    // exchanges)
    uint32_t l = k0, h = k0 + nk;
#pragma unroll
    for (int it = 0; it < 7; ++it) {
      const uint32_t mid = (l + h) >> 1;
      const uint64_t pm = shfl64(pk, (int)(mid < 63 ? mid : 63));
      if (l < h) {
        if (pm < p)
          l = mid + 1;
        else
          h = mid;
      }
    }
    const uint64_t pl = shfl64(pk, (int)(l < 63 ? l : 63));
    const bool has = l < k0 + nk && pl == p;
    if (todo_p && !has) {
      uint32_t* w = reinterpret_cast<uint32_t*>(u.dir_w + kDirWords * p);
#pragma unroll
      for (int x = 0; x < 16; ++x) w[x] = body[x];
    }
    if (base + kWave < base) break;  // (no wrap)
  }
}

}  // namespace dev
}  // namespace shm
