// locate.hip — the insert path's descent (Tree::insert down to the target
// level, src/Tree.cpp:353-403, with page_search's fence / sibling rule,
// Tree.cpp:593-663): out_page[i] = the page of level `target_level` whose
// fences [lowest, highest) hold keys[i].
//
// A locate needs a page's header, not its entries: lane = op, and each hop
// reads the 44 B header plus the rear version word straight from global
// memory (two 64 B lines instead of the 1 KB page a get must scan).
//   * target level 0 starts at the leaf directory entry of the key (leafdir.hip;
//     usually the leaf itself, else a covering internal page), level >= 1 at
//     the root;
//   * version check front == rear (Tree.h:306-327), re-read on mismatch;
//   * k >= highest -> sibling (B-link turn right), k < lowest -> error;
//   * internal page above the target: branchless search over its sorted keys
//     (child = #keys <= k, internal_page_search, Tree.cpp:665-685), 6 dependent
//     8 B loads from L2-resident upper levels.
//   * with out_slot (the upsert locate): a leaf that has a summary line
//     (layout.h) is resolved from it instead of its header -- highest and
//     sibling for the fence rule, then the entries whose fingerprint matches
//     the key.  An op whose key the leaf holds (the first valid slot: key
//     equal, value != 0, upsert.hip's rule) is an update: the lane writes
//     the entry -- value, f_version + 1, r_version = f_version
//     (Tree.cpp:878-912) -- with one 18 B write, the page never read whole
//     (write_page_and_unlock of the entry, Tree.cpp:915-920).  No lock word
//     is taken for it: the chunk's keys are unique, so no other op of the
//     chunk touches that entry, and chunks run one after another on the
//     device (the reference's lock_and_read_page, Tree.cpp:851-852, orders
//     concurrent clients; measured: the word's atomic cost 9 us of a 69 us
//     C5 locate and ordered nothing).  Any other op marks its leaf
//     out_new[page] = tag: only such pages are staged by the upsert (under
//     their lock words), which skips the ops applied here.
// Op keys arrive sorted, so neighbouring lanes read the same header lines.
#include <stdlib.h>

#include "device_common.h"
#include "kernels.h"

namespace shm {
namespace dev {

namespace {

constexpr int kLocBlock = 256;

__device__ __forceinline__ uint64_t g_u64(const uint32_t* p, int d) {
  return (uint64_t)p[d] | ((uint64_t)p[d + 1] << 32);
}

}  // namespace

template <bool PAIRS>
__device__ __forceinline__ void locate_body(const WalkArgs& a) {
  const uint64_t i = (uint64_t)blockIdx.x * kLocBlock + threadIdx.x;
  const uint64_t n = a.n_dev ? *a.n_dev : a.n;
  if (i >= n) return;
  const uint64_t k = a.keys[i];
  const bool match = a.out_slot != nullptr && a.target_level == 0;
  const uint64_t v = match ? a.vals[i] : 0;  // with the key: the update needs no later load
  uint64_t ptr = a.root;
  uint32_t err = 0;
  int retries = 0;
  uint64_t out = 0;
  uint32_t slot = 0;
  uint64_t alt = 0;  // a tie's safe start (dir_start_e): an update is found optimistically
  bool known = false;  // an exact entry placed a new key: out is its leaf, no walk
  if (a.dir && a.target_level == 0) {
    u32x4 e[4];
    bool fpform;
    // (alt's address is always passed: a pointer chosen at run time kept it
    // in scratch memory, a store and a load on every op's path)
    ptr = dir_start_e(a.dir, a.dir_lo, a.dir_shift, a.dir_n, a.node, k, ptr, e, fpform, &alt);
    if (!match) alt = 0;
    // a quiet tree's pair form (layout.h kDirPairs): the prefix's own keys'
    // slots, in up to four leaves -- an update found there is written in
    // place like one found through the fingerprints
    bool pu = false;
    const uint32_t pc = PAIRS && match && !fpform ? dir_pair_cand(e, k, pu) : 0u;
    // an exact pair entry without the key (and no tie at a split point):
    // the key is new and belongs to the leaf its split points name
    known = PAIRS && match && pu && a.dir_exact && alt == 0 && ptr_ok(ptr, a.node, a.arena_bytes);
    for (uint32_t rest = pc; rest && !slot; rest &= rest - 1) {  // lowest pair first
      uint32_t pgi;
      int sl;
      dir_pair_slot(e, (int)__builtin_ctz(rest), pgi, sl);
      const uint64_t ga = dir_page_ga(pgi, a.node);
      if (!ptr_ok(ga, a.node, a.arena_bytes)) continue;
      uint32_t* pg = const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(a.arena + ga_offset(ga)));
      uint64_t ek, ev;
      uint32_t ef, er;
      lane_entry(reinterpret_cast<const uint8_t*>(pg), sl, ek, ev, ef, er);
      if (ek == k && ev != kValueNull) {
        const uint32_t nf = ((ef & 0xF) + 1) & 0xF;
        put_leaf_entry(pg, sl, k, v, (ef & 0xF0) | nf, (er & 0xF0) | nf);
        slot = 0x80000000u | (uint32_t)sl;
        out = ga;
      }
    }
    if (known && !slot) out = ptr;
    // (not found through the pairs: the summary walk below, unless exact)
    if (match && fpform && ptr_ok(ptr, a.node, a.arena_bytes)) {
      // the prefix lies in one leaf and the entry holds its fingerprints: an
      // op whose key that leaf holds updates it without the summary line (a
      // key has one valid slot, so a hit through a stale copy is the slot);
      // any other op takes the summary walk below
      const uint32_t* pg = reinterpret_cast<const uint32_t*>(a.arena + ga_offset(ptr));
      uint64_t cand = dir_fp_cand(e, k);
      while (cand) {
        const int sl = ctz64(cand);
        uint64_t ek, ev;
        uint32_t ef, er;
        lane_entry(reinterpret_cast<const uint8_t*>(pg), sl, ek, ev, ef, er);
        if (ek == k && ev != kValueNull) {
          const uint32_t nf = ((ef & 0xF) + 1) & 0xF;
          put_leaf_entry(const_cast<uint32_t*>(pg), sl, k, v, (ef & 0xF0) | nf, (er & 0xF0) | nf);
          slot = 0x80000000u | (uint32_t)sl;
          out = ptr;
          break;
        }
        cand &= cand - 1;
      }
      // an exact fingerprint entry (every slot of the prefix's one leaf)
      // without the key: a new key of this leaf
      if (!slot && a.dir_exact) {
        out = ptr;
        known = true;
      }
    }
  }
  for (int hop = 0; !slot && !known; ++hop) {
    if (hop > kMaxRounds) {
      err |= kErrLocateHops;
      break;
    }
    if (!ptr_ok(ptr, a.node, a.arena_bytes)) {
      err |= kErrBadPtr;
      break;
    }
    const uint64_t off = ga_offset(ptr);
    const uint32_t* pg = reinterpret_cast<const uint32_t*>(a.arena + off);
    if (match) {
      SumLine sl;
      if (sum_read(a.sum, off, k, sl)) {
        if (k >= sl.highest) {  // turn right (Tree.cpp:626-629)
          const uint64_t sib = page_sibling(a.arena + off);
          if (!sib) {
            err |= kErrFence;
            break;
          }
          ptr = sib;
          continue;
        }
        out = ptr;
        uint64_t cand = sl.cand;
        while (cand) {  // the first valid slot holding k (upsert.hip's rule)
          const int sl = ctz64(cand);
          uint64_t ek, ev;
          uint32_t ef, er;
          lane_entry(reinterpret_cast<const uint8_t*>(pg), sl, ek, ev, ef, er);
          if (ek == k && ev != kValueNull) {
            const uint32_t nf = ((ef & 0xF) + 1) & 0xF;
            put_leaf_entry(const_cast<uint32_t*>(pg), sl, k, v, (ef & 0xF0) | nf,
                           (er & 0xF0) | nf);
            slot = 0x80000000u | (uint32_t)sl;
            break;
          }
          cand &= cand - 1;
        }
        if (!slot && alt) {
          // a tie's optimistic leaf does not hold k: a new key may belong to
          // the leaf on its left, so walk again from the safe start
          ptr = alt;
          alt = 0;
          continue;
        }
        break;
      }
    }
    const u32x4 A = *reinterpret_cast<const u32x4*>(pg);      // dwords 0..3
    const u32x4 B = *reinterpret_cast<const u32x4*>(pg + 4);  // dwords 4..7
    const u32x4 C = *reinterpret_cast<const u32x4*>(pg + 8);  // dwords 8..11
    const uint2 Z = *reinterpret_cast<const uint2*>(pg + 254);
    const uint64_t leftmost = (uint64_t)((A.z >> 8) | (A.w << 24)) |
                              ((uint64_t)((A.w >> 8) | (B.x << 24)) << 32);
    const uint64_t sibling = (uint64_t)((B.x >> 8) | (B.y << 24)) |
                             ((uint64_t)((B.y >> 8) | (B.z << 24)) << 32);
    const int level = (int)((B.z >> 8) & 0xFF);  // byte 25
    const int cnt = (int)(int16_t)(B.z >> 16) + 1;
    const uint64_t lowest = (uint64_t)B.w | ((uint64_t)C.x << 32);
    const uint64_t highest = (uint64_t)C.y | ((uint64_t)C.z << 32);
    const bool is_leaf = leftmost == 0;
    const uint32_t rver = (is_leaf ? Z.x : Z.y) & 0xFF;
    if ((A.z & 0xFF) != rver) {  // torn page: read it again
      if (++retries > kMaxRetries) {
        err |= kErrInconsistent;
        break;
      }
      continue;
    }
    if (k >= highest && sibling != 0) {  // turn right (Tree.cpp:626-629)
      ptr = sibling;
      continue;
    }
    if (k < lowest && alt) {  // a tie's optimistic leaf: k lies to its left
      ptr = alt;
      alt = 0;
      continue;
    }
    if (k < lowest || k >= highest || level < a.target_level) {
      err |= kErrFence;
      break;
    }
    if (level == a.target_level) {
      out = ptr;
      break;
    }
    // internal page above the target: number of keys <= k (keys increase)
    int pos = 0;
#pragma unroll
    for (int step = 32; step > 0; step >>= 1) {
      const int idx = pos + step - 1;
      const int ci = idx < 60 ? idx : 60;
      const uint64_t kk = g_u64(pg, 11 + 4 * ci);
      pos += (idx < cnt && kk <= k) ? step : 0;
    }
    ptr = pos == 0 ? leftmost : g_u64(pg, 13 + 4 * (pos - 1));
  }
  if (err) atomicOr(a.err, err);
  a.out_page[i] = out;
  if (match) {
    a.out_slot[i] = slot;
    // a new key (or a leaf without a summary): its page is staged whole
    // (out = 0 after an error marks page 0: staged, rejected as a bad pointer)
    if (!slot && a.out_new) a.out_new[ga_offset(out) >> 10] = new_mark(a.out_new_tag);
  }
  if (match && a.any_new) {
    const uint64_t m = ballot(!slot);
    if (m && lane_id() == ctz64(m)) *a.any_new = a.out_new_tag;  // one store per wave
  }
}

// PAIRS: the pair-aware form, for a directory in pair form; the other keeps
// the fingerprint form's code (and its 82 VGPRs: the pair loop in every
// locate cost C5 2 %, same box)
template <bool PAIRS>
__global__ __launch_bounds__(kLocBlock) void k_locate(WalkArgs a) { locate_body<PAIRS>(a); }
void launch_locate(const WalkArgs& a, uint64_t n_upper, hipStream_t s) {
  if (n_upper == 0) return;
  const dim3 g((unsigned)((n_upper + kLocBlock - 1) / kLocBlock));
  if (a.dir_pairs)
    hipLaunchKernelGGL(k_locate<true>, g, dim3(kLocBlock), 0, s, a);
  else
    hipLaunchKernelGGL(k_locate<false>, g, dim3(kLocBlock), 0, s, a);
}

}  // namespace dev
}  // namespace shm
