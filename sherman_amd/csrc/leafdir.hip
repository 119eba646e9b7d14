// leafdir.hip — the leaf directory: a flat index from key prefixes to leaves.
//
// Plays the role of Sherman's index cache (src/IndexCache.h, include/
// CacheEntry.h: cached level-1 pages let a search jump straight to its leaf;
// dead in the reference fork, Directory.cpp:8/77-79) for the batched get.
// Entry p covers keys [lo_p, lo_p + 2^shift), lo_p = dir_lo + (p << shift),
// and lists the up to four leaves that cover that range, in key order, in
// 32 B (four entries per 128 B L2 line):
//   u32[8] = {pg0, pg1, pg2, pg3, t1, t2, t3, n}
// pg_i = page index of leaf i (GlobalAddress offset / 1 KB), t_i = the top
// 32 bits of (sep_i - lo_p) with sep_i = lowest fence of leaf i (all of it
// when shift <= 32).  A query k starts at leaf i for the largest i < n whose
// t_i is below k's (dir_start, device_common.h).  n == 0 marks a prefix
// spanning more than four leaves: pg0 is then the deepest internal page whose
// fences cover the whole prefix.
//
// Stale entries stay correct: a page's lowest fence never changes (a split
// keeps the left half in place, Tree.cpp:926-945), so ptr_i remains a valid
// B-link entry point for keys >= sep_i and keys past its current highest
// fence move right along the sibling chain (Tree.cpp:626-629).  The host
// rebuilds the directory when the tree has grown enough to make the extra
// hops matter.
#include "device_common.h"
#include "dir_upkeep.h"
#include "kernels.h"

namespace shm {
namespace dev {

namespace {
__device__ __forceinline__ uint64_t pg64(const uint8_t* pg, int o) {  // 4-aligned
  const uint32_t* d = reinterpret_cast<const uint32_t*>(pg + o);
  return (uint64_t)d[0] | ((uint64_t)d[1] << 32);
}
__device__ __forceinline__ uint64_t pg64_b1(const uint8_t* pg, int d) {  // byte 4d+1
  const uint32_t* w = reinterpret_cast<const uint32_t*>(pg) + d;
  return (uint64_t)((w[0] >> 8) | (w[1] << 24)) | ((uint64_t)((w[1] >> 8) | (w[2] << 24)) << 32);
}
// internal_page_search (Tree.cpp:665-685): number of keys <= x
__device__ __forceinline__ int keys_le(const uint8_t* pg, int cnt, uint64_t x) {
  int lo = 0, hi = cnt;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (pg64(pg, kOffRecords + kInternalEntry * mid) <= x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}
}  // namespace

__global__ __launch_bounds__(256) void k_leaf_dir(const uint8_t* __restrict__ arena,
                                                  uint64_t arena_bytes, uint16_t node,
                                                  uint64_t root, uint64_t dir_lo,
                                                  uint32_t shift, uint64_t n_ent,
                                                  uint64_t* __restrict__ dir,
                                                  uint32_t* __restrict__ hint, int from_hint,
                                                  const uint8_t* __restrict__ sum,
                                                  uint32_t* err, int pairs) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_ent) return;
  const uint64_t lo = dir_lo + (p << shift);
  const uint64_t span = (1ull << shift) - 1;
  const uint64_t hi = lo > ~0ull - span ? ~0ull : lo + span;
  uint64_t ptr = root, cover = root;
  uint64_t out[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t h1 = 0, h2 = 0;  // level-1 / level-2 pages on lo's path
  // a rebuild starts at the level-1 page the previous build recorded on lo's
  // path: a page keeps its lowest fence when it splits, so it is still a
  // B-link start for lo (right moves past its new highest fence); the
  // level-2 hint is kept as it was (a stale one is a valid start as well)
  bool hinted = false;
  if (from_hint && hint && hint[p]) {
    ptr = dir_page_ga(hint[p], node);
    h2 = hint[n_ent + p];
    hinted = true;
  }
  bool ok = false;
  for (int it = 0; it < 4096; ++it) {
    if (!ptr_ok(ptr, node, arena_bytes)) break;
    const uint8_t* pg = arena + ga_offset(ptr);
    const uint64_t leftmost = pg64_b1(pg, 2);
    const uint64_t sibling = pg64_b1(pg, 4);
    const uint64_t highest = pg64(pg, kOffHighest);
    if (hinted && (leftmost == 0 || pg[kOffLevel] != 1 || lo < pg64(pg, kOffLowest))) {
      // not a level-1 page on lo's path any more (the root page grew a
      // level): descend from the root
      hinted = false;
      ptr = root;
      h2 = 0;
      continue;
    }
    if (lo >= highest) {  // turn right (Tree.cpp:626-629)
      if (sibling == 0) break;
      ptr = sibling;
      continue;
    }
    if (leftmost != 0) {  // internal: descend towards lo
      const uint32_t lv = pg[kOffLevel];
      if (lv == 1) h1 = dir_page_index(ptr);
      if (lv == 2) h2 = dir_page_index(ptr);
      const int cnt = (int)(int16_t)(pg[kOffLastIndex] | (pg[kOffLastIndex + 1] << 8)) + 1;
      const int c = keys_le(pg, cnt, lo);
      // the deepest internal page whose fences hold the whole prefix (lo is
      // past its lowest on the path): the start of a prefix of > 4 leaves
      if (hi < highest) cover = ptr;
      ptr = c == 0 ? leftmost : pg64(pg, kOffRecords + kInternalEntry * (c - 1) + 8);
      hinted = false;  // below the hinted level now
      continue;
    }
    // leaf containing lo; collect the leaves that cover [lo, hi]
    out[0] = ptr;
    uint64_t h = highest, sib = sibling;
    int n = 1;
    while (h <= hi && sib != 0 && n <= 4) {
      if (n == 4 || !ptr_ok(sib, node, arena_bytes)) {
        n = 5;  // too many leaves: fall back to the covering internal page
        break;
      }
      const uint8_t* sp = arena + ga_offset(sib);
      out[n] = sib;
      out[3 + n] = pg64(sp, kOffLowest);  // sep_n = lowest of ptr_n
      h = pg64(sp, kOffHighest);
      sib = pg64_b1(sp, 4);
      ++n;
    }
    if (n <= 4) {
      out[7] = (uint64_t)n;
    } else {
      for (int i = 0; i < 8; ++i) out[i] = 0;
      out[0] = cover;
    }
    ok = true;
    break;
  }
  if (!ok) {
    atomicOr(err, kErrBadPtr);
    for (int i = 0; i < 8; ++i) out[i] = 0;
    out[0] = root;
  }
  // out = {ptr0..3, sep1..3, n} -> the 64 B entry
  const uint32_t sh = shift > 32 ? shift - 32 : 0;
  uint32_t t[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = (uint32_t)((out[4 + i] - lo) >> sh);
  if (hint) {
    hint[p] = ok ? h1 : 0u;
    hint[n_ent + p] = ok ? h2 : 0u;
  }
  u32x4* e = reinterpret_cast<u32x4*>(dir + kDirWords * p);
  const uint32_t pg0 = dir_page_index(out[0]);
  if (pairs && out[7] >= 1) {
    // the leaf list, pair form: k_dir_pairs adds the prefix's keys
    e[0] = u32x4{pg0, dir_page_index(out[1]), dir_page_index(out[2]), dir_page_index(out[3])};
    e[1] = u32x4{t[0], t[1], t[2], (uint32_t)out[7] | kDirPairs};
    e[2] = u32x4{0u, 0u, 0u, 0u};
    e[3] = u32x4{0u, 0u, 0u, 0u};
    return;
  }
  if (sum && out[7] == 1) {
    // one leaf covers the whole prefix: the entry carries its summary's
    // fingerprints (layout.h kDirFp), so a get of a key it holds reads the
    // entry and then the key's slot, without the summary line
    const u32x4* line = reinterpret_cast<const u32x4*>(sum + (ga_offset(out[0]) >> 10) * kSumBytes);
    u32x4 l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) l[j] = line[j];
    if ((l[0].z & 0xFF) == kSumLeaf) {
      uint8_t fp[kLeafCardinality];
#pragma unroll
      for (int sl = 0; sl < kLeafCardinality; ++sl) {
        const int b = (int)kSumOffFp + sl;
        const u32x4 v = l[b >> 4];
        const int d = (b >> 2) & 3;
        const uint32_t x = d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
        fp[sl] = (uint8_t)(x >> (8 * (b & 3)));
      }
      uint32_t w[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = 0;
      w[0] = pg0;
      w[7] = 1u | kDirFp;
#pragma unroll
      for (int sl = 0; sl < kLeafCardinality; ++sl) {
        const int b = sl < 24 ? 4 + sl : 8 + sl;  // dir_fp_cand's placement
        w[b >> 2] |= (uint32_t)fp[sl] << (8 * (b & 3));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) e[j] = u32x4{w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]};
      return;
    }
  }
  e[0] = u32x4{pg0, dir_page_index(out[1]), dir_page_index(out[2]), dir_page_index(out[3])};
  e[1] = u32x4{t[0], t[1], t[2], (uint32_t)out[7]};
  e[2] = u32x4{0u, 0u, 0u, 0u};
  e[3] = u32x4{0u, 0u, 0u, 0u};
}

void launch_leaf_dir(const uint8_t* arena, uint64_t arena_bytes, uint16_t node, uint64_t root,
                     uint64_t dir_lo, uint32_t shift, uint64_t n_ent, uint64_t* dir,
                     uint32_t* hint, int from_hint, const uint8_t* sum, uint32_t* err,
                     hipStream_t s, int pairs) {
  if (!n_ent) return;
  hipLaunchKernelGGL(k_leaf_dir, dim3((unsigned)((n_ent + 255) / 256)), dim3(256), 0, s, arena,
                     arena_bytes, node, root, dir_lo, shift, n_ent, dir, hint, from_hint, sum,
                     err, pairs);
}

// The pair form's pairs (round 5): one wave per page; a leaf's valid entries
// (value != 0, f == r: the entries a get can find, Tree.cpp:687-697) each
// add (fingerprint, slot | leaf << 6) to the entry of their key's prefix,
// leaf = the page's place in that entry's leaf list.  A key in a leaf the
// list does not name marks the entry unusable (kDirPairsBad); more than
// kDirPairMax keys leave it unusable as well (the count says so).  A get
// reads the directory entry and then only the slots whose pair matches its
// fingerprint: 16 B of candidates for the ~4-9 keys of a prefix instead of
// the fingerprints of every slot of its leaf (fewer false candidates), and
// prefixes that span up to four leaves are answered the same way.
__global__ __launch_bounds__(256) void k_dir_pairs(const uint8_t* __restrict__ arena,
                                                   uint64_t n_pages, uint16_t node,
                                                   uint64_t dir_lo, uint32_t shift,
                                                   uint64_t n_ent, uint64_t* __restrict__ dir) {
  const int lane = lane_id();
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / kWave);
  for (uint64_t pi = 1 + (uint64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
       pi < n_pages; pi += nw) {
    const uint8_t* pg = arena + (pi << 10);
    if (pg[kOffLevel] != 0 || pg64_b1(pg, 2) != 0) continue;  // a leaf (no leftmost)
    if (lane >= kLeafCardinality) continue;
    uint64_t k, v;
    uint32_t f, r;
    lane_entry(pg, lane, k, v, f, r);
    if (v == kValueNull || ((f ^ r) & 0xF) != 0) continue;
    if (k < dir_lo || ((k - dir_lo) >> shift) >= n_ent) continue;
    uint32_t* w = reinterpret_cast<uint32_t*>(dir + kDirWords * ((k - dir_lo) >> shift));
    const uint32_t cw = w[7];
    if (!(cw & kDirPairs)) continue;
    const uint32_t n = cw & 0xFFu;
    const uint32_t me = (uint32_t)pi;
    uint32_t j = 4;
    for (uint32_t x = 0; x < n && x < 4; ++x)
      if (w[x] == me) j = x;
    if (j == 4) {
      atomicOr(w + 7, kDirPairsBad);
      continue;
    }
    const uint32_t pos = (atomicAdd(w + 7, 1u << 16) >> 16) & 0xFFu;
    if (pos < kDirPairMax)
      reinterpret_cast<uint16_t*>(w + 8)[pos] =
          (uint16_t)(key_fp(k) | (((uint32_t)lane | (j << 6)) << 8));
  }
}

void launch_dir_pairs(const uint8_t* arena, uint64_t n_pages, uint16_t node, uint64_t dir_lo,
                      uint32_t shift, uint64_t n_ent, uint64_t* dir, hipStream_t s) {
  if (n_pages <= 1 || !n_ent) return;
  hipLaunchKernelGGL(k_dir_pairs, dim3(2048), dim3(256), 0, s, arena, n_pages, node, dir_lo,
                     shift, n_ent, dir);
}

// The exact entry of prefix p as a build would write it (one wave): word
// `lane` of the 64 B entry in *v for lanes < 16; false when the walk failed
// (a bad pointer).  In the pair form *np_out = the pair count.
__device__ __forceinline__ bool dir_exact_entry(const uint8_t* __restrict__ arena,
                                                uint64_t arena_bytes, uint16_t node, uint64_t root,
                                                uint64_t dir_lo, uint32_t shift, uint64_t p,
                                                const uint32_t* __restrict__ hint, int form,
                                                uint32_t* v_out, uint32_t* np_out,
                                                bool prefix_fps = false) {
  const int lane = lane_id();
  const uint64_t span = (1ull << shift) - 1;
  const uint32_t sh = shift > 32 ? shift - 32 : 0;
  const uint64_t lo = dir_lo + (p << shift);
  const uint64_t hi = lo > ~0ull - span ? ~0ull : lo + span;
  // the leaf holding lo, the leaves covering [lo, hi] (k_leaf_dir's walk),
  // one dependent round per page: the whole page in one 16 B slice per lane
  // (header and every internal record, load_page_slice), the child by a
  // ballot over the records
  uint64_t pgs[4] = {0, 0, 0, 0}, seps[4] = {0, 0, 0, 0};
  uint32_t n = 0;
  uint64_t cover = root;
  bool ok = false;
  {
    uint64_t ptr = root;
    bool hinted = false;
    if (hint && hint[p]) {
      ptr = dir_page_ga(hint[p], node);
      hinted = true;
    }
    for (int it = 0; it < 4096; ++it) {  // (wave-uniform)
      if (!ptr_ok(ptr, node, arena_bytes)) break;
      const u32x4 w = load_page_slice(arena, ga_offset(ptr));
      const Hdr h = parse_hdr(w);
      if (hinted && (h.leftmost == 0 || h.level != 1 || lo < h.lowest)) {
        hinted = false;  // not a level-1 page on lo's path any more
        ptr = root;
        continue;
      }
      if (lo >= h.highest) {  // turn right (Tree.cpp:626-629)
        if (h.sibling == 0) break;
        ptr = h.sibling;
        continue;
      }
      if (h.leftmost != 0) {  // internal: the child of #keys <= lo (Tree.cpp:665-685)
        const IntRec r = internal_record(w);
        const int j = lane - 3;
        const int cnt = h.last_index + 1;
        const uint64_t le = ballot(j >= 0 && j < cnt && j < kInternalCardinality && r.key <= lo);
        const int c = popc64(le);
        if (hi < h.highest) cover = ptr;
        ptr = c == 0 ? h.leftmost : rl64(r.ptr, 3 + c - 1);
        hinted = false;
        continue;
      }
      pgs[0] = ptr;
      uint64_t hh = h.highest, sib = h.sibling;
      n = 1;
      while (hh <= hi && sib != 0 && n <= 4) {
        if (n == 4 || !ptr_ok(sib, node, arena_bytes)) {
          n = 5;  // more than four leaves: the covering internal page
          break;
        }
        const Hdr hs = parse_hdr(load_page_slice(arena, ga_offset(sib)));
        pgs[n] = sib;
        seps[n] = hs.lowest;
        hh = hs.highest;
        sib = hs.sibling;
        ++n;
      }
      ok = true;
      break;
    }
  }
  *np_out = 0;
  if (!ok) return false;
  uint32_t v = 0;  // word `lane` of the entry (lanes < 16)
  if (n > 4) {
    if (lane == 0) v = dir_page_index(cover);  // count 0: start at the covering page
  } else if (form == kDirFormFp && n == 1) {
    // the leaf's fingerprints (valid slots; 0 for empty ones)
    const uint8_t* pg = arena + ga_offset(pgs[0]);
    uint64_t k = 0, val = 0;
    uint32_t f = 0, r = 0;
    if (lane < kLeafCardinality) lane_entry(pg, lane, k, val, f, r);
    // (prefix_fps: only the slots whose keys lie in the prefix -- what a
    // get or a locate of a key of this prefix relies on; the copy of the
    // leaf's other slots only adds candidates)
    const bool in = !prefix_fps || (k >= lo && k <= hi);
    const uint32_t fp = lane < kLeafCardinality && val != kValueNull && in ? key_fp(k) : 0u;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int byte = 4 * (lane & 15) + b;
      const int s = byte >= 4 && byte < 28 ? byte - 4 : byte >= 32 && byte < 62 ? byte - 8 : -1;
      const uint32_t x = shfl32(fp, s >= 0 ? s : 0);
      if (s >= 0) v |= (x & 0xFFu) << (8 * b);
    }
    if (lane == 0) v = dir_page_index(pgs[0]);
    if (lane == 7) v = 1u | kDirFp;
  } else {
    // the leaf list and its split points (words 0..7)
    const uint32_t t1 = n > 1 ? (uint32_t)((seps[1] - lo) >> sh) : 0u;
    const uint32_t t2 = n > 2 ? (uint32_t)((seps[2] - lo) >> sh) : 0u;
    const uint32_t t3 = n > 3 ? (uint32_t)((seps[3] - lo) >> sh) : 0u;
    if (lane < 4)
      v = (uint32_t)lane < n
              ? dir_page_index(lane == 0 ? pgs[0] : lane == 1 ? pgs[1] : lane == 2 ? pgs[2] : pgs[3])
              : 0u;
    if (lane == 4) v = t1;
    if (lane == 5) v = t2;
    if (lane == 6) v = t3;
    uint32_t cw = n;
    if (form == kDirFormPairs) {
      // the pairs: leaf j's valid entries inside [lo, hi], leaf then slot order
      uint32_t np = 0;
      uint32_t pos[4] = {~0u, ~0u, ~0u, ~0u};  // this lane's (slot's) pair position in leaf j
      uint32_t pr[4] = {0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if ((uint32_t)j >= n) break;
        const uint8_t* pg = arena + ga_offset(pgs[j]);
        uint64_t k = 0, val = 0;
        uint32_t f = 0, r = 0;
        if (lane < kLeafCardinality) lane_entry(pg, lane, k, val, f, r);
        const bool in = lane < kLeafCardinality && val != kValueNull && ((f ^ r) & 0xF) == 0 &&
                        k >= lo && k <= hi;
        const uint64_t b = ballot(in);
        if (in) {
          pos[j] = np + (uint32_t)popc64(b & lanemask_lt());
          pr[j] = key_fp(k) | (((uint32_t)lane | ((uint32_t)j << 6)) << 8);
        }
        np += (uint32_t)popc64(b);
      }
      // pair q (q < 16) to lane 8 + q / 2, half q & 1 (positions are dense:
      // pair q is held by the lane whose pos[j] == q)
      uint32_t lo16 = 0, hi16 = 0;
      for (uint32_t q = 0; q < np && q < kDirPairMax; ++q) {
        uint32_t got = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint64_t b = ballot(pos[j] == q);
          if (b) got = shfl32(pr[j], ctz64(b));
        }
        if (lane == 8 + (int)(q >> 1)) {
          if (q & 1u)
            hi16 = got;
          else
            lo16 = got;
        }
      }
      if (lane >= 8 && lane < 16) v = (lo16 & 0xFFFFu) | ((hi16 & 0xFFFFu) << 16);
      cw |= kDirPairs | ((np < 255u ? np : 255u) << 16);
      *np_out = np;
    }
    if (lane == 7) v = cw;
  }
  *v_out = v;
  return true;
}

// The entries an insert chunk's writers could not keep exact (dir_upkeep.h:
// prefixes a split page shares with a neighbour, a new key whose prefix's
// list does not name its leaf) were marked for the summary walk and listed;
// after the chunk, one wave per listed prefix rebuilds its entry from the
// tree exactly as k_leaf_dir (+ k_dir_pairs) would (dir_exact_entry): the
// leaf holding the prefix's first key (walked from the prefix's level-1
// hint, a B-link start that stays valid), the up to four leaves covering
// the prefix, and in the pair form the (fingerprint, slot | leaf << 6) pairs
// of their valid entries inside the prefix, in leaf then slot order; in the
// fingerprint form an entry whose prefix lies in one leaf carries that
// leaf's fingerprints.  fix_n[par] holds the chunk's count (past cap: lost
// repairs, added to *lost in host memory, which the host reads as
// staleness); the launch zeroes the next chunk's counter.
__global__ __launch_bounds__(256) void k_dir_repair(const uint8_t* __restrict__ arena,
                                                    uint64_t arena_bytes, uint16_t node,
                                                    uint64_t root, uint64_t dir_lo, uint32_t shift,
                                                    uint64_t n_ent, uint64_t* __restrict__ dir,
                                                    const uint32_t* __restrict__ hint, int form,
                                                    const uint32_t* __restrict__ fix,
                                                    uint32_t* fix_n, uint32_t par, uint32_t cap,
                                                    uint64_t* lost, uint32_t* err) {
  const int lane = lane_id();
  const uint32_t n_fix = fix_n[par];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    fix_n[par ^ 1u] = 0;  // the next chunk's list (its writers run after this launch)
    if (lost) {
      if (n_fix > cap) {
        const uint64_t l = __hip_atomic_load(lost, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(lost, l + (n_fix - cap), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      // the upkeep's work so far and the count of upkeeps done, for the
      // host's idle rule (tree.cpp insert_apply); k_dir_upkeep finished
      uint64_t* ctr = reinterpret_cast<uint64_t*>(fix_n + kDirWorkWord);
      const uint64_t done = ctr[1] + 1;
      ctr[1] = done;
      __hip_atomic_store(lost + 1, ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(lost + 2, done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  const uint32_t m = n_fix < cap ? n_fix : cap;
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / kWave);
  for (uint64_t wi = (uint64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave); wi < m;
       wi += nw) {
    const uint64_t p = fix[wi];
    if (p >= n_ent) continue;
    uint32_t* w = reinterpret_cast<uint32_t*>(dir + kDirWords * p);
    uint32_t v = 0, np = 0;
    if (!dir_exact_entry(arena, arena_bytes, node, root, dir_lo, shift, p, hint, form, &v, &np)) {
      if (lane == 0) {  // left to the summary walk from the root; reported
        atomicOr(err, kErrBadPtr);
        w[0] = dir_page_index(root);
        w[7] = 0u;
      }
      continue;
    }
    if (lane < 16) w[lane] = v;
  }
}

// The chunk's directory upkeep, after its k_upper (round 6; dir_upkeep.h):
// one wave per staged segment of the chunk (the leaves that got a new key).
// A segment applied in place: each new key's pair / fingerprint goes into
// its prefix's entry (dir_note_new), its slot found in the page.  A split
// segment: its P pages, from page 0 (the segment's page, or the root's left
// half when the root grew) along the sibling chain, each rewrites the
// entries inside its fences and lists the ones it shares
// (dir_note_split_page).  Off the upsert's and k_upper's dependent chains:
// the tree is final when this runs, and k_dir_repair follows it.
__global__ __launch_bounds__(256) void k_dir_upkeep(UpperArgs u, const uint32_t* __restrict__ oslot,
                                                    const uint64_t* __restrict__ pages,
                                                    const uint64_t* __restrict__ n_ops_dev) {
  const int lane = lane_id();
  const uint64_t n_ops = *n_ops_dev;
  const uint32_t ns = *u.ns_dev;
  const uint64_t nwin = ((n_ops > ns ? n_ops : (uint64_t)ns) + kWave - 1) / kWave;
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / kWave);
  uint64_t work = 0;  // new keys + split pages this wave handled
  for (uint64_t win = (uint64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
       win < nwin; win += nw) {
    // (a) the new keys the upsert stored in place, lane = op
    const uint64_t i = win * kWave + (uint64_t)lane;
    bool placed = false;
    if (i < n_ops) {
      const uint32_t o = oslot[i];
      placed = (o & kOpPlaced) && !(o >> 31);
      if (placed)
        dir_note_new(u, u.op_key[i], (uint32_t)(ga_offset(pages[i]) >> 10), (int)(o & 63u));
    }
    work += (uint64_t)__popcll(ballot(placed));
    // (b) the split segments of this window, one after another
    const uint64_t g = win * kWave + (uint64_t)lane;
    const bool split = g < ns && u.seg_T[g] != 0 && u.seg_P[g] > 1;
    uint64_t m = ballot(split);
    while (m) {
      const int l = ctz64(m);
      m &= m - 1;
      const uint64_t gs = rl64(g, l);
      const uint32_t P = u.seg_P[gs];
      uint64_t page = u.seg_page[gs];
      if (!ptr_ok(page, u.node, u.arena_bytes)) continue;
      // page 0 is the segment's page, unless that page became the root's
      // internal page (the root grew: its left half is the leftmost)
      {
        const Hdr h = parse_hdr(load_page_slice(u.arena, ga_offset(page)));
        if (h.leftmost != 0) page = h.leftmost;
      }
      for (uint32_t q = 0; q < P && ptr_ok(page, u.node, u.arena_bytes); ++q) {
        const uint8_t* pg = u.arena + ga_offset(page);
        const Hdr h = parse_hdr(load_page_slice(u.arena, ga_offset(page)));
        if (h.leftmost != 0) break;  // not a leaf
        const uint32_t c = (uint32_t)(h.last_index + 1);
        uint64_t k = 0, v = 0;
        uint32_t f = 0, r = 0;
        if ((uint32_t)lane < c && lane < kLeafCardinality) lane_entry(pg, lane, k, v, f, r);
        dir_note_split_page(u, (uint32_t)(ga_offset(page) >> 10), h.lowest, h.highest, k,
                            c < (uint32_t)kLeafCardinality ? c : (uint32_t)kLeafCardinality);
        page = h.sibling;
        ++work;
      }
    }
  }
  if (work && lane == 0)
    atomicAdd(reinterpret_cast<unsigned long long*>(u.dir_fix_n + kDirWorkWord),
              (unsigned long long)work);
}

void launch_dir_upkeep(const UpperArgs& u, const uint32_t* oslot, const uint64_t* pages,
                       const uint64_t* n_ops_dev, uint64_t n_max, hipStream_t s) {
  if (!n_max) return;
  static unsigned nb = 0;
  if (!nb) {
    int cus = 0, dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    nb = (unsigned)(cus > 0 ? cus : 256) * 5;  // every resident wave slot at 5 per SIMD
  }
  const uint64_t need = (n_max + 4 * kWave - 1) / (4 * kWave);  // a 64-op window per wave
  hipLaunchKernelGGL(k_dir_upkeep, dim3((unsigned)(need < nb ? need : nb)), dim3(256), 0, s, u,
                     oslot, pages, n_ops_dev);
}

// Diagnostics (shm__dir_verify): every entry the walks trust -- a usable
// pair-form entry, a fingerprint-form entry -- against the exact entry of
// the tree as it is: out[0] entries checked, out[1] leaf lists or split
// points that differ, out[2] pair sets that differ, out[3] fingerprint
// copies that miss a valid slot's fingerprint, out[4..7] the first bad
// prefixes (+ 1; 0 = none)
__global__ __launch_bounds__(256) void k_dir_verify(const uint8_t* __restrict__ arena,
                                                    uint64_t arena_bytes, uint16_t node,
                                                    uint64_t root, uint64_t dir_lo, uint32_t shift,
                                                    uint64_t n_ent, const uint64_t* __restrict__ dir,
                                                    const uint32_t* __restrict__ hint,
                                                    unsigned long long* out) {
  const int lane = lane_id();
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / kWave);
  for (uint64_t p = (uint64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave); p < n_ent;
       p += nw) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(dir + kDirWords * p);
    const uint32_t cw = w[7];
    const uint32_t npst = (cw >> 16) & 0xFFu;
    const bool pairs = (cw & kDirPairs) && !(cw & kDirPairsBad) && npst <= kDirPairMax;
    const bool fp = (cw & kDirFp) != 0;
    if (!pairs && !fp) continue;
    uint32_t v = 0, np = 0;
    const int form = pairs ? kDirFormPairs : kDirFormFp;
    if (!dir_exact_entry(arena, arena_bytes, node, root, dir_lo, shift, p, hint, form, &v, &np,
                         true))
      continue;
    const uint32_t st = lane < 16 ? w[lane] : 0u;
    bool bad_list = false, bad_pairs = false, bad_fp = false;
    if (pairs) {
      const uint32_t vcw = rl32(v, 7);
      // leaf count, pages and split points
      const uint32_t nl = vcw & 0xFFu;
      const bool used = (lane < 4 && (uint32_t)lane < nl) || (lane >= 4 && lane < 7 && (uint32_t)(lane - 3) < nl);
      bad_list = ballot(used && st != v) != 0 || nl != (cw & 0xFFu) || (vcw & kDirPairs) == 0;
      // pair sets: every exact pair stored, same count
      const uint32_t want = (uint32_t)((vcw >> 16) & 0xFFu);
      bool miss = false;
      if (want <= kDirPairMax) {
        for (uint32_t q = 0; q < want; ++q) {
          const uint32_t ex = (rl32(v, 8 + (int)(q >> 1)) >> (16 * (q & 1u))) & 0xFFFFu;
          bool found = false;
          for (uint32_t x = 0; x < npst; ++x)
            if (((rl32(st, 8 + (int)(x >> 1)) >> (16 * (x & 1u))) & 0xFFFFu) == ex) found = true;
          miss = miss || !found;
        }
      }
      // (extra stored pairs -- deleted keys' -- only cost a read; a missing
      // one would hide a key)
      bad_pairs = miss || want > kDirPairMax;
    } else {
      // the stored fingerprint copy must hold the fingerprint of every valid
      // slot whose key lies in the prefix, and name the exact leaf
      const bool one = (rl32(v, 7) & kDirFp) != 0;
      bad_list = !one || rl32(v, 0) != rl32(st, 0);
      if (one) {
        // compare the fingerprint words, masking slots the exact copy has 0
        const uint32_t ex = lane >= 1 && lane < 16 && lane != 7 ? v : 0u;
        const uint32_t sv = lane >= 1 && lane < 16 && lane != 7 ? st : 0u;
        uint32_t mask = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if ((ex >> (8 * b)) & 0xFFu) mask |= 0xFFu << (8 * b);
        bad_fp = ballot((ex & mask) != (sv & mask)) != 0;
      }
    }
    if (lane == 0) {
      atomicAdd(out + 0, 1ull);
      if (bad_list) atomicAdd(out + 1, 1ull);
      if (bad_pairs) atomicAdd(out + 2, 1ull);
      if (bad_fp) atomicAdd(out + 3, 1ull);
      if (bad_list || bad_pairs || bad_fp)
        for (int i = 0; i < 4; ++i)
          if (atomicCAS(out + 4 + i, 0ull, (unsigned long long)p + 1) == 0ull) break;
    }
  }
}

void launch_dir_verify(const uint8_t* arena, uint64_t arena_bytes, uint16_t node, uint64_t root,
                       uint64_t dir_lo, uint32_t shift, uint64_t n_ent, const uint64_t* dir,
                       const uint32_t* hint, unsigned long long* out, hipStream_t s) {
  hipLaunchKernelGGL(k_dir_verify, dim3(2048), dim3(256), 0, s, arena, arena_bytes, node, root,
                     dir_lo, shift, n_ent, dir, hint, out);
}

void launch_dir_repair(const uint8_t* arena, uint64_t arena_bytes, uint16_t node, uint64_t root,
                       uint64_t dir_lo, uint32_t shift, uint64_t n_ent, uint64_t* dir,
                       const uint32_t* hint, int form, const uint32_t* fix, uint32_t* fix_n,
                       uint32_t par, uint32_t cap, uint64_t* lost, uint32_t* err, hipStream_t s) {
  static unsigned nb = 0;
  if (!nb) {
    int cus = 0, dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    nb = (unsigned)(cus > 0 ? cus : 256) * 5;  // every resident wave slot at 5 per SIMD
  }
  hipLaunchKernelGGL(k_dir_repair, dim3(nb), dim3(256), 0, s, arena, arena_bytes, node, root,
                     dir_lo, shift, n_ent, dir, hint, form, fix, fix_n, par, cap, lost, err);
}

}  // namespace dev
}  // namespace shm
