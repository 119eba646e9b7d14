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

}  // namespace dev
}  // namespace shm
