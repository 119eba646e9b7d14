// device_common.h — wave64 helpers and page (de)serialisation for gfx950.
//
// A 1 KB Sherman page is moved as ONE global_load_dwordx4 per lane: lane l
// holds bytes [16l, 16l+16) in a u32x4.  Header fields come out with
// v_readlane (they live in lanes 0..2 and 63), internal records are lane
// aligned (record j = lane j+3 after a one-lane shift), and the 18-byte leaf
// entries (2-byte aligned) are staged through a per-wave 1 KB LDS slot.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.h"

namespace shm {
namespace dev {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;
constexpr int kBlock = 256;  // 4 waves per workgroup
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kPageDwords = 256;
constexpr int kMaxRounds = 4096;   // walk rounds per wave before giving up
constexpr int kMaxRetries = 1000;  // version-mismatch re-reads (Tree.cpp:600)
constexpr uint32_t kMaxLockSpins = 1u << 22;

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t rl32(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
  return (uint64_t)rl32((uint32_t)v, l) |
         ((uint64_t)rl32((uint32_t)(v >> 32), l) << 32);
}
__device__ __forceinline__ int ctz64(uint64_t m) { return __builtin_ctzll(m); }
__device__ __forceinline__ int popc64(uint64_t m) { return __popcll(m); }
__device__ __forceinline__ uint32_t shfl32(uint32_t v, int src) {
  return (uint32_t)__shfl((int)v, src);
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  return (uint64_t)shfl32((uint32_t)v, src) |
         ((uint64_t)shfl32((uint32_t)(v >> 32), src) << 32);
}
__device__ __forceinline__ uint64_t lanemask_lt() {
  const int l = lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}
// order this wave's LDS traffic (LDS executes in order per wave; this keeps
// the compiler from moving accesses across and drains the counter)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// A block's index in a decoupled look-back launch (k_bin_unique, k_seg_fill,
// k_scan_u64), taken by one atomic add as the block starts: a block waits
// only on smaller indices, which blocks already running (or done) hold, so
// the look-back cannot wait on a block the dispatcher has not placed.  With
// blockIdx it could: another kernel or another process on the card may hold
// the CUs a smaller blockIdx needs while larger ones spin (seen with two
// ranks sharing one GPU: k_bin_unique's spin bound, kErrBinSpin).  The
// launch's last taker resets the counter for the next launch of the kernel
// (launches sharing a counter are stream-ordered).  Either every block of a
// launch calls this or none does (an exit taken before it must be uniform
// over the grid); ctr == nullptr keeps blockIdx.
__device__ __forceinline__ uint32_t lookback_index(uint32_t* ctr) {
  if (!ctr) return blockIdx.x;
  __shared__ uint32_t s_idx;
  if (threadIdx.x == 0) {
    const uint32_t i = atomicAdd(ctr, 1u);
    if (i == gridDim.x - 1) atomicExch(ctr, 0u);
    s_idx = i;
  }
  __syncthreads();
  return s_idx;
}

__device__ __forceinline__ u32x4 load_page_slice(const uint8_t* arena,
                                                  uint64_t off) {
  return *reinterpret_cast<const u32x4*>(arena + off + 16 * lane_id());
}

// Header (Tree.h:130-160) + page versions, wave-uniform.
struct Hdr {
  uint64_t leftmost, sibling, lowest, highest;
  uint32_t level;
  int32_t last_index;
  uint32_t fver, rver_internal, rver_leaf;
};

__device__ __forceinline__ Hdr parse_hdr(const u32x4 w) {
  const uint32_t a2 = rl32(w.z, 0), a3 = rl32(w.w, 0);
  const uint32_t b0 = rl32(w.x, 1), b1 = rl32(w.y, 1), b2 = rl32(w.z, 1),
                 b3 = rl32(w.w, 1);
  const uint32_t c0 = rl32(w.x, 2), c1 = rl32(w.y, 2), c2 = rl32(w.z, 2);
  const uint32_t z2 = rl32(w.z, 63), z3 = rl32(w.w, 63);
  Hdr h;
  h.fver = a2 & 0xFF;  // byte 8
  h.leftmost = (uint64_t)((a2 >> 8) | (a3 << 24)) |  // bytes 9..16
               ((uint64_t)((a3 >> 8) | (b0 << 24)) << 32);
  h.sibling = (uint64_t)((b0 >> 8) | (b1 << 24)) |  // bytes 17..24
              ((uint64_t)((b1 >> 8) | (b2 << 24)) << 32);
  h.level = (b2 >> 8) & 0xFF;                   // byte 25
  h.last_index = (int32_t)(int16_t)(b2 >> 16);  // bytes 26..27
  h.lowest = (uint64_t)b3 | ((uint64_t)c0 << 32);   // bytes 28..35
  h.highest = (uint64_t)c1 | ((uint64_t)c2 << 32);  // bytes 36..43
  h.rver_internal = z3 & 0xFF;                       // byte 1020
  h.rver_leaf = z2 & 0xFF;                           // byte 1016
  return h;
}

// Internal record j = lane - 3 (Tree.h:163-172): key straddles lanes j+2/j+3.
struct IntRec {
  uint64_t key, ptr;
};
__device__ __forceinline__ IntRec internal_record(const u32x4 w) {
  const uint32_t prev_w3 = (uint32_t)__shfl_up((int)w.w, 1);
  IntRec r;
  r.key = ((uint64_t)w.x << 32) | prev_w3;
  r.ptr = (uint64_t)w.y | ((uint64_t)w.z << 32);
  return r;
}

// Leaf entry i = lane (Tree.h:174-187), read from the wave's LDS page image.
struct LeafEnt {
  uint64_t key, val;
  uint32_t fraw, rraw;  // full bytes; versions are the low nibbles
};
__device__ __forceinline__ void stage_page(uint32_t* lp, const u32x4 w) {
  *reinterpret_cast<u32x4*>(lp + 4 * lane_id()) = w;
}
__device__ __forceinline__ LeafEnt leaf_entry(const uint32_t* lp, int i) {
  const int s = kOffRecords + kLeafEntry * i;
  const int d = s >> 2;
  const uint32_t sh = (uint32_t)(s & 3);
  const uint32_t a0 = lp[d], a1 = lp[d + 1], a2 = lp[d + 2], a3 = lp[d + 3],
                 a4 = lp[d + 4];
  const uint32_t e0 = __builtin_amdgcn_alignbyte(a1, a0, sh);
  const uint32_t e1 = __builtin_amdgcn_alignbyte(a2, a1, sh);
  const uint32_t e2 = __builtin_amdgcn_alignbyte(a3, a2, sh);
  const uint32_t e3 = __builtin_amdgcn_alignbyte(a4, a3, sh);
  const uint32_t e4 = __builtin_amdgcn_alignbyte(0u, a4, sh);
  LeafEnt e;
  e.fraw = e0 & 0xFF;
  e.key = (uint64_t)((e0 >> 8) | (e1 << 24)) |
          ((uint64_t)((e1 >> 8) | (e2 << 24)) << 32);
  e.val = (uint64_t)((e2 >> 8) | (e3 << 24)) |
          ((uint64_t)((e3 >> 8) | (e4 << 24)) << 32);
  e.rraw = (e4 >> 8) & 0xFF;
  return e;
}
// write an 18 B entry at its 2-byte aligned slot: an even slot starts on a
// dword (4 dword stores + 1 halfword), an odd one 2 bytes past (1 halfword +
// 4 dword stores)
__device__ __forceinline__ void put_leaf_entry(uint32_t* lp, int i,
                                               uint64_t key, uint64_t val,
                                               uint32_t fraw, uint32_t rraw) {
  uint8_t* b = reinterpret_cast<uint8_t*>(lp) + kOffRecords + kLeafEntry * i;
  const uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
  const uint32_t v0 = (uint32_t)val, v1 = (uint32_t)(val >> 32);
  const uint32_t f = fraw & 0xFF, r = rraw & 0xFF;
  if ((i & 1) == 0) {  // f k0..k2 | k3..k6 | k7 v0..v2 | v3..v6 | v7 r
    uint32_t* d = reinterpret_cast<uint32_t*>(b);
    d[0] = f | (k0 << 8);
    d[1] = (k0 >> 24) | (k1 << 8);
    d[2] = (k1 >> 24) | (v0 << 8);
    d[3] = (v0 >> 24) | (v1 << 8);
    *reinterpret_cast<uint16_t*>(b + 16) = (uint16_t)((v1 >> 24) | (r << 8));
  } else {  // f k0 | k1..k4 | k5..k7 v0 | v1..v4 | v5..v7 r
    *reinterpret_cast<uint16_t*>(b) = (uint16_t)(f | ((k0 & 0xFF) << 8));
    uint32_t* d = reinterpret_cast<uint32_t*>(b + 2);
    d[0] = (k0 >> 8) | (k1 << 24);
    d[1] = (k1 >> 8) | (v0 << 24);
    d[2] = (v0 >> 8) | (v1 << 24);
    d[3] = (v1 >> 8) | (r << 24);
  }
}

// Header dword d (0..10) of a page image (bytes 0..43); lock word = 0.
__device__ __forceinline__ uint32_t header_dword(int d, uint32_t fver,
                                                 uint64_t leftmost,
                                                 uint64_t sibling,
                                                 uint32_t level,
                                                 int32_t last_index,
                                                 uint64_t lowest,
                                                 uint64_t highest) {
  switch (d) {
    case 2: return (fver & 0xFF) | (uint32_t)((leftmost & 0xFFFFFF) << 8);
    case 3: return (uint32_t)(leftmost >> 24);
    case 4: return (uint32_t)(leftmost >> 56) | (uint32_t)((sibling & 0xFFFFFF) << 8);
    case 5: return (uint32_t)(sibling >> 24);
    case 6:
      return (uint32_t)(sibling >> 56) | ((level & 0xFF) << 8) |
             ((uint32_t)(last_index & 0xFFFF) << 16);
    case 7: return (uint32_t)lowest;
    case 8: return (uint32_t)(lowest >> 32);
    case 9: return (uint32_t)highest;
    case 10: return (uint32_t)(highest >> 32);
    default: return 0;
  }
}

// zero the slot and write a fresh header (all lanes call)
__device__ __forceinline__ void init_page_image(uint32_t* lp, uint32_t fver,
                                                uint64_t leftmost,
                                                uint64_t sibling,
                                                uint32_t level,
                                                int32_t last_index,
                                                uint64_t lowest,
                                                uint64_t highest) {
  const int l = lane_id();
  *reinterpret_cast<u32x4*>(lp + 4 * l) = u32x4{0, 0, 0, 0};
  wave_lds_sync();
  if (l < 11)
    lp[l] = header_dword(l, fver, leftmost, sibling, level, last_index, lowest,
                         highest);
}

__device__ __forceinline__ void store_page(uint8_t* arena, uint64_t off,
                                           const uint32_t* lp) {
  wave_lds_sync();
  const u32x4 w = *reinterpret_cast<const u32x4*>(lp + 4 * lane_id());
  *reinterpret_cast<u32x4*>(arena + off + 16 * lane_id()) = w;
}

// leaf directory lookup (leafdir.hip): the start page for key k, `fallback`
// when k is outside the directory.  Entry p is 64 B (kDirWords u64), its
// first 32 B u32[8] = {pg0..pg3, t1..t3, count}: the leaves covering prefix
// p as page indices (GlobalAddress offset / 1 KB) and their split points
// t_i, the top 32 bits of (sep_i - lo_p) within the prefix (exact when the
// prefix spans <= 2^32 keys); count 0: pg0 is the deepest internal page
// covering the prefix.  count & kDirFp: ONE leaf covers the prefix and the
// entry carries a copy of its summary fingerprints (dir_fp_cand below) in
// place of pg1..pg3 / t1..t3 and in bytes 32..61.
// Leaf i is taken only when t_i < t(k), which proves k > sep_i; on a tie the
// walk starts one leaf to the left and moves right (B-link, Tree.cpp:626-629).
// k lies inside the directory's key range (and is not kKeyMax)
__device__ __forceinline__ bool dir_covers(uint64_t dir_lo, uint32_t dir_shift, uint64_t dir_n,
                                           uint64_t k) {
  return k >= dir_lo && ((k - dir_lo) >> dir_shift) < dir_n && k != kKeyMax;
}
__device__ __forceinline__ uint64_t dir_start(const uint64_t* dir, uint64_t dir_lo,
                                              uint32_t dir_shift, uint64_t dir_n,
                                              uint16_t node, uint64_t k, uint64_t fallback) {
  const uint64_t p = (k - dir_lo) >> dir_shift;
  if (k < dir_lo || p >= dir_n || k == kKeyMax) return fallback;
  const u32x4* e = reinterpret_cast<const u32x4*>(dir + kDirWords * p);
  const u32x4 e0 = e[0], e1 = e[1];
  const uint64_t off = (k - dir_lo) - (p << dir_shift);
  const bool exact = dir_shift <= 32;
  const uint32_t tk = exact ? (uint32_t)off : (uint32_t)(off >> (dir_shift - 32));
  const uint32_t cnt = e1.w & 0xFFu;
  auto past = [&](uint32_t t) { return t < tk || (exact && t == tk); };
  const uint32_t i = (uint32_t)(cnt > 1 && past(e1.x)) + (uint32_t)(cnt > 2 && past(e1.y)) +
                     (uint32_t)(cnt > 3 && past(e1.z));
  const uint32_t pg = i == 0 ? e0.x : i == 1 ? e0.y : i == 2 ? e0.z : e0.w;
  return dir_page_ga(pg, node);
}

// dir_start reading the whole 64 B entry into e (one request): *fpform when
// it is in fingerprint form (its one leaf returned, candidates by dir_fp_cand).
// alt (nullable), round 4: on a tie (k's top 32 offset bits equal leaf i's
// split point's) the leaf i itself is returned and *alt = the safe start one
// leaf to the left, else *alt = 0.  The split points are keys (each leaf's
// lowest fence), so a lookup of the first key of a leaf is exactly such a
// tie: 2.7 % of C2's gets started left and moved right (a summary and a
// header read more).  A caller that finds k in the returned leaf is done (a
// key lives in one leaf); one that does not must walk again from *alt (k may
// lie below leaf i's lowest fence, in leaf i - 1).
__device__ __forceinline__ uint64_t dir_start_e(const uint64_t* dir, uint64_t dir_lo,
                                                uint32_t dir_shift, uint64_t dir_n, uint16_t node,
                                                uint64_t k, uint64_t fallback, u32x4 (&e)[4],
                                                bool& fpform, uint64_t* alt = nullptr) {
  fpform = false;
  if (alt) *alt = 0;
  const uint64_t p = (k - dir_lo) >> dir_shift;
  if (k < dir_lo || p >= dir_n || k == kKeyMax) {
    // no entry: a zero one (count 0, no form flag), so the callers' pair /
    // fingerprint decoding of e[] sees no candidates
#pragma unroll
    for (int j = 0; j < 4; ++j) e[j] = u32x4{0u, 0u, 0u, 0u};
    return fallback;
  }
  const u32x4* ep = reinterpret_cast<const u32x4*>(dir + kDirWords * p);
#pragma unroll
  for (int j = 0; j < 4; ++j) e[j] = ep[j];
  const uint64_t off = (k - dir_lo) - (p << dir_shift);
  const bool exact = dir_shift <= 32;
  const uint32_t tk = exact ? (uint32_t)off : (uint32_t)(off >> (dir_shift - 32));
  const uint32_t cnt = e[1].w & 0xFFu;
  fpform = (e[1].w & kDirFp) != 0;
  auto past = [&](uint32_t t) { return t < tk || (exact && t == tk); };
  const uint32_t i = fpform ? 0u
                            : (uint32_t)(cnt > 1 && past(e[1].x)) +
                                  (uint32_t)(cnt > 2 && past(e[1].y)) +
                                  (uint32_t)(cnt > 3 && past(e[1].z));
  auto page_of = [&](uint32_t j) {
    return j == 0 ? e[0].x : j == 1 ? e[0].y : j == 2 ? e[0].z : e[0].w;
  };
  if (alt && !fpform && !exact && i + 1 < cnt) {
    const uint32_t tn = i == 0 ? e[1].x : i == 1 ? e[1].y : e[1].z;  // leaf i + 1's split
    if (tn == tk) {
      *alt = dir_page_ga(page_of(i), node);
      return dir_page_ga(page_of(i + 1), node);
    }
  }
  return dir_page_ga(page_of(i), node);
}

// A directory entry in fingerprint form (count == 1 | kDirFp, layout.h):
// the candidate slots of its one leaf for key k, from the copy of the leaf's
// summary fingerprints taken when the directory was built: fp[s] at bytes
// 4..27 (s < 24) and 32..61 (s >= 24) of the entry.  The copy may be stale
// (the leaf got keys or split since): a candidate is only a slot to read,
// and a get that finds no valid entry with its key there walks the summary
// path (never a wrong answer, a stale copy only costs that fallback).
__device__ __forceinline__ uint64_t dir_fp_cand(const u32x4 (&e)[4], uint64_t k) {
  const uint32_t fq = key_fp(k);
  uint64_t cand = 0;
#pragma unroll
  for (int s = 0; s < kLeafCardinality; ++s) {
    const int b = s < 24 ? 4 + s : 8 + s;  // 24 fps at 4..27, 30 at 32..61
    const u32x4 v = e[b >> 4];
    const int d = (b >> 2) & 3;
    const uint32_t x = d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
    cand |= (uint64_t)(((x >> (8 * (b & 3))) & 0xFFu) == fq) << s;
  }
  return cand;
}

// A directory entry in pair form (layout.h kDirPairs): usable when its build
// finished clean (no kDirPairsBad, at most kDirPairMax pairs); the pairs
// whose fingerprint equals k's (bit j: pair j), each naming a slot of one of
// the entry's leaves (dir_pair_slot).  Like the fingerprint form's, a
// candidate is only a slot to read (a stale pair costs the summary walk).
__device__ __forceinline__ uint32_t dir_pair_cand(const u32x4 (&e)[4], uint64_t k, bool& usable) {
  const uint32_t cw = e[1].w;
  const uint32_t np = (cw >> 16) & 0xFFu;
  usable = (cw & kDirPairs) && !(cw & kDirPairsBad) && np <= kDirPairMax;
  if (!usable) return 0;
  const uint32_t fq = key_fp(k);
  const uint32_t w[8] = {e[2].x, e[2].y, e[2].z, e[2].w, e[3].x, e[3].y, e[3].z, e[3].w};
  uint32_t cand = 0;
#pragma unroll
  for (int j = 0; j < (int)kDirPairMax; ++j) {
    const uint32_t pr = (w[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
    cand |= (uint32_t)((uint32_t)j < np && (pr & 0xFFu) == fq) << j;
  }
  return cand;
}
// pair j's leaf (page index from the entry's list) and slot
__device__ __forceinline__ void dir_pair_slot(const u32x4 (&e)[4], int j, uint32_t& pg, int& slot) {
  const uint32_t w = (j < 8 ? (j < 4 ? (j < 2 ? e[2].x : e[2].y) : (j < 6 ? e[2].z : e[2].w))
                            : (j < 12 ? (j < 10 ? e[3].x : e[3].y) : (j < 14 ? e[3].z : e[3].w)));
  const uint32_t pr = (w >> (16 * (j & 1))) & 0xFFFFu;
  const uint32_t leaf = (pr >> 14) & 3u;
  slot = (int)((pr >> 8) & 63u);
  pg = leaf == 0 ? e[0].x : leaf == 1 ? e[0].y : leaf == 2 ? e[0].z : e[0].w;
}

__device__ __forceinline__ bool ptr_ok(uint64_t ga, uint16_t node,
                                       uint64_t arena_bytes) {
  const uint64_t off = ga_offset(ga);
  return ga != 0 && ga_node(ga) == node && (off & (kPageSize - 1)) == 0 &&
         off >= kPageSize && off + kPageSize <= arena_bytes;
}

// a key's offset in the shard range [lo, lo + 2^bits), scaled to 64 bits
// (clamped outside the range): the ordering key of both passes
struct KeyRange {
  uint64_t lo;
  uint32_t bits;
};
__device__ __forceinline__ uint64_t rel_key(uint64_t k, KeyRange r) {
  if (r.bits >= 64) return k;
  if (k < r.lo) return 0;
  const uint64_t d = k - r.lo;
  return (d >> r.bits) ? ~0ull : d << (64 - r.bits);
}
__device__ __forceinline__ uint32_t coarse_of(uint64_t k, KeyRange r) {
  return (uint32_t)(rel_key(k, r) >> 56);
}
__device__ __forceinline__ uint32_t fine_of(uint64_t k, KeyRange r) {
  return (uint32_t)(rel_key(k, r) >> 48) & 0xFF;
}

// in-wave ascending bitonic sort of (key, tag) over 64 lanes; branch-free
// compare-exchange (xor shuffles with constant masks)
__device__ __forceinline__ void wave_sort64(uint64_t& key, uint32_t& tag) {
  const int l = lane_id();
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const uint64_t pk = (uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)key, j) |
                          ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(key >> 32), j) << 32);
      const uint32_t pt = (uint32_t)__shfl_xor((int)tag, j);
      // keep the smaller key iff this lane is the lower one of an ascending
      // pair or the upper one of a descending pair
      const uint32_t want_min = (uint32_t)(((l & k) == 0) == ((l & j) == 0));
      const uint32_t take = (want_min & (uint32_t)(pk < key)) |
                            ((want_min ^ 1u) & (uint32_t)(pk > key));
      key = take ? pk : key;
      tag = take ? pt : tag;
    }
  }
}

// lower_bound over a sorted global u64 array [lo, hi)
__device__ __forceinline__ uint64_t lower_bound64(const uint64_t* a,
                                                  uint64_t lo, uint64_t hi,
                                                  uint64_t k) {
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a[mid] < k)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// A leaf's summary line (layout.h) from one wave: lane s < 54 gives slot
// s's fingerprint (0 = empty), lane 0 the highest fence; the tag byte last.
__device__ __forceinline__ void put_leaf_sum(uint8_t* sum, uint64_t page_off, uint64_t highest,
                                             uint32_t fp) {
  if (!sum) return;
  uint8_t* line = sum + (page_off >> 10) * kSumBytes;
  const int lane = lane_id();
  if (lane < kLeafCardinality) line[kSumOffFp + lane] = (uint8_t)fp;
  if (lane == 0) {
    *reinterpret_cast<uint64_t*>(line + kSumOffHighest) = highest;
    line[kSumOffTag] = kSumLeaf;
  }
}
// mark a page's line as not describing a leaf
__device__ __forceinline__ void clear_leaf_sum(uint8_t* sum, uint64_t page_off) {
  if (sum) sum[(page_off >> 10) * kSumBytes + kSumOffTag] = 0;
}
// clear slot s's fingerprint (the slot became empty)
__device__ __forceinline__ void clear_leaf_fp(uint8_t* sum, uint64_t page_off, int s) {
  if (sum) sum[(page_off >> 10) * kSumBytes + kSumOffFp + s] = 0;
}
// set slot s's fingerprint (a new key took the slot)
__device__ __forceinline__ void set_leaf_fp(uint8_t* sum, uint64_t page_off, int s, uint64_t k) {
  if (sum) sum[(page_off >> 10) * kSumBytes + kSumOffFp + s] = (uint8_t)key_fp(k);
}

// ---- per-lane leaf access (the summary walk, the update matcher) --------------

// leaf entry s of a page (18 B at 44 + 18 s, 2-byte aligned)
__device__ __forceinline__ void lane_entry(const uint8_t* page, int s, uint64_t& key,
                                           uint64_t& val, uint32_t& f, uint32_t& r) {
  const uint32_t off = (uint32_t)(kOffRecords + kLeafEntry * s);
  const uint32_t* d = reinterpret_cast<const uint32_t*>(page + (off & ~3u));
  const uint32_t d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3], d4 = d[4];
  const uint32_t sh = off & 3u;  // 0 or 2
  const uint32_t q0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
  const uint32_t q1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
  const uint32_t q2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
  const uint32_t q3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
  const uint32_t q4 = d4 >> (8 * sh);
  f = q0 & 0xFF;
  key = (uint64_t)((q0 >> 8) | (q1 << 24)) | ((uint64_t)((q1 >> 8) | (q2 << 24)) << 32);
  val = (uint64_t)((q2 >> 8) | (q3 << 24)) | ((uint64_t)((q3 >> 8) | (q4 << 24)) << 32);
  r = (q4 >> 8) & 0xFF;
}

// lane_entry in two halves, so several entries (and a summary line) can be
// requested before any is decoded: the raw dwords of entry s, then its fields
struct RawEntry {
  uint32_t d[5];
  uint32_t sh;
};
__device__ __forceinline__ void entry_load(const uint8_t* page, int s, RawEntry& r) {
  const uint32_t off = (uint32_t)(kOffRecords + kLeafEntry * s);
  const uint32_t* d = reinterpret_cast<const uint32_t*>(page + (off & ~3u));
#pragma unroll
  for (int j = 0; j < 5; ++j) r.d[j] = d[j];
  r.sh = off & 3u;
}
__device__ __forceinline__ void entry_decode(const RawEntry& e, uint64_t& key, uint64_t& val,
                                             uint32_t& f, uint32_t& r) {
  const uint32_t q0 = __builtin_amdgcn_alignbyte(e.d[1], e.d[0], e.sh);
  const uint32_t q1 = __builtin_amdgcn_alignbyte(e.d[2], e.d[1], e.sh);
  const uint32_t q2 = __builtin_amdgcn_alignbyte(e.d[3], e.d[2], e.sh);
  const uint32_t q3 = __builtin_amdgcn_alignbyte(e.d[4], e.d[3], e.sh);
  const uint32_t q4 = e.d[4] >> (8 * e.sh);
  f = q0 & 0xFF;
  key = (uint64_t)((q0 >> 8) | (q1 << 24)) | ((uint64_t)((q1 >> 8) | (q2 << 24)) << 32);
  val = (uint64_t)((q2 >> 8) | (q3 << 24)) | ((uint64_t)((q3 >> 8) | (q4 << 24)) << 32);
  r = (q4 >> 8) & 0xFF;
}

__device__ __forceinline__ bool entry_hit(uint64_t key, uint64_t val, uint32_t f, uint32_t r,
                                          uint64_t k) {
  return key == k && val != kValueNull && ((f ^ r) & 0xF) == 0;
}

// A leaf's summary line read whole (one 128 B request): false if it does not
// describe a current leaf; else its highest fence, sibling and the slots
// whose 8-bit fingerprint equals k's (bit s for slot s)
struct SumLine {
  uint64_t highest, cand;
};
__device__ __forceinline__ void sum_load(const uint8_t* sum, uint64_t page_off, u32x4 (&l)[4]) {
  const u32x4* line = reinterpret_cast<const u32x4*>(sum + (page_off >> 10) * kSumBytes);
#pragma unroll
  for (int j = 0; j < 4; ++j) l[j] = line[j];
}
__device__ __forceinline__ bool sum_decode(const u32x4 (&l)[4], uint64_t k, SumLine& o) {
  if ((l[0].z & 0xFF) != kSumLeaf) return false;
  o.highest = (uint64_t)l[0].x | ((uint64_t)l[0].y << 32);
  const uint32_t fq = key_fp(k);
  uint64_t cand = 0;
#pragma unroll
  for (int s = 0; s < kLeafCardinality; ++s) {  // byte 9 + s of the line
    const int b = (int)kSumOffFp + s;
    const u32x4 v = l[b >> 4];
    const int d = (b >> 2) & 3;
    const uint32_t x = d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
    cand |= (uint64_t)(((x >> (8 * (b & 3))) & 0xFFu) == fq) << s;
  }
  o.cand = cand;
  return true;
}
__device__ __forceinline__ bool sum_read(const uint8_t* sum, uint64_t page_off, uint64_t k,
                                         SumLine& o) {
  u32x4 l[4];
  sum_load(sum, page_off, l);
  return sum_decode(l, k, o);
}
// a page's sibling pointer from its header (bytes 17..24, Tree.h:130-160):
// the right turn of a summary walk
__device__ __forceinline__ uint64_t page_sibling(const uint8_t* page) {
  const u32x4 B = *reinterpret_cast<const u32x4*>(page + 16);
  return (uint64_t)((B.x >> 8) | (B.y << 24)) | ((uint64_t)((B.y >> 8) | (B.z << 24)) << 32);
}

}  // namespace dev
}  // namespace shm
