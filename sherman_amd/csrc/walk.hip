// walk.hip — batched B-link tree walk (Tree::search, and the leaf/parent
// locate step of Tree::insert).
//
// Restates src/Tree.cpp:405-459 (search), 593-663 (page_search),
// 665-685 (internal_page_search) and 687-697 (leaf_page_search) for a batch.
//
// One wave64 owns 64 queries.  It first sorts them by key across its lanes
// (bitonic, in registers), so at every level the queries that wait on the
// same page occupy a contiguous run of lanes: the pages of a round are the run
// heads, one ballot away, with no per-page matching loop.  The round's pages
// stream through a per-wave ring of R 1 KB LDS slots, one
// global_load_lds_dwordx4 per page (LDS-DMA: pages never occupy VGPRs; R - 1
// pages stay in flight while one is resolved).  Each staged page is resolved
// with wave-uniform branches on its type (scalar, from readfirstlane of the
// header) and per-lane selects, no divergent if-blocks:
//   * fences: k >= highest -> sibling, the B-link "turn right"
//     (Tree.cpp:626-629, 648-651); front != rear -> re-read next round
//     (Tree.cpp:616-618);
//   * internal page: child = #keys <= k (Tree.cpp:665-685) by a fixed 6-step
//     branchless search over the staged keys in every lane at once;
//   * leaf page: lane i holds entry i and one ballot per distinct key gives
//     slot = ffs(key_i == k && value_i != 0 && f_i == r_i) (Tree.cpp:687-697).
// The batch arrives bucketed by key (partition.hip), so the queries of a wave
// share their internal pages and same-leaf queries share one leaf read.
#include "device_common.h"
#include "kernels.h"
#include "lds_dma.h"

namespace shm {
namespace dev {

namespace {

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// internal record j (key at byte 44+16j = dword 11+4j), j <= 60
__device__ __forceinline__ uint64_t lds_ikey(const uint32_t* lp, int j) {
  return (uint64_t)lp[11 + 4 * j] | ((uint64_t)lp[12 + 4 * j] << 32);
}
__device__ __forceinline__ uint64_t lds_iptr(const uint32_t* lp, int j) {
  return (uint64_t)lp[13 + 4 * j] | ((uint64_t)lp[14 + 4 * j] << 32);
}

}  // namespace

template <bool LOCATE, int R>
__global__ __launch_bounds__(kBlock) void k_walk(WalkArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t s_ring[kWavesPerBlock][R][kPageDwords];
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  const uint64_t n = a.n_dev ? *a.n_dev : a.n;
  const uint64_t wave_base =
      ((uint64_t)blockIdx.x * kWavesPerBlock + (uint64_t)wv) * kWave;
  if (wave_base >= n) return;  // wave-uniform
  const uint32_t nact = (uint32_t)(n - wave_base < (uint64_t)kWave ? n - wave_base : kWave);
  const uint32_t ring_lds = rfl((uint32_t)(uintptr_t)(
      (__attribute__((address_space(3))) uint32_t*)&s_ring[wv][0][0]));

  // sort this wave's queries by key; tag = lane the query came from
  uint64_t k = (uint32_t)lane < nact ? a.keys[wave_base + lane] : kKeyMax;
  uint32_t tag = (uint32_t)lane;
  wave_sort64(k, tag);
  const bool active = tag < nact;

  uint64_t ptr = (!LOCATE && a.start) ? a.start[k >> a.start_shift] : a.root;
  bool done = !active;
  uint64_t val = 0, page_out = 0;
  // kKeyMax can never be stored (root highest is exclusive, Tree.h:150)
  if (!LOCATE && k == kKeyMax) done = true;
  uint32_t err = 0;
  int rounds = 0, retries = 0;

  for (;;) {
    const uint64_t pend = ballot(!done);
    if (pend == 0) break;
    if (++rounds > kMaxRounds) {
      err |= kErrRounds;
      break;
    }
    // run heads: first lane of each run of equal page pointers
    const int pl = lane == 0 ? 0 : lane - 1;
    const uint64_t prev = shfl64(ptr, pl);
    const bool prev_pend = ((pend >> pl) & 1) != 0;
    const bool head = !done && (lane == 0 || !prev_pend || prev != ptr);
    uint64_t hq = ballot(head);  // heads still to resolve
    uint64_t hi = hq;            // heads still to load
    const int m = popc64(hq);
    // invalid pointers load the superblock (always mapped) and are rejected
    // when resolved, so every slot sees exactly one DMA
    const bool pok = ptr_ok(ptr, a.node, a.arena_bytes);
    const uint64_t badm = ballot(!pok);
    const uint64_t pload = pok ? ptr : 0;
#pragma unroll
    for (int j = 0; j < R - 1; ++j) {
      if (hi) {
        glds16(a.arena + ga_offset(rl64(pload, ctz64(hi))), ring_lds + j * kPageSize);
        hi &= hi - 1;
      }
    }

    for (int j = 0; j < m; ++j) {
      // refill the slot resolved last iteration, then wait for page j
      const bool refill = hi != 0;
      if (refill) {
        glds16(a.arena + ga_offset(rl64(pload, ctz64(hi))),
               ring_lds + ((j + R - 1) % R) * kPageSize);
        hi &= hi - 1;
        wait_vm<R - 1>();
      } else {
        wait_vm<0>();
      }
      const uint32_t* lp = &s_ring[wv][j % R][0];
      const int hl = ctz64(hq);
      hq &= hq - 1;
      const uint64_t pj = rl64(ptr, hl);
      const bool mine = !done && ptr == pj;
      if ((badm >> hl) & 1) {
        if (mine) done = true;
        err |= kErrBadPtr;
      } else {
        // header: uniform-address loads (one LDS broadcast each)
        const u32x4 A = *reinterpret_cast<const u32x4*>(lp);      // dwords 0..3
        const u32x4 B = *reinterpret_cast<const u32x4*>(lp + 4);  // dwords 4..7
        const u32x4 C = *reinterpret_cast<const u32x4*>(lp + 8);  // dwords 8..11
        const u32x2 Z = *reinterpret_cast<const u32x2*>(lp + 254);
        // leaf entries, read speculatively (cheap for internal pages too)
        const LeafEnt e = leaf_entry(lp, lane < kLeafCardinality ? lane : 0);
        const uint32_t az = rfl(A.z), aw = rfl(A.w), bx = rfl(B.x), bz = rfl(B.z);
        const bool is_leaf = ((az >> 8) | aw | (bx & 0xFF)) == 0;  // leftmost == 0
        const uint32_t rver = rfl(is_leaf ? Z.x : Z.y) & 0xFF;
        const uint64_t leftmost = (uint64_t)((az >> 8) | (aw << 24)) |
                                  ((uint64_t)((aw >> 8) | (bx << 24)) << 32);
        const uint64_t sibling = (uint64_t)((B.x >> 8) | (B.y << 24)) |
                                 ((uint64_t)((B.y >> 8) | (B.z << 24)) << 32);
        const uint64_t lowest = (uint64_t)B.w | ((uint64_t)C.x << 32);
        const uint64_t highest = (uint64_t)C.y | ((uint64_t)C.z << 32);
        const int level = (int)((bz >> 8) & 0xFF);
        const int cnt = (int)(int16_t)(bz >> 16) + 1;
        if ((az & 0xFF) != rver) {
          // torn / in-flight page: its queries re-list it next round
          if (++retries > kMaxRetries) {
            if (mine) done = true;
            err |= kErrInconsistent;
          }
        } else {
          const bool right = mine && k >= highest;  // turn right
          const bool low = mine && k < lowest;      // mis-routed
          const bool here = mine && !right && !low;
          if (ballot(low)) err |= kErrFence;
          if (LOCATE && level == a.target_level) {
            page_out = here ? pj : page_out;
          } else if (LOCATE && level < a.target_level) {
            if (ballot(here)) err |= kErrFence;  // below the target level
          } else if (!is_leaf) {
            // every lane runs the branchless search; `here` lanes commit
            int pos = 0;  // number of keys <= k (keys strictly increase)
#pragma unroll
            for (int step = 32; step > 0; step >>= 1) {
              const int idx = pos + step - 1;
              const int ci = idx < 60 ? idx : 60;
              if (idx < cnt && lds_ikey(lp, ci) <= k) pos += step;
            }
            const uint64_t child = pos == 0 ? leftmost : lds_iptr(lp, pos - 1);
            ptr = here ? child : ptr;
          } else if (!LOCATE) {
            // leaf (level 0): lane i holds entry i
            const bool ok = lane < kLeafCardinality && e.val != kValueNull &&
                            (e.fraw & 0xF) == (e.rraw & 0xF);
            uint64_t qm = ballot(here);
            while (qm) {  // one ballot per distinct key of the sorted run
              const uint64_t kq = rl64(k, ctz64(qm));
              const bool same = here && k == kq;
              qm &= ~ballot(same);
              const uint64_t mm = ballot(ok && e.key == kq);
              const uint64_t v = mm ? rl64(e.val, ctz64(mm)) : 0;
              val = same ? v : val;
            }
          }
          ptr = right ? sibling : ptr;
          const bool finished =
              (LOCATE && level <= a.target_level) || (!LOCATE && is_leaf);
          done = done || low || (right && sibling == 0) ||
                 (here && (finished || ptr == 0));
        }
      }
      // the slot's LDS reads are complete before its next DMA lands
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  if (err) atomicOr(a.err, err);
  if (active) {
    const uint64_t i = wave_base + tag;
    const uint64_t o = a.perm ? (uint64_t)a.perm[i] : i;
    if (LOCATE) {
      a.out_page[o] = page_out;
    } else {
      a.out_val[o] = val;
      if (a.out_found) a.out_found[o] = val != kValueNull ? 1 : 0;
    }
  }
}

namespace {
// 4-byte aligned u64 at byte offset o of a page
__device__ __forceinline__ uint64_t pg_u64(const uint8_t* pg, int o) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(pg + o);
  return (uint64_t)d[0] | ((uint64_t)d[1] << 32);
}
// u64 at byte offset 4d+1 (leftmost @9, sibling @17)
__device__ __forceinline__ uint64_t pg_u64_b1(const uint8_t* pg, int d) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(pg) + d;
  return (uint64_t)((w[0] >> 8) | (w[1] << 24)) | ((uint64_t)((w[1] >> 8) | (w[2] << 24)) << 32);
}
// internal_page_search (Tree.cpp:665-685): index of the child covering x,
// 0 = leftmost, j + 1 = records[j]
__device__ __forceinline__ int child_index(const uint8_t* pg, int cnt, uint64_t x) {
  int lo = 0, hi = cnt;  // number of keys <= x
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (pg_u64(pg, kOffRecords + kInternalEntry * mid) <= x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}
}  // namespace

__global__ __launch_bounds__(256) void k_start_table(const uint8_t* __restrict__ arena,
                                                     uint64_t arena_bytes, uint16_t node,
                                                     uint64_t root, uint32_t bits,
                                                     uint64_t* __restrict__ table,
                                                     uint32_t* err) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >> bits) return;
  const uint64_t lo = p << (64 - bits);
  const uint64_t hi = lo | (~0ull >> bits);
  uint64_t ptr = root;
  for (int it = 0; it < 256; ++it) {
    if (!ptr_ok(ptr, node, arena_bytes)) {
      atomicOr(err, kErrBadPtr);
      ptr = root;
      break;
    }
    const uint8_t* pg = arena + ga_offset(ptr);
    const uint64_t leftmost = pg_u64_b1(pg, 2);
    const uint64_t sibling = pg_u64_b1(pg, 4);
    const uint64_t highest = pg_u64(pg, kOffHighest);
    if (lo >= highest) {  // B-link turn right (Tree.cpp:626-629)
      if (sibling == 0) break;
      ptr = sibling;
      continue;
    }
    if (leftmost == 0 || hi >= highest) break;  // leaf, or prefix leaves this page
    const int cnt = (int)(int16_t)(pg[kOffLastIndex] | (pg[kOffLastIndex + 1] << 8)) + 1;
    const int c = child_index(pg, cnt, lo);
    if (child_index(pg, cnt, hi) != c) break;  // prefix spans two children
    ptr = c == 0 ? leftmost : pg_u64(pg, kOffRecords + kInternalEntry * (c - 1) + 8);
  }
  table[p] = ptr;
}

void launch_start_table(const uint8_t* arena, uint64_t arena_bytes, uint16_t node,
                        uint64_t root, uint32_t bits, uint64_t* table, uint32_t* err,
                        hipStream_t s) {
  const uint64_t n = 1ull << bits;
  hipLaunchKernelGGL(k_start_table, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     arena, arena_bytes, node, root, bits, table, err);
}

static int ring_depth() {
  static const int r = [] {
    const char* e = getenv("SHM_WALK_RING");
    const int v = e ? atoi(e) : 4;
    return (v == 2 || v == 4 || v == 6 || v == 8) ? v : 4;
  }();
  return r;
}

void launch_walk(const WalkArgs& a, uint64_t n_upper, int depth, bool locate,
                 hipStream_t s) {
  (void)depth;
  if (n_upper == 0) return;
  const uint64_t waves = (n_upper + kWave - 1) / kWave;
  const dim3 grid((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock));
  if (locate) {
    hipLaunchKernelGGL((k_walk<true, 4>), grid, dim3(kBlock), 0, s, a);
    return;
  }
  switch (ring_depth()) {
    case 2: hipLaunchKernelGGL((k_walk<false, 2>), grid, dim3(kBlock), 0, s, a); break;
    case 6: hipLaunchKernelGGL((k_walk<false, 6>), grid, dim3(kBlock), 0, s, a); break;
    case 8: hipLaunchKernelGGL((k_walk<false, 8>), grid, dim3(kBlock), 0, s, a); break;
    default: hipLaunchKernelGGL((k_walk<false, 4>), grid, dim3(kBlock), 0, s, a); break;
  }
}

}  // namespace dev
}  // namespace shm
