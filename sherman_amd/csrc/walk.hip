// walk.hip — batched B-link tree walk (Tree::search, and the leaf/parent
// locate step of Tree::insert).
//
// Restates src/Tree.cpp:405-459 (search), 593-663 (page_search),
// 665-685 (internal_page_search) and 687-697 (leaf_page_search) for a batch.
// One wave64 owns 64 queries (one per lane).  Each round the wave lists the
// distinct pages its unfinished queries wait on, streams them through a
// per-wave ring of kRing 1 KB LDS slots with one global_load_lds_dwordx4 per
// page (LDS-DMA: the page never occupies VGPRs; kRing pages in flight per
// wave), and resolves every waiting query against the staged page:
//   * fences first (k >= highest -> sibling, the B-link "turn right",
//     Tree.cpp:626-629 / 648-651), page versions (front == rear, else re-read,
//     Tree.cpp:616-618);
//   * internal page: child = #keys <= k (Tree.cpp:665-685).  A page shared by
//     few queries uses the lane-parallel compare + ballot per query; a page
//     shared by many (the upper levels of a sorted batch) lets every query
//     lane run a fixed 6-step branchless search over the staged keys, which
//     costs the same instructions for 64 queries as for one;
//   * leaf page: lane i holds entry i; slot = ffs(ballot(key_i == k &&
//     value_i != 0 && f_i == r_i)) (Tree.cpp:687-697), once per distinct key.
// Queries that share a page (the batch is bucketed by key first) share one
// page read.
#include "device_common.h"
#include "kernels.h"

// m0 is set by the LDS-DMA asm below; nothing else in these kernels uses it
#pragma clang diagnostic ignored "-Winline-asm"

namespace shm {
namespace dev {

namespace {

constexpr int kRing = 4;           // LDS page slots per wave
constexpr int kBallotQueries = 2;  // <= this many queries: ballot per query

// One page -> one LDS slot: global_load_lds_dwordx4, lane l's 16 bytes land
// at slot + 16 l.  Issued from inline asm on purpose: hipcc treats a visible
// LDS-DMA as a pending LDS write and puts s_waitcnt vmcnt(0) in front of every
// later ds_read, which would drain the whole ring; the ring's waits are
// counted by hand instead (wait_vm below).
__device__ __forceinline__ void glds16(const uint8_t* gsrc, uint32_t* lds) {
  const uint64_t ga = (uint64_t)(gsrc + 16 * lane_id());
  const uint32_t la = (uint32_t)__builtin_amdgcn_readfirstlane(
      (int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds);
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "global_load_lds_dwordx4 %0, off"
      :
      : "v"(ga), "s"(la)
      : "memory", "m0");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// header (Tree.h:130-160) + versions from a staged page
__device__ __forceinline__ Hdr lds_hdr(const uint32_t* lp) {
  const int l = lane_id();
  const uint32_t v = l < 11 ? lp[l] : (l == 11 ? lp[254] : lp[255]);
  const uint32_t a2 = rl32(v, 2), a3 = rl32(v, 3);
  const uint32_t b0 = rl32(v, 4), b1 = rl32(v, 5), b2 = rl32(v, 6), b3 = rl32(v, 7);
  const uint32_t c0 = rl32(v, 8), c1 = rl32(v, 9), c2 = rl32(v, 10);
  const uint32_t z2 = rl32(v, 11), z3 = rl32(v, 12);
  Hdr h;
  h.fver = a2 & 0xFF;
  h.leftmost = (uint64_t)((a2 >> 8) | (a3 << 24)) |
               ((uint64_t)((a3 >> 8) | (b0 << 24)) << 32);
  h.sibling = (uint64_t)((b0 >> 8) | (b1 << 24)) |
              ((uint64_t)((b1 >> 8) | (b2 << 24)) << 32);
  h.level = (b2 >> 8) & 0xFF;
  h.last_index = (int32_t)(int16_t)(b2 >> 16);
  h.lowest = (uint64_t)b3 | ((uint64_t)c0 << 32);
  h.highest = (uint64_t)c1 | ((uint64_t)c2 << 32);
  h.rver_internal = z3 & 0xFF;
  h.rver_leaf = z2 & 0xFF;
  return h;
}

// internal record j (key at byte 44+16j = dword 11+4j)
__device__ __forceinline__ uint64_t lds_ikey(const uint32_t* lp, int j) {
  return (uint64_t)lp[11 + 4 * j] | ((uint64_t)lp[12 + 4 * j] << 32);
}
__device__ __forceinline__ uint64_t lds_iptr(const uint32_t* lp, int j) {
  return (uint64_t)lp[13 + 4 * j] | ((uint64_t)lp[14 + 4 * j] << 32);
}

}  // namespace

template <bool LOCATE>
__global__ __launch_bounds__(kBlock) void k_walk(WalkArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t s_ring[kWavesPerBlock][kRing][kPageDwords];
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  const uint64_t n = a.n_dev ? *a.n_dev : a.n;
  const uint64_t wave_base =
      ((uint64_t)blockIdx.x * kWavesPerBlock + (uint64_t)wv) * kWave;
  if (wave_base >= n) return;  // wave-uniform
  const uint64_t i = wave_base + (uint64_t)lane;
  const bool active = i < n;
  const uint64_t k = active ? a.keys[i] : 0;
  uint64_t ptr = a.root;
  bool done = !active;
  uint64_t val = 0, page_out = 0;
  bool fnd = false;
  // kKeyMax can never be stored (root highest is exclusive, Tree.h:150)
  if (!LOCATE && k == kKeyMax) done = true;
  uint32_t* ring = &s_ring[wv][0][0];
  uint32_t err = 0;
  int rounds = 0, retries = 0;

  for (;;) {
    const uint64_t pend = ballot(!done);
    if (pend == 0) break;
    if (++rounds > kMaxRounds) {
      err |= kErrRounds;
      break;
    }
    // ---- distinct pages of this round: lane j holds the j-th -------------
    uint64_t plist = 0;
    int m = 0;
    for (uint64_t rem = pend; rem;) {
      const uint64_t p = rl64(ptr, ctz64(rem));
      rem &= ~ballot(!done && ptr == p);
      if (lane == m) plist = p;
      ++m;
    }
    // invalid pointers load the superblock (always mapped) and are rejected
    // when processed, so every slot sees exactly one DMA
    const bool pbad = lane < m && !ptr_ok(plist, a.node, a.arena_bytes);
    const uint64_t pload = pbad ? 0 : plist;
    const int pre = m < kRing ? m : kRing;
    for (int j = 0; j < pre; ++j)
      glds16(a.arena + ga_offset(rl64(pload, j)), ring + j * kPageDwords);

    for (int j = 0; j < m; ++j) {
      if (j + kRing <= m)
        wait_vm<kRing - 1>();
      else
        wait_vm<0>();
      const uint32_t* lp = ring + (j % kRing) * kPageDwords;
      const uint64_t pj = rl64(plist, j);
      uint64_t qm = ballot(!done && ptr == pj);
      if (!ptr_ok(pj, a.node, a.arena_bytes)) {
        if (ptr == pj) done = true;
        err |= kErrBadPtr;
      } else if (qm) {
        const Hdr h = lds_hdr(lp);
        const bool is_leaf = h.leftmost == 0;
        const uint32_t rv = is_leaf ? h.rver_leaf : h.rver_internal;
        const bool mine = !done && ptr == pj;
        if (h.fver != rv) {
          // torn / in-flight page: the queries re-list it next round
          if (++retries > kMaxRetries) {
            if (mine) done = true;
            err |= kErrInconsistent;
          }
        } else if (LOCATE && (int)h.level == a.target_level) {
          if (mine) {
            if (k >= h.highest) {
              ptr = h.sibling;
              if (ptr == 0) done = true;
            } else if (k < h.lowest) {
              done = true;
              err |= kErrFence;
            } else {
              page_out = pj;
              done = true;
            }
          }
        } else if (!is_leaf) {
          const int cnt = h.last_index + 1;
          if (LOCATE && (int)h.level < a.target_level) {
            if (mine) done = true;
            err |= kErrFence;
          } else if (popc64(qm) <= kBallotQueries) {
            // lane-parallel compare, ballot child select per query
            const int jr = lane - 3;
            const bool valid = jr >= 0 && jr < cnt;
            const uint64_t rk = valid ? lds_ikey(lp, jr) : 0;
            while (qm) {
              const int q = ctz64(qm);
              qm &= qm - 1;
              const uint64_t kq = rl64(k, q);
              uint64_t np;
              bool bad = false;
              if (kq >= h.highest) {
                np = h.sibling;
              } else if (kq < h.lowest) {
                np = a.root;  // stale route: restart (Tree.cpp:652-657)
                bad = true;
              } else {
                const int c = popc64(ballot(valid && rk <= kq));
                np = c == 0 ? h.leftmost : lds_iptr(lp, c - 1);
              }
              if (lane == q) {
                ptr = np;
                if (np == 0) done = true;
                if (bad) err |= kErrFence;
              }
            }
          } else if (mine) {
            // many queries: each lane runs a branchless 6-step search
            if (k >= h.highest) {
              ptr = h.sibling;
              if (ptr == 0) done = true;
            } else if (k < h.lowest) {
              ptr = a.root;
              err |= kErrFence;
            } else {
              int pos = 0;  // number of keys <= k
#pragma unroll
              for (int step = 32; step > 0; step >>= 1) {
                const int idx = pos + step - 1;
                if (idx < cnt && lds_ikey(lp, idx) <= k) pos += step;
              }
              ptr = pos == 0 ? h.leftmost : lds_iptr(lp, pos - 1);
              if (ptr == 0) done = true;
            }
          }
        } else {
          // leaf (level 0): lane i holds entry i
          const LeafEnt e = leaf_entry(lp, lane < kLeafCardinality ? lane : 0);
          const bool ok = lane < kLeafCardinality && e.val != kValueNull &&
                          (e.fraw & 0xF) == (e.rraw & 0xF);
          while (qm) {
            const uint64_t kq = rl64(k, ctz64(qm));
            const uint64_t same = ballot(!done && ptr == pj && k == kq);
            qm &= ~same;
            const bool me = (same >> lane) & 1;
            if (kq >= h.highest) {
              if (me) {
                ptr = h.sibling;
                if (ptr == 0) done = true;
              }
            } else if (kq < h.lowest) {
              if (me) {
                done = true;
                err |= kErrFence;
              }
            } else if (LOCATE) {
              if (me) {  // reached a leaf below the target level
                done = true;
                err |= kErrFence;
              }
            } else {
              const uint64_t mm = ballot(ok && e.key == kq);
              uint64_t v = 0;
              if (mm) v = rl64(e.val, ctz64(mm));
              if (me) {
                done = true;
                if (mm) {
                  val = v;
                  fnd = true;
                }
              }
            }
          }
        }
      }
      // the slot's LDS reads are complete before its next DMA lands
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (j + kRing < m)
        glds16(a.arena + ga_offset(rl64(pload, j + kRing)),
               ring + (j % kRing) * kPageDwords);
    }
  }
  if (err) atomicOr(a.err, err);
  if (active) {
    const uint64_t o = a.perm ? (uint64_t)a.perm[i] : i;
    if (LOCATE) {
      a.out_page[o] = page_out;
    } else {
      a.out_val[o] = val;
      if (a.out_found) a.out_found[o] = fnd ? 1 : 0;
    }
  }
}

void launch_walk(const WalkArgs& a, uint64_t n_upper, int depth, bool locate,
                 hipStream_t s) {
  (void)depth;
  if (n_upper == 0) return;
  const uint64_t waves = (n_upper + kWave - 1) / kWave;
  const dim3 grid((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock));
  if (locate)
    hipLaunchKernelGGL((k_walk<true>), grid, dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((k_walk<false>), grid, dim3(kBlock), 0, s, a);
}

}  // namespace dev
}  // namespace shm
