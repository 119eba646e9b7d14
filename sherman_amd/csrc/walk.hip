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
// stream through a per-wave ring of kRing 1 KB LDS slots, one
// global_load_lds_dwordx4 per page (LDS-DMA: pages never occupy VGPRs;
// kRing - 1 pages stay in flight while one is resolved).  Header fields are
// read with uniform-address LDS loads into (uniform) VGPRs, so fences and
// versions are checked by each query lane itself:
//   * k >= highest -> sibling, the B-link "turn right" (Tree.cpp:626-629,
//     648-651); front != rear -> re-read next round (Tree.cpp:616-618);
//   * internal page: child = #keys <= k (Tree.cpp:665-685) by a fixed 6-step
//     branchless search over the staged keys in every waiting lane at once;
//   * leaf page: lane i holds entry i and one ballot per distinct key gives
//     slot = ffs(key_i == k && value_i != 0 && f_i == r_i) (Tree.cpp:687-697).
// The batch arrives bucketed by key (partition.hip), so the queries of a wave
// share their internal pages and same-leaf queries share one leaf read.
#include "device_common.h"
#include "kernels.h"

// m0 is set by the LDS-DMA asm below; nothing else in these kernels uses it
#pragma clang diagnostic ignored "-Winline-asm"

namespace shm {
namespace dev {

namespace {

constexpr int kRing = 4;  // LDS page slots per wave

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

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Header (Tree.h:130-160) + page versions as uniform VGPR values, from three
// uniform-address 16-byte LDS loads and one 8-byte load.
struct UHdr {
  uint64_t leftmost, sibling, lowest, highest;
  uint32_t level, fver, rver;
  int32_t cnt;
};
__device__ __forceinline__ UHdr uniform_hdr(const uint32_t* lp) {
  const u32x4 a = *reinterpret_cast<const u32x4*>(lp);       // dwords 0..3
  const u32x4 b = *reinterpret_cast<const u32x4*>(lp + 4);   // dwords 4..7
  const u32x4 c = *reinterpret_cast<const u32x4*>(lp + 8);   // dwords 8..11
  const u32x2 z = *reinterpret_cast<const u32x2*>(lp + 254); // 254..255
  UHdr h;
  h.fver = a.z & 0xFF;
  h.leftmost = (uint64_t)((a.z >> 8) | (a.w << 24)) |
               ((uint64_t)((a.w >> 8) | (b.x << 24)) << 32);
  h.sibling = (uint64_t)((b.x >> 8) | (b.y << 24)) |
              ((uint64_t)((b.y >> 8) | (b.z << 24)) << 32);
  h.level = (b.z >> 8) & 0xFF;
  h.cnt = (int32_t)(int16_t)(b.z >> 16) + 1;
  h.lowest = (uint64_t)b.w | ((uint64_t)c.x << 32);
  h.highest = (uint64_t)c.y | ((uint64_t)c.z << 32);
  // rear version: byte 1016 (leaf) or 1020 (internal)
  h.rver = h.leftmost == 0 ? (z.x & 0xFF) : (z.y & 0xFF);
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
  const uint32_t nact = (uint32_t)(n - wave_base < (uint64_t)kWave ? n - wave_base : kWave);

  // sort this wave's queries by key; tag = lane the query came from
  uint64_t k = (uint32_t)lane < nact ? a.keys[wave_base + lane] : kKeyMax;
  uint32_t tag = (uint32_t)lane;
  wave_sort64(k, tag);
  const bool active = tag < nact;

  uint64_t ptr = a.root;
  bool done = !active;
  uint64_t val = 0, page_out = 0;
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
    const uint64_t pload = ptr_ok(ptr, a.node, a.arena_bytes) ? ptr : 0;
    const int pre = m < kRing ? m : kRing;
    for (int j = 0; j < pre; ++j) {
      glds16(a.arena + ga_offset(rl64(pload, ctz64(hi))), ring + j * kPageDwords);
      hi &= hi - 1;
    }

    for (int j = 0; j < m; ++j) {
      if (j + kRing <= m)
        wait_vm<kRing - 1>();
      else
        wait_vm<0>();
      const uint32_t* lp = ring + (j % kRing) * kPageDwords;
      const int hl = ctz64(hq);
      hq &= hq - 1;
      const uint64_t pj = rl64(ptr, hl);
      const bool mine = !done && ptr == pj;
      if (!ptr_ok(pj, a.node, a.arena_bytes)) {
        if (mine) done = true;
        err |= kErrBadPtr;
      } else {
        const UHdr h = uniform_hdr(lp);
        const bool is_leaf = h.leftmost == 0;
        if (h.fver != h.rver) {
          // torn / in-flight page: its queries re-list it next round
          if (++retries > kMaxRetries) {
            if (mine) done = true;
            err |= kErrInconsistent;
          }
        } else if (mine && k >= h.highest) {
          ptr = h.sibling;  // turn right
          if (ptr == 0) done = true;
        } else if (mine && k < h.lowest) {
          ptr = a.root;  // stale route: restart (Tree.cpp:652-657)
          err |= kErrFence;
        } else if (LOCATE && (int)h.level == a.target_level) {
          if (mine) {
            page_out = pj;
            done = true;
          }
        } else if (!is_leaf) {
          if (LOCATE && (int)h.level < a.target_level) {
            if (mine) {
              done = true;
              err |= kErrFence;
            }
          } else if (mine) {
            int pos = 0;  // number of keys <= k (keys strictly increase)
#pragma unroll
            for (int step = 32; step > 0; step >>= 1) {
              const int idx = pos + step - 1;
              if (idx < h.cnt && lds_ikey(lp, idx) <= k) pos += step;
            }
            ptr = pos == 0 ? h.leftmost : lds_iptr(lp, pos - 1);
            if (ptr == 0) done = true;
          }
        } else if (LOCATE) {
          if (mine) {  // reached a leaf below the target level
            done = true;
            err |= kErrFence;
          }
        } else {
          // leaf (level 0): lane i holds entry i
          const LeafEnt e = leaf_entry(lp, lane < kLeafCardinality ? lane : 0);
          const bool ok = lane < kLeafCardinality && e.val != kValueNull &&
                          (e.fraw & 0xF) == (e.rraw & 0xF);
          // waiting queries are a sorted run: one ballot per distinct key
          uint64_t qm = ballot(mine);
          while (qm) {
            const uint64_t kq = rl64(k, ctz64(qm));
            const uint64_t same = ballot(mine && k == kq);
            qm &= ~same;
            const uint64_t mm = ballot(ok && e.key == kq);
            const uint64_t v = mm ? rl64(e.val, ctz64(mm)) : 0;
            if ((same >> lane) & 1) {
              done = true;
              val = v;
            }
          }
        }
      }
      // the slot's LDS reads are complete before its next DMA lands
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (hi) {
        glds16(a.arena + ga_offset(rl64(pload, ctz64(hi))),
               ring + (j % kRing) * kPageDwords);
        hi &= hi - 1;
      }
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
