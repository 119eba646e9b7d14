// walk.hip — batched B-link tree walk (Tree::search / locate for insert).
//
// Restates src/Tree.cpp:405-459 (search), 593-663 (page_search),
// 665-685 (internal_page_search) and 687-697 (leaf_page_search) for a batch:
// one wave64 owns 64 queries (one per lane).  Each round the wave picks up to
// D distinct page pointers among its unfinished queries, loads each 1 KB page
// with one coalesced dwordx4 per lane (D pages in flight), and resolves every
// query waiting on that page with a lane-parallel compare + ballot:
//   internal: child = popcount(ballot(key_j <= k)) -> leftmost / ptr[c-1]
//   leaf    : slot  = ffs(ballot(key_i == k && value_i != 0 && f_i == r_i))
// Queries that share a page (sorted batches) share one page read.  Fences are
// checked on every page (k >= highest -> sibling, the B-link "turn right");
// a page whose front/rear versions differ is re-read (Tree.cpp:616-618).
#include "device_common.h"
#include "kernels.h"

namespace shm {
namespace dev {

template <int D, bool LOCATE>
__global__ __launch_bounds__(kBlock) void k_walk(WalkArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t s_page[kWavesPerBlock][kPageDwords + 8];
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  const uint64_t n = a.n_dev ? *a.n_dev : a.n;
  const uint64_t wave_base =
      ((uint64_t)blockIdx.x * kWavesPerBlock + (uint64_t)wv) * kWave;
  if (wave_base >= n) return;  // wave-uniform
  const uint64_t i = wave_base + (uint64_t)lane;
  const bool active = i < n;
  // query i of the walk is input position perm[i] (key read and output)
  const uint64_t src = active ? (a.perm ? (uint64_t)a.perm[i] : i) : 0;
  const uint64_t k = active ? a.keys[src] : 0;
  uint64_t ptr = a.root;
  bool done = !active;
  uint64_t val = 0, page_out = 0;
  bool fnd = false;
  // kKeyMax can never be stored (root highest is exclusive, Tree.h:150)
  if (!LOCATE && k == kKeyMax) done = true;
  uint32_t* lp = s_page[wv];
  uint32_t err = 0;
  int rounds = 0, retries = 0;

  for (;;) {
    const uint64_t pend = ballot(!done);
    if (pend == 0) break;
    if (++rounds > kMaxRounds) {
      err |= kErrRounds;
      break;
    }
    // ---- pick up to D distinct pages --------------------------------------
    uint64_t P[D];
    uint64_t rem = pend;
#pragma unroll
    for (int j = 0; j < D; ++j) {
      P[j] = 0;
      if (rem) {
        const uint64_t p = rl64(ptr, ctz64(rem));
        P[j] = p;
        rem &= ~ballot(!done && ptr == p);
      }
    }
    // ---- issue all loads ----------------------------------------------------
    u32x4 pg[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
      if (P[j]) {
        if (!ptr_ok(P[j], a.node, a.arena_bytes)) {
          if (ptr == P[j]) done = true;
          err |= kErrBadPtr;
          P[j] = 0;
        } else {
          pg[j] = load_page_slice(a.arena, ga_offset(P[j]));
        }
      }
    }
    // ---- resolve every query waiting on each page -------------------------
#pragma unroll
    for (int j = 0; j < D; ++j) {
      if (!P[j]) continue;
      const uint64_t pj = P[j];
      const Hdr h = parse_hdr(pg[j]);
      const bool is_leaf = h.leftmost == 0;
      uint64_t qm = ballot(!done && ptr == pj);
      const uint32_t rv = is_leaf ? h.rver_leaf : h.rver_internal;
      if (h.fver != rv) {  // torn / in-flight page: re-read next round
        if (++retries > kMaxRetries) {
          if (ptr == pj) done = true;
          err |= kErrInconsistent;
        }
        continue;
      }
      if (LOCATE && (int)h.level == a.target_level) {
        // Tree::insert stops at the target level; fence check first
        while (qm) {
          const int q = ctz64(qm);
          qm &= qm - 1;
          const uint64_t kq = rl64(k, q);
          if (lane == q) {
            if (kq >= h.highest) {
              ptr = h.sibling;
              if (ptr == 0) done = true;
            } else if (kq < h.lowest) {
              done = true;
              err |= kErrFence;
            } else {
              page_out = pj;
              done = true;
            }
          }
        }
        continue;
      }
      if (!is_leaf) {
        if (LOCATE && (int)h.level < a.target_level) {
          if (ptr == pj) done = true;
          err |= kErrFence;
          continue;
        }
        const IntRec r = internal_record(pg[j]);
        const int cnt = h.last_index + 1;
        const bool valid = lane >= 3 && lane - 3 < cnt;
        while (qm) {
          const int q = ctz64(qm);
          qm &= qm - 1;
          const uint64_t kq = rl64(k, q);
          uint64_t np;
          bool bad = false;
          if (kq >= h.highest) {
            np = h.sibling;  // turn right (Tree.cpp:648-651)
          } else if (kq < h.lowest) {
            np = a.root;     // stale route: restart (Tree.cpp:652-657)
            bad = true;
          } else {
            const int c = popc64(ballot(valid && r.key <= kq));
            np = c == 0 ? h.leftmost : rl64(r.ptr, c + 2);
          }
          if (lane == q) {
            ptr = np;
            if (np == 0) done = true;
            if (bad) err |= kErrFence;
          }
        }
      } else {
        // leaf (level 0)
        stage_page(lp, pg[j]);
        wave_lds_sync();
        const LeafEnt e = leaf_entry(lp, lane < kLeafCardinality ? lane : 0);
        const bool ok = lane < kLeafCardinality && e.val != kValueNull &&
                        (e.fraw & 0xF) == (e.rraw & 0xF);
        while (qm) {
          const int q = ctz64(qm);
          qm &= qm - 1;
          const uint64_t kq = rl64(k, q);
          if (kq >= h.highest) {
            if (lane == q) {
              ptr = h.sibling;
              if (ptr == 0) done = true;
            }
          } else if (kq < h.lowest) {
            if (lane == q) {
              done = true;
              err |= kErrFence;
            }
          } else {
            const uint64_t mm = ballot(ok && e.key == kq);
            uint64_t v = 0;
            if (mm) v = rl64(e.val, ctz64(mm));
            if (lane == q) {
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
  }
  if (err) atomicOr(a.err, err);
  if (active) {
    if (LOCATE) {
      a.out_page[src] = page_out;
    } else {
      a.out_val[src] = val;
      if (a.out_found) a.out_found[src] = fnd ? 1 : 0;
    }
  }
}

void launch_walk(const WalkArgs& a, uint64_t n_upper, int depth, bool locate,
                 hipStream_t s) {
  if (n_upper == 0) return;
  const uint64_t waves = (n_upper + kWave - 1) / kWave;
  const dim3 grid((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock));
  if (locate) {
    hipLaunchKernelGGL((k_walk<4, true>), grid, dim3(kBlock), 0, s, a);
  } else if (depth >= 8) {
    hipLaunchKernelGGL((k_walk<8, false>), grid, dim3(kBlock), 0, s, a);
  } else {
    hipLaunchKernelGGL((k_walk<4, false>), grid, dim3(kBlock), 0, s, a);
  }
}

}  // namespace dev
}  // namespace shm
