// range.hip — batched range scans: the intended Tree::range_query
// (src/Tree.cpp:461-540: every leaf overlapping [from, to] in key order via
// the sibling chain, valid entries in slot order, Tree.cpp:509-516).
//
// The count pass stages each scan's first stage_cap values; the fill pass
// then copies the scans that fit and walks only the longer ones again.
//
// Four scans per wave, 16 lanes per scan.  A scan is a chain of dependent
// page reads (start leaf, then its siblings), so a wave that walks one scan
// waits on one page at a time; four independent chains per wave put four
// times the page reads in flight at the same occupancy.  Lane li of scan
// group q reads 16 B chunks li, li + 16, li + 32, li + 48 of the group's
// page (256 B coalesced per group per load), stages them in the group's
// 1 KB LDS slot, and compares 4 consecutive 18 B entries (leaf_chunk.h).
// The start leaf comes from the leaf directory (or a descent from the
// covering internal page / the root: 4 separators per lane, the child is
// the count of separators <= from); B-link right turns fix a stale start.
// Along the leaf chain the sibling page is loaded into registers as soon as
// the current header says the scan continues, so its HBM latency overlaps
// the current leaf's compare and stores.  offsets == nullptr -> count only.
#include "device_common.h"
#include "kernels.h"
#include "leaf_chunk.h"

namespace shm {
namespace dev {

namespace {
constexpr int kRangeWaves = 4;
constexpr int kRG = 4;                        // scans per wave
constexpr int kRL = kWave / kRG;              // lanes per scan
constexpr int kRE = 4;                        // leaf entries per lane
constexpr int kRCD = kLeafEntry * kRE / 4;    // dwords of a lane's entry chunk
constexpr int kRChunks = kPageSize / 16 / kRL;  // 16 B page chunks per lane
static_assert(kRL * kRE >= kLeafCardinality, "entries per group");

struct RPage {
  u32x4 c[kRChunks];
};

__device__ __forceinline__ void rload(const uint8_t* arena, uint64_t p, int li, RPage& w) {
  const uint8_t* b = arena + ga_offset(p) + 16 * li;
#pragma unroll
  for (int k = 0; k < kRChunks; ++k) w.c[k] = *reinterpret_cast<const u32x4*>(b + 16 * kRL * k);
}
// chunks 0..2 (bytes 0..767: the header and slots 0..39); chunk 3 (slots
// 40..53 and the rear version) only when the leaf's occupancy bound says a
// valid slot may lie there (layout.h leaf_hw: every slot >= hw is empty)
constexpr uint32_t kChunk3Hw = 41;  // slot 40 ends past byte 767
__device__ __forceinline__ void rload3(const uint8_t* arena, uint64_t p, int li, RPage& w) {
  const uint8_t* b = arena + ga_offset(p) + 16 * li;
#pragma unroll
  for (int k = 0; k < kRChunks - 1; ++k)
    w.c[k] = *reinterpret_cast<const u32x4*>(b + 16 * kRL * k);
}
__device__ __forceinline__ void rload_last(const uint8_t* arena, uint64_t p, int li, RPage& w) {
  w.c[kRChunks - 1] =
      *reinterpret_cast<const u32x4*>(arena + ga_offset(p) + 16 * li + 16 * kRL * (kRChunks - 1));
}
__device__ __forceinline__ void rstage(uint32_t* lp, int li, const RPage& w) {
#pragma unroll
  for (int k = 0; k < kRChunks; ++k) *reinterpret_cast<u32x4*>(lp + 4 * (li + kRL * k)) = w.c[k];
}
__device__ __forceinline__ uint64_t lds_u64(const uint32_t* lp, int d) {
  return (uint64_t)lp[d] | ((uint64_t)lp[d + 1] << 32);
}
// header fields of a staged page (Tree.h:130-160; bytes 9..43)
__device__ __forceinline__ uint64_t hdr_leftmost(const uint32_t* lp) {
  const uint32_t a2 = lp[2], a3 = lp[3], b0 = lp[4];
  return (uint64_t)((a2 >> 8) | (a3 << 24)) | ((uint64_t)((a3 >> 8) | (b0 << 24)) << 32);
}
__device__ __forceinline__ uint64_t hdr_sibling(const uint32_t* lp) {
  const uint32_t b0 = lp[4], b1 = lp[5], b2 = lp[6];
  return (uint64_t)((b0 >> 8) | (b1 << 24)) | ((uint64_t)((b1 >> 8) | (b2 << 24)) << 32);
}
// exclusive prefix of v over the 16 lanes of each scan group; *tot = group sum
__device__ __forceinline__ uint32_t group_scan(uint32_t v, int li, uint32_t* tot) {
  uint32_t incl = v;
#pragma unroll
  for (int off = 1; off < kRL; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, off, kRL);
    if (li >= off) incl += y;
  }
  *tot = (uint32_t)__shfl((int)incl, kRL - 1, kRL);
  return incl - v;
}
}  // namespace

// The scan's leaves as the leaf directory lists them (the plan).  Lane li
// of the group reads entry p0 + li of the prefixes [lo, hi] spans (32 B;
// the group's reads are in flight together, in place of the one dir_start
// read) and contributes the leaves of its entry that may hold keys in
// [lo, hi]: from lo's leaf (dir_start's rule) in the first entry, up to the
// last leaf whose split point is <= hi's in the last one, minus the previous
// entry's last leaf (a leaf spanning prefixes is listed by each).  A prefix
// of more than four leaves (an entry naming an internal page) ends the plan
// before it.  Returns the plan length m (0: no plan); lane j of the group
// holds leaf j's page index in pl (j < m).  The directory may be stale: the
// walk follows the plan only while each leaf's sibling pointer names the
// next planned leaf, so a plan only decides which page reads are issued
// early, never what the scan returns.  Wave-uniform call.
__device__ __forceinline__ uint32_t range_plan(const RangeArgs& a, bool act, uint64_t lo,
                                               uint64_t hi, int li, int q, uint32_t* sp,
                                               uint32_t& pl) {
  const bool ok =
      act && a.plan && a.dir != nullptr && dir_covers(a.dir_lo, a.dir_shift, a.dir_n, lo);
  uint64_t p0 = 0, p1 = 0;
  bool hi_in = false;  // hi inside the directory (else its last entry is taken whole)
  if (ok) {
    p0 = (lo - a.dir_lo) >> a.dir_shift;
    p1 = (hi - a.dir_lo) >> a.dir_shift;
    hi_in = p1 < a.dir_n;
    if (!hi_in) p1 = a.dir_n - 1;
  }
  const uint64_t pe = p0 + (uint64_t)li;
  const bool mine = ok && pe <= p1;
  u32x4 e0{0u, 0u, 0u, 0u}, e1{0u, 0u, 0u, 0u};
  if (mine) {
    const u32x4* ep = reinterpret_cast<const u32x4*>(a.dir + kDirWords * pe);
    e0 = ep[0];
    e1 = ep[1];
  }
  const uint32_t cnt = e1.w & 0xFFu;
  const bool fp = (e1.w & kDirFp) != 0;
  uint32_t is = 0, ie = cnt ? cnt - 1 : 0;
  if (mine && !fp && cnt > 1) {
    const bool exact = a.dir_shift <= 32;
    auto tkey = [&](uint64_t k) {
      const uint64_t off = (k - a.dir_lo) - (pe << a.dir_shift);
      return exact ? (uint32_t)off : (uint32_t)(off >> (a.dir_shift - 32));
    };
    if (li == 0) {  // dir_start's rule: the leaves whose split point is past lo's
      const uint32_t tk = tkey(lo);
      auto past = [&](uint32_t t) { return t < tk || (exact && t == tk); };
      is = (uint32_t)past(e1.x) + (uint32_t)(cnt > 2 && past(e1.y)) +
           (uint32_t)(cnt > 3 && past(e1.z));
    }
    if (pe == p1 && hi_in) {  // the leaves that may hold a key <= hi
      const uint32_t tk = tkey(hi);
      ie = (uint32_t)(e1.x <= tk) + (uint32_t)(cnt > 2 && e1.y <= tk) +
           (uint32_t)(cnt > 3 && e1.z <= tk);
      if (ie < is) ie = is;
    }
  }
  auto comp = [&](uint32_t i) { return i == 0 ? e0.x : i == 1 ? e0.y : i == 2 ? e0.z : e0.w; };
  // the plan stops before the first entry that names an internal page
  const uint32_t badm = (uint32_t)(ballot(mine && cnt == 0) >> (kRL * q)) & 0xFFFFu;
  const int first_bad = badm ? __builtin_ctz(badm) : kRL;
  uint32_t c = mine && li < first_bad ? ie - is + 1 : 0u;
  const uint32_t lastpg = comp(ie);
  const uint32_t prevlast = (uint32_t)__shfl((int)lastpg, li > 0 ? li - 1 : 0, kRL);
  if (c && li > 0 && comp(is) == prevlast) {
    ++is;
    --c;
  }
  uint32_t tot;
  const uint32_t x = group_scan(c, li, &tot);
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k)
    if (k < c && x + k < (uint32_t)kRL) sp[x + k] = comp(is + k);
  wave_lds_sync();
  const uint32_t m = tot < (uint32_t)kRL ? tot : (uint32_t)kRL;
  pl = (uint32_t)li < m ? sp[li] : 0u;
  wave_lds_sync();  // plan read before the group's slot is reused
  return m;
}

// a leaf's page read: bytes 0..767 always, the last 256 B when its
// occupancy bound h reaches slot 40
__device__ __forceinline__ void rload_hw(const uint8_t* arena, uint64_t p, uint32_t h, int li,
                                         RPage& w) {
  rload3(arena, p, li, w);
  if (h >= kChunk3Hw) rload_last(arena, p, li, w);
}

// Walks one scan per group of the wave (act: the group has one) from the
// leaf directory / root down to lo's leaf and along the sibling chain to hi;
// its hit values in key order go to dst0[slot] for slot < cap0, then to
// dst1[slot - cap0] for the next cap1 slots (either nullable with cap 0).
// Returns the scan's value count.  Wave-uniform call (ballot loops); lp =
// the group's 1 KB LDS page slot, sp = its plan words (kRL).
//
// With a directory plan (range_plan) the leaf reads are issued two ahead:
// while leaf j is compared, leaves j + 1 and j + 2 are in flight, their
// addresses taken from the plan instead of from the previous leaf's header,
// so a scan of L leaves waits about one page latency instead of L.  The two
// register pages alternate roles (the chain loop is unrolled by two), so no
// page is copied between registers.
__device__ __forceinline__ uint64_t range_walk(const RangeArgs& a, bool act, uint64_t lo,
                                               uint64_t hi, uint32_t* lp, uint32_t* sp, int li,
                                               int q, uint64_t* dst0, uint64_t cap0,
                                               uint64_t* dst1, uint64_t cap1, uint32_t& err) {
  uint64_t cnt = 0;
  // ---- plan, then descend to the leaf whose fences hold lo ---------------------
  uint32_t pl = 0;
  const uint32_t m = range_plan(a, act, lo, hi, li, q, sp, pl);
  // occupancy bound of planned leaf li (the 1.8 MB array is L2-resident)
  uint32_t hwl = kLeafHwFull;
  if (a.leaf_hw && (uint32_t)li < m) hwl = a.leaf_hw[pl];
  RPage w, wn;
  uint64_t p = 0;
  int hops = 0;
  uint32_t hw = kLeafCardinality;  // slots of the current leaf that may be valid
  bool planned = m > 0;            // the current leaf is plan[j]
  uint32_t j = 0;
  bool y_ok = false;  // the other register page holds leaf yp (issued)
  uint64_t yp = 0;
  uint32_t hwy = kLeafCardinality;
  const uint64_t pp0 = dir_page_ga((uint32_t)__shfl((int)pl, 0, kRL), a.node);
  const uint64_t pp1 = dir_page_ga((uint32_t)__shfl((int)pl, 1, kRL), a.node);
  if (act) {
    if (planned) {
      // the first two planned leaves' first 768 B at once
      p = pp0;
      if (ptr_ok(p, a.node, a.arena_bytes)) rload3(a.arena, p, li, w);
      if (m > 1 && ptr_ok(pp1, a.node, a.arena_bytes)) {
        yp = pp1;
        y_ok = true;
        rload3(a.arena, yp, li, wn);
      }
    } else {
      p = a.dir ? dir_start(a.dir, a.dir_lo, a.dir_shift, a.dir_n, a.node, lo, a.root) : a.root;
    }
  }
  const uint32_t h0 = (uint32_t)__shfl((int)hwl, 0, kRL);
  const uint32_t h1 = (uint32_t)__shfl((int)hwl, 1, kRL);
  if (act) {
    if (!ptr_ok(p, a.node, a.arena_bytes)) {
      err |= kErrBadPtr;
      act = false;
    } else if (planned) {
      // their last 256 B once the occupancy bounds are in
      if (h0 >= kChunk3Hw) rload_last(a.arena, p, li, w);
      hw = h0 < (uint32_t)kLeafCardinality ? h0 : (uint32_t)kLeafCardinality;
      if (y_ok) {
        if (h1 >= kChunk3Hw) rload_last(a.arena, yp, li, wn);
        hwy = h1 < (uint32_t)kLeafCardinality ? h1 : (uint32_t)kLeafCardinality;
      }
    } else if (a.leaf_hw) {
      // the start page's last 256 B only if its occupancy bound reaches
      // slot 40 (internal pages: kLeafHwFull, read whole)
      const uint32_t h = a.leaf_hw[ga_offset(p) >> 10];
      rload_hw(a.arena, p, h, li, w);
      hw = h < (uint32_t)kLeafCardinality ? h : (uint32_t)kLeafCardinality;
    } else {
      rload(a.arena, p, li, w);
    }
  }
  bool desc = act;
  while (ballot(desc)) {
    if (desc) rstage(lp, li, w);
    wave_lds_sync();
    if (desc) {
      const uint64_t sibling = hdr_sibling(lp);
      const uint64_t highest = lds_u64(lp, 9);
      const uint64_t leftmost = hdr_leftmost(lp);
      uint64_t np = 0;
      if (lo >= highest && sibling) {
        np = sibling;
      } else if (leftmost != 0) {
        // internal page (Tree.cpp:665-685): child = number of keys <= lo
        const int last = (int)(int16_t)(lp[6] >> 16);
        uint32_t c = 0;
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
          const int jj = li + kRL * mm;
          c += (jj <= last && jj < kInternalCardinality && lds_u64(lp, 11 + 4 * jj) <= lo) ? 1u : 0u;
        }
        uint32_t tot;
        (void)group_scan(c, li, &tot);
        np = tot == 0 ? leftmost : lds_u64(lp, 13 + 4 * ((int)tot - 1));
      }
      if (np) {
        planned = false;  // a stale start: the chain from here
        y_ok = false;
        if (++hops > kMaxRounds || !ptr_ok(np, a.node, a.arena_bytes)) {
          err |= kErrBadPtr;
          act = false;
          desc = false;
        } else {
          p = np;
          hw = kLeafCardinality;  // read whole below
        }
      } else {
        desc = false;  // a leaf: w holds it
      }
    }
    wave_lds_sync();  // LDS reads done before the next stage
    if (desc) rload(a.arena, p, li, w);
  }

  // ---- scan the leaf chain; X holds leaf p --------------------------------------
  // (a leaf's bytes past slot hw - 1 are not read)
  const int ebase = chunk_base<kRE>(li);
  auto step = [&](RPage& X, RPage& Y) {
    // leaf j + 2 of the plan (all lanes: the shuffles are wave-wide)
    const uint32_t j2 = j + 2 < (uint32_t)kRL ? j + 2 : (uint32_t)kRL - 1;
    const uint32_t pg2 = (uint32_t)__shfl((int)pl, (int)j2, kRL);
    const uint32_t hw2 = (uint32_t)__shfl((int)hwl, (int)j2, kRL);
    if (act) rstage(lp, li, X);
    wave_lds_sync();
    bool more = false, late = false, x_ok = false;
    uint64_t sibling = 0, xp = 0;
    uint32_t hwn = kLeafHwFull;
    bool hit[kRE];
    uint64_t ev[kRE];
#pragma unroll
    for (int jj = 0; jj < kRE; ++jj) {
      hit[jj] = false;
      ev[jj] = 0;
    }
    if (act) {
      sibling = hdr_sibling(lp);
      const uint64_t highest = lds_u64(lp, 9);
      more = sibling != 0 && highest <= hi;
      if (more) {
        if (++hops > (1 << 24) || !ptr_ok(sibling, a.node, a.arena_bytes)) {
          err |= kErrBadPtr;
          more = false;
        } else {
          if (!(y_ok && yp == sibling)) {
            // off the plan (or none): the sibling's bound (L2-resident) and
            // its first 768 bytes now, its last 256 B after the compare
            planned = false;
            if (a.leaf_hw) hwn = a.leaf_hw[ga_offset(sibling) >> 10];
            rload3(a.arena, sibling, li, Y);
            late = true;
          }
          if (planned && j + 2 < m) {
            // X is staged: it takes leaf j + 2 while j is compared
            xp = dir_page_ga(pg2, a.node);
            if (ptr_ok(xp, a.node, a.arena_bytes)) {
              rload_hw(a.arena, xp, hw2, li, X);
              x_ok = true;
            }
          }
        }
      }
      uint32_t D[kRCD];
      const uint32_t* ep = lp + (kOffRecords + kLeafEntry * ebase) / 4;
#pragma unroll
      for (int i = 0; i < kRCD; ++i) D[i] = ep[i];
      uint64_t ek[kRE];
      uint32_t ef[kRE], er[kRE];
      chunk_entries<kRE>(D, ek, ev, ef, er);
#pragma unroll
      for (int jj = 0; jj < kRE; ++jj)
        hit[jj] = ebase + jj >= li * kRE && (uint32_t)(ebase + jj) < hw &&
                  ev[jj] != kValueNull && ((ef[jj] ^ er[jj]) & 0xF) == 0 && ek[jj] >= lo &&
                  ek[jj] <= hi;
    }
    uint32_t c = 0;
#pragma unroll
    for (int jj = 0; jj < kRE; ++jj) c += hit[jj] ? 1u : 0u;
    uint32_t tot;
    uint64_t slot = cnt + group_scan(c, li, &tot);
#pragma unroll
    for (int jj = 0; jj < kRE; ++jj) {
      if (hit[jj]) {
        if (slot < cap0)
          dst0[slot] = ev[jj];
        else if (slot - cap0 < cap1)
          dst1[slot - cap0] = ev[jj];
        ++slot;
      }
    }
    cnt += tot;
    wave_lds_sync();  // LDS reads done before the next stage
    if (act) {
      if (more) {
        if (late) {
          if (hwn >= kChunk3Hw) rload_last(a.arena, sibling, li, Y);
          hw = hwn < (uint32_t)kLeafCardinality ? hwn : (uint32_t)kLeafCardinality;
        } else {
          hw = hwy;
        }
        p = sibling;
        ++j;
        y_ok = x_ok;  // the next step's other page is X
        yp = xp;
        hwy = hw2 < (uint32_t)kLeafCardinality ? hw2 : (uint32_t)kLeafCardinality;
      } else {
        act = false;
      }
    }
  };
  while (ballot(act)) {
    step(w, wn);
    if (!ballot(act)) break;
    step(wn, w);
  }
  return cnt;
}

__global__ __launch_bounds__(kRangeWaves* kWave) void k_range(RangeArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t s_page[kRangeWaves][kRG * kPageDwords];
  __shared__ uint32_t s_plan[kRangeWaves][kRG * kRL];
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  const int q = lane / kRL, li = lane % kRL;
  const uint64_t Q = ((uint64_t)blockIdx.x * kRangeWaves + (uint64_t)wv) * kRG + (uint64_t)q;
  const bool has = Q < a.n;
  if (!ballot(has)) return;  // wave-uniform
  uint32_t* lp = s_page[wv] + q * kPageDwords;
  uint32_t* sp = s_plan[wv] + q * kRL;
  uint64_t lo = 0, hi = 0, out = 0;
  if (has) {
    lo = a.from[Q];
    hi = a.to[Q];
    if (a.offsets) out = a.offsets[Q];
  }
  uint32_t err = 0;
  uint64_t* stq = (a.stage && has) ? a.stage + Q * (uint64_t)a.stage_cap : nullptr;
  bool act = has && lo <= hi;
  bool copied = false;
  if (a.offsets && stq) {
    // fill pass, staged scan: copy its values out, no second walk
    const uint64_t c = a.counts[Q];
    copied = c <= a.stage_cap;
    if (copied) {
      for (uint64_t b = 0; b < c; b += kRL * 4) {
        uint64_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint64_t i = b + (uint64_t)(li + kRL * u);
          v[u] = i < c ? stq[i] : 0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint64_t i = b + (uint64_t)(li + kRL * u);
          if (i < c && out + i < a.vals_cap) a.vals[out + i] = v[u];
        }
      }
      act = false;
    }
  }

  uint64_t* dst = stq;
  uint64_t cap = stq ? a.stage_cap : 0;
  if (a.offsets) {
    dst = a.vals + out;
    cap = out < a.vals_cap ? a.vals_cap - out : 0;
  }
  const uint64_t cnt = range_walk(a, act, lo, hi, lp, sp, li, q, dst, cap, nullptr, 0, err);
  if (has && !copied && li == 0) {
    a.counts[Q] = cnt;
    if (a.status && cnt > a.stage_cap)
      atomicAdd(reinterpret_cast<unsigned long long*>(a.status), 1ull);
  }
  if (err) {
    atomicOr(a.err, err);
    if (a.status) atomicOr(reinterpret_cast<unsigned long long*>(a.status + 1), (unsigned long long)err);
  }
}

void launch_range(const RangeArgs& a, hipStream_t s) {
  if (!a.n) return;
  const uint64_t per = (uint64_t)kRangeWaves * kRG;
  hipLaunchKernelGGL(k_range, dim3((unsigned)((a.n + per - 1) / per)), dim3(kRangeWaves * kWave),
                     0, s, a);
}

// zero-copy read-back (tree.cpp readback): one wave copies the words into
// mapped host memory with vector stores, fences at system scope, then lane 0
// publishes the sequence number the host spins on
__global__ void k_readback(uint32_t* dst, const uint32_t* src, uint32_t nw, uint32_t* flag,
                           uint32_t seq) {
  for (uint32_t l = threadIdx.x; l < nw; l += blockDim.x) dst[l] = src[l];
  const uint32_t l = threadIdx.x;
  __threadfence_system();
  __syncthreads();
  if (l == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_readback(uint32_t* dst, const uint32_t* src, uint32_t nw, uint32_t* flag,
                     uint32_t seq, hipStream_t s) {
  hipLaunchKernelGGL(k_readback, dim3(1), dim3(64), 0, s, dst, src, nw, flag, seq);
}

__global__ void k_add_u64(uint64_t* x, uint64_t n, uint64_t c) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] += c;
}

void launch_add_u64(uint64_t* x, uint64_t n, uint64_t c, hipStream_t s) {
  if (n && c) hipLaunchKernelGGL(k_add_u64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                                 x, n, c);
}

}  // namespace dev
}  // namespace shm
