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

// Walks one scan per group of the wave (act: the group has one) from the
// leaf directory / root down to lo's leaf and along the sibling chain to hi;
// its hit values in key order go to dst0[slot] for slot < cap0, then to
// dst1[slot - cap0] for the next cap1 slots (either nullable with cap 0).
// Returns the scan's value count.  Wave-uniform call (ballot loops); lp =
// the group's 1 KB LDS page slot.
__device__ __forceinline__ uint64_t range_walk(const RangeArgs& a, bool act, uint64_t lo,
                                               uint64_t hi, uint32_t* lp, int li, uint64_t* dst0,
                                               uint64_t cap0, uint64_t* dst1, uint64_t cap1,
                                               uint32_t& err) {
  uint64_t cnt = 0;
  // ---- descend to the leaf whose fences hold lo ------------------------------
  RPage w;
  uint64_t p = 0;
  int hops = 0;
  uint32_t hw = kLeafCardinality;  // slots of the current leaf that may be valid
  if (act) {
    p = a.dir ? dir_start(a.dir, a.dir_lo, a.dir_shift, a.dir_n, a.node, lo, a.root) : a.root;
    if (!ptr_ok(p, a.node, a.arena_bytes)) {
      err |= kErrBadPtr;
      act = false;
    } else if (a.leaf_hw) {
      // the start page's last 256 B only if its occupancy bound reaches
      // slot 40 (internal pages: kLeafHwFull, read whole)
      const uint32_t h = a.leaf_hw[ga_offset(p) >> 10];
      rload3(a.arena, p, li, w);
      if (h >= kChunk3Hw) rload_last(a.arena, p, li, w);
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
        for (int m = 0; m < 4; ++m) {
          const int j = li + kRL * m;
          c += (j <= last && j < kInternalCardinality && lds_u64(lp, 11 + 4 * j) <= lo) ? 1u : 0u;
        }
        uint32_t tot;
        (void)group_scan(c, li, &tot);
        np = tot == 0 ? leftmost : lds_u64(lp, 13 + 4 * ((int)tot - 1));
      }
      if (np) {
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

  // ---- scan the leaf chain; w holds leaf p ------------------------------------
  // (a leaf's bytes past slot hw - 1 are not read)
  const int ebase = chunk_base<kRE>(li);
  while (ballot(act)) {
    if (act) rstage(lp, li, w);
    wave_lds_sync();
    bool more = false;
    uint64_t sibling = 0;
    uint32_t hwn = kLeafHwFull;
    // w is staged: its registers take the sibling's bytes (one page of
    // registers per lane, not two: 88 -> 77 VGPRs, 5 -> 6 waves per SIMD,
    // k_range 63.4 -> 62.7 us in the bench's profile pass.  Pages by LDS-DMA
    // instead, one slot per scan, measured 66.3: the slot refills only after
    // the page's compare, and the entry unpack still held 86 VGPRs)
    bool hit[kRE];
    uint64_t ev[kRE];
#pragma unroll
    for (int j = 0; j < kRE; ++j) {
      hit[j] = false;
      ev[j] = 0;
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
          // in flight: the sibling's bound (a 1.8 MB array, L2-resident) and
          // its first 768 bytes
          if (a.leaf_hw) hwn = a.leaf_hw[ga_offset(sibling) >> 10];
          rload3(a.arena, sibling, li, w);
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
      for (int j = 0; j < kRE; ++j)
        hit[j] = ebase + j >= li * kRE && (uint32_t)(ebase + j) < hw && ev[j] != kValueNull &&
                 ((ef[j] ^ er[j]) & 0xF) == 0 && ek[j] >= lo && ek[j] <= hi;
    }
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < kRE; ++j) c += hit[j] ? 1u : 0u;
    uint32_t tot;
    uint64_t slot = cnt + group_scan(c, li, &tot);
#pragma unroll
    for (int j = 0; j < kRE; ++j) {
      if (hit[j]) {
        if (slot < cap0)
          dst0[slot] = ev[j];
        else if (slot - cap0 < cap1)
          dst1[slot - cap0] = ev[j];
        ++slot;
      }
    }
    cnt += tot;
    wave_lds_sync();  // LDS reads done before the next stage
    if (act) {
      if (more) {
        if (hwn >= kChunk3Hw) rload_last(a.arena, sibling, li, w);
        hw = hwn < (uint32_t)kLeafCardinality ? hwn : (uint32_t)kLeafCardinality;
        p = sibling;
      } else {
        act = false;
      }
    }
  }
  return cnt;
}

__global__ __launch_bounds__(kRangeWaves* kWave) void k_range(RangeArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t s_page[kRangeWaves][kRG * kPageDwords];
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  const int q = lane / kRL, li = lane % kRL;
  const uint64_t Q = ((uint64_t)blockIdx.x * kRangeWaves + (uint64_t)wv) * kRG + (uint64_t)q;
  const bool has = Q < a.n;
  if (!ballot(has)) return;  // wave-uniform
  uint32_t* lp = s_page[wv] + q * kPageDwords;
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
  const uint64_t cnt = range_walk(a, act, lo, hi, lp, li, dst, cap, nullptr, 0, err);
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
// publishes the sequence number the host spins on.  clear: each word is
// taken by an atomic exchange with 0 (the error block: a bit another stream
// sets after the exchange stays for the next read)
__global__ void k_readback(uint32_t* dst, uint32_t* src, uint32_t nw, uint32_t* flag,
                           uint32_t seq, int clear) {
  for (uint32_t l = threadIdx.x; l < nw; l += blockDim.x)
    dst[l] = clear ? atomicExch(src + l, 0u) : src[l];
  const uint32_t l = threadIdx.x;
  __threadfence_system();
  // the fence's write-back performed before the flag (the returned exchanges
  // above let the compiler drop the fence's own wait: MI355X_MICROARCH.md
  // "Compiler hazard")
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (l == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_readback(uint32_t* dst, const uint32_t* src, uint32_t nw, uint32_t* flag,
                     uint32_t seq, int clear, hipStream_t s) {
  hipLaunchKernelGGL(k_readback, dim3(1), dim3(64), 0, s, dst, const_cast<uint32_t*>(src), nw,
                     flag, seq, clear);
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
