// range.hip — batched range scans: the intended Tree::range_query
// (src/Tree.cpp:461-540: every leaf overlapping [from, to] in key order via
// the sibling chain, valid entries in slot order, Tree.cpp:509-516).
//
// The count pass stages each scan's first stage_cap values; the fill pass
// then copies the scans that fit and walks only the longer ones again.
//
// One wave per scan.  The start leaf comes from the leaf directory (or a
// descent from the covering internal page / the root with a ballot child
// select); B-link right turns fix a stale start.  Along the leaf chain the
// sibling page is loaded into registers as soon as the current header says
// the scan continues, so its HBM latency overlaps the current leaf's compare
// and store.  offsets == nullptr -> count only.
#include "device_common.h"
#include "kernels.h"

namespace shm {
namespace dev {

namespace {
constexpr int kRangeWaves = 4;
}

__global__ __launch_bounds__(kRangeWaves* kWave) void k_range(RangeArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t s_page[kRangeWaves][kPageDwords + 8];
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  const uint64_t q = (uint64_t)blockIdx.x * kRangeWaves + wv;
  if (q >= a.n) return;  // wave-uniform
  uint32_t* lp = s_page[wv];
  const uint64_t lo = a.from[q], hi = a.to[q];
  uint64_t cnt = 0;
  const uint64_t out = a.offsets ? a.offsets[q] : 0;
  uint32_t err = 0;
  uint64_t* stq = a.stage ? a.stage + q * (uint64_t)a.stage_cap : nullptr;
  if (a.offsets && stq && a.counts[q] <= a.stage_cap) {
    // fill pass, staged scan: copy its values out, no second walk
    const uint64_t c = a.counts[q];
    for (uint64_t i = (uint64_t)lane; i < c && out + i < a.vals_cap; i += kWave)
      a.vals[out + i] = stq[i];
    return;
  }
  if (lo <= hi) {
    uint64_t p = a.dir ? dir_start(a.dir, a.dir_lo, a.dir_shift, a.dir_n, a.node, lo, a.root) : a.root;
    int hops = 0;
    u32x4 w;
    // descend to the leaf whose fences hold lo
    for (;;) {
      if (++hops > kMaxRounds || !ptr_ok(p, a.node, a.arena_bytes)) {
        err |= kErrBadPtr;
        p = 0;
        break;
      }
      w = load_page_slice(a.arena, ga_offset(p));
      const Hdr h = parse_hdr(w);
      if (lo >= h.highest && h.sibling) {
        p = h.sibling;
        continue;
      }
      if (h.leftmost == 0) break;
      const IntRec r = internal_record(w);
      const int c = popc64(ballot(lane >= 3 && lane - 3 < h.last_index + 1 && r.key <= lo));
      p = c == 0 ? h.leftmost : rl64(r.ptr, c + 2);
    }
    // scan the leaf chain; w holds leaf p
    while (p) {
      const Hdr h = parse_hdr(w);
      const bool more = h.sibling != 0 && h.highest <= hi;
      u32x4 wn = w;
      if (more) {
        if (++hops > (1 << 24) || !ptr_ok(h.sibling, a.node, a.arena_bytes)) {
          err |= kErrBadPtr;
          break;
        }
        wn = load_page_slice(a.arena, ga_offset(h.sibling));  // in flight
      }
      stage_page(lp, w);
      wave_lds_sync();
      const LeafEnt e = leaf_entry(lp, lane < kLeafCardinality ? lane : 0);
      const bool hit = lane < kLeafCardinality && e.val != kValueNull &&
                       (e.fraw & 0xF) == (e.rraw & 0xF) && e.key >= lo && e.key <= hi;
      const uint64_t m = ballot(hit);
      const uint64_t slot = cnt + popc64(m & lanemask_lt());
      if (a.offsets && hit && out + slot < a.vals_cap) a.vals[out + slot] = e.val;
      if (!a.offsets && stq && hit && slot < a.stage_cap) stq[slot] = e.val;
      cnt += popc64(m);
      wave_lds_sync();  // LDS reads done before the next stage
      if (!more) break;
      p = h.sibling;
      w = wn;
    }
  }
  if (lane == 0) {
    if (err) atomicOr(a.err, err);
    a.counts[q] = cnt;
  }
}

void launch_range(const RangeArgs& a, hipStream_t s) {
  if (!a.n) return;
  hipLaunchKernelGGL(k_range, dim3((unsigned)((a.n + kRangeWaves - 1) / kRangeWaves)),
                     dim3(kRangeWaves * kWave), 0, s, a);
}

// zero-copy read-back (tree.cpp readback): one wave copies the words into
// mapped host memory with vector stores, fences at system scope, then lane 0
// publishes the sequence number the host spins on
__global__ void k_readback(uint32_t* dst, const uint32_t* src, uint32_t nw, uint32_t* flag,
                           uint32_t seq) {
  const uint32_t l = threadIdx.x;
  if (l < nw) dst[l] = src[l];
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
