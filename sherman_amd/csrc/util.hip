// util.hip — batch bookkeeping kernels (sort companions, segmentation,
// multi-GPU routing, key generation) and the batched range scan.
#include "device_common.h"
#include "kernels.h"

namespace shm {
namespace dev {

namespace {
constexpr int kT = 256;
inline dim3 grid1(uint64_t n, int per = kT) {
  return dim3((unsigned)((n + per - 1) / per));
}
}  // namespace

__global__ void k_iota(uint32_t* idx, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) idx[i] = (uint32_t)i;
}
void launch_iota(uint32_t* idx, uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_iota, grid1(n), dim3(kT), 0, s, idx, n);
}

__global__ void k_top32(const uint64_t* keys, uint64_t n, uint32_t* out,
                        uint32_t* idx) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    out[i] = (uint32_t)(keys[i] >> 32);
    idx[i] = (uint32_t)i;
  }
}
void launch_top32(const uint64_t* keys, uint64_t n, uint32_t* out,
                  uint32_t* idx, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_top32, grid1(n), dim3(kT), 0, s, keys, n, out, idx);
}

// last occurrence of each key in the (stable) sorted batch wins
// (last writer in batch order); low word counts upserts, high word deletes.
__global__ void k_mark_unique(const uint64_t* sk, const uint32_t* sidx,
                              const uint64_t* vals, uint64_t n, uint64_t* flags,
                              uint32_t* err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = sk[i];
  const bool last = i + 1 == n || sk[i + 1] != k;
  uint64_t f = 0;
  if (k == kKeyMax) {
    atomicOr(err, 1u << 31);  // EINVAL marker
  } else if (last) {
    f = vals[sidx[i]] != kValueNull ? 1ull : (1ull << 32);
  }
  flags[i] = f;
}
void launch_mark_unique(const uint64_t* sk, const uint32_t* sidx,
                        const uint64_t* vals, uint64_t n, uint64_t* flags,
                        uint32_t* err, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_mark_unique, grid1(n), dim3(kT), 0, s, sk, sidx, vals, n, flags, err);
}

__global__ void k_compact_unique(const uint64_t* sk, const uint32_t* sidx,
                                 const uint64_t* vals, const uint64_t* flags,
                                 const uint64_t* pos, uint64_t n, uint64_t* uk,
                                 uint64_t* uv, uint64_t* dk, uint64_t* counts) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t f = flags[i], p = pos[i];
  if (f & 0xFFFFFFFFull) {
    uk[p & 0xFFFFFFFFull] = sk[i];
    uv[p & 0xFFFFFFFFull] = vals[sidx[i]];
  } else if (f >> 32) {
    dk[p >> 32] = sk[i];
  }
  if (i + 1 == n) {
    const uint64_t t = p + f;
    counts[0] = t & 0xFFFFFFFFull;
    counts[1] = t >> 32;
  }
}
void launch_compact_unique(const uint64_t* sk, const uint32_t* sidx,
                           const uint64_t* vals, const uint64_t* flags,
                           const uint64_t* pos, uint64_t n, uint64_t* uk,
                           uint64_t* uv, uint64_t* dk, uint64_t* counts,
                           hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_compact_unique, grid1(n), dim3(kT), 0, s, sk, sidx, vals, flags, pos, n, uk, uv, dk, counts);
}

__global__ void k_seg_heads(const uint64_t* page, uint64_t n, uint32_t* heads) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  heads[i] = (i == 0 || page[i] != page[i - 1]) ? 1u : 0u;
}
void launch_seg_heads(const uint64_t* page, uint64_t n, uint32_t* heads,
                      hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_seg_heads, grid1(n), dim3(kT), 0, s, page, n, heads);
}

__global__ void k_seg_fill(const uint64_t* page, const uint32_t* heads,
                           const uint32_t* pos, uint64_t n, uint32_t* seg_start,
                           uint64_t* seg_page, uint32_t* num_seg) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (heads[i]) {
    seg_start[pos[i]] = (uint32_t)i;
    seg_page[pos[i]] = page[i];
  }
  if (i + 1 == n) {
    const uint32_t ns = pos[i] + heads[i];
    *num_seg = ns;
    seg_start[ns] = (uint32_t)n;
  }
}
void launch_seg_fill(const uint64_t* page, const uint32_t* heads,
                     const uint32_t* pos, uint64_t n, uint32_t* seg_start,
                     uint64_t* seg_page, uint32_t* num_seg, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_seg_fill, grid1(n), dim3(kT), 0, s, page, heads, pos, n, seg_start, seg_page, num_seg);
}

// to_key without / with the modulus (test/benchmark.cpp:43-46)
__global__ void k_gen_keys(uint64_t first, uint64_t n, uint64_t keyspace,
                           uint64_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = cityhash64_u64(first + i) + 1;
  out[i] = keyspace ? h % keyspace : h;
}
void launch_gen_keys(uint64_t first, uint64_t n, uint64_t keyspace,
                     uint64_t* out, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_gen_keys, grid1(n), dim3(kT), 0, s, first, n, keyspace, out);
}

// ---- multi-GPU routing: shard s owns [s*2^64/P, (s+1)*2^64/P) -------------
__device__ __forceinline__ uint32_t owner_of(uint64_t k, uint32_t shards) {
  return (uint32_t)__umul64hi(k, (uint64_t)shards);
}
constexpr int kRouteMaxShards = 64;
constexpr int kRoutePer = 4;  // keys per thread

__global__ void k_route_count(const uint64_t* keys, uint64_t n, uint32_t shards,
                              uint32_t* cnt) {
  __shared__ uint32_t c[kRouteMaxShards];
  if (threadIdx.x < kRouteMaxShards) c[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kT * kRoutePer;
  for (int r = 0; r < kRoutePer; ++r) {
    const uint64_t i = base + (uint64_t)r * kT + threadIdx.x;
    if (i < n) atomicAdd(&c[owner_of(keys[i], shards)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < shards && c[threadIdx.x]) atomicAdd(&cnt[threadIdx.x], c[threadIdx.x]);
}
// cursor[s] = exclusive prefix of cnt; counts_out[s] = cnt[s]
__global__ void k_route_scan(const uint32_t* cnt, uint32_t shards,
                             uint32_t* cursor, uint64_t* counts_out) {
  if (threadIdx.x != 0) return;
  uint32_t acc = 0;
  for (uint32_t s = 0; s < shards; ++s) {
    cursor[s] = acc;
    counts_out[s] = cnt[s];
    acc += cnt[s];
  }
}
__global__ void k_route_scatter(const uint64_t* keys, uint64_t n,
                                uint32_t shards, uint32_t* cursor,
                                uint64_t* keys_out, uint32_t* perm) {
  __shared__ uint32_t c[kRouteMaxShards];
  __shared__ uint32_t b[kRouteMaxShards];
  if (threadIdx.x < kRouteMaxShards) c[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kT * kRoutePer;
  uint32_t own[kRoutePer], rank[kRoutePer];
  uint64_t kk[kRoutePer];
  for (int r = 0; r < kRoutePer; ++r) {
    const uint64_t i = base + (uint64_t)r * kT + threadIdx.x;
    own[r] = ~0u;
    if (i < n) {
      kk[r] = keys[i];
      own[r] = owner_of(kk[r], shards);
      rank[r] = atomicAdd(&c[own[r]], 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x < shards) b[threadIdx.x] = c[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], c[threadIdx.x]) : 0;
  __syncthreads();
  for (int r = 0; r < kRoutePer; ++r) {
    if (own[r] == ~0u) continue;
    const uint64_t i = base + (uint64_t)r * kT + threadIdx.x;
    const uint32_t o = b[own[r]] + rank[r];
    keys_out[o] = kk[r];
    perm[o] = (uint32_t)i;
  }
}
void launch_route_bucket(const uint64_t* keys, uint64_t n, uint32_t shards,
                         uint64_t* counts, uint64_t* keys_out, uint32_t* perm,
                         uint32_t* cursor, hipStream_t s) {
  // cursor: 2 * kRouteMaxShards scratch words (cnt, cursor)
  (void)hipMemsetAsync(cursor, 0, sizeof(uint32_t) * 2 * kRouteMaxShards, s);
  const dim3 g = grid1(n, kT * kRoutePer);
  if (n) hipLaunchKernelGGL(k_route_count, g, dim3(kT), 0, s, keys, n, shards, cursor);
  hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(64), 0, s, cursor, shards, cursor + kRouteMaxShards, counts);
  if (n) hipLaunchKernelGGL(k_route_scatter, g, dim3(kT), 0, s, keys, n, shards, cursor + kRouteMaxShards, keys_out, perm);
}

__global__ void k_unpermute(const uint64_t* in, const uint32_t* perm,
                            uint64_t n, uint64_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[perm[i]] = in[i];
}
void launch_unpermute(const uint64_t* in, const uint32_t* perm, uint64_t n,
                      uint64_t* out, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_unpermute, grid1(n), dim3(kT), 0, s, in, perm, n, out);
}

// ---- batched range scan (intended Tree::range_query, Tree.cpp:461-540) ----
// One wave per query: descend to the leaf holding `from` (ballot child
// select), then follow sibling links while the leaf may hold keys <= to,
// collecting valid entries in slot order.  offsets == nullptr -> count only.
__global__ __launch_bounds__(kBlock) void k_range(
    const uint8_t* arena, uint64_t arena_bytes, uint16_t node, uint64_t root,
    const uint64_t* from, const uint64_t* to, uint64_t n, uint64_t* counts,
    const uint64_t* offsets, uint64_t* vals, uint32_t* err) {
  __shared__ __attribute__((aligned(16))) uint32_t s_page[kWavesPerBlock][kPageDwords + 8];
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  const uint64_t q = (uint64_t)blockIdx.x * kWavesPerBlock + wv;
  if (q >= n) return;
  uint32_t* lp = s_page[wv];
  const uint64_t lo = from[q], hi = to[q];
  uint64_t cnt = 0;
  uint64_t out = offsets ? offsets[q] : 0;
  if (lo <= hi) {
    uint64_t p = root;
    int hops = 0;
    // descend
    for (;;) {
      if (++hops > kMaxRounds || !ptr_ok(p, node, arena_bytes)) {
        if (lane == 0) atomicOr(err, kErrBadPtr);
        p = 0;
        break;
      }
      const u32x4 w = load_page_slice(arena, ga_offset(p));
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
    // scan leaves
    while (p) {
      if (++hops > (1 << 24) || !ptr_ok(p, node, arena_bytes)) {
        if (lane == 0) atomicOr(err, kErrBadPtr);
        break;
      }
      const u32x4 w = load_page_slice(arena, ga_offset(p));
      const Hdr h = parse_hdr(w);
      stage_page(lp, w);
      wave_lds_sync();
      const LeafEnt e = leaf_entry(lp, lane < kLeafCardinality ? lane : 0);
      const bool hit = lane < kLeafCardinality && e.val != kValueNull &&
                       (e.fraw & 0xF) == (e.rraw & 0xF) && e.key >= lo && e.key <= hi;
      const uint64_t m = ballot(hit);
      if (offsets && hit) vals[out + cnt + popc64(m & lanemask_lt())] = e.val;
      cnt += popc64(m);
      if (h.sibling == 0 || h.highest > hi) break;
      p = h.sibling;
      wave_lds_sync();
    }
  }
  if (lane == 0) counts[q] = cnt;
}
void launch_range_count(const uint8_t* arena, uint64_t arena_bytes,
                        uint16_t node, uint64_t root, const uint64_t* from,
                        const uint64_t* to, uint64_t n, uint64_t* counts,
                        const uint64_t* offsets, uint64_t* vals, uint32_t* err,
                        hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_range, grid1(n, kWavesPerBlock), dim3(kBlock), 0, s,
                     arena, arena_bytes, node, root, from, to, n, counts,
                     offsets, vals, err);
}

}  // namespace dev
}  // namespace shm
