// util.hip — batch bookkeeping kernels (segmentation with lock-ahead, tile
// scans, multi-GPU routing, key generation).
#include "device_common.h"
#include "kernels.h"
#include "upper_quick.h"
#include "seg_tile.h"

namespace shm {
namespace dev {

namespace {
constexpr int kT = 256;
inline dim3 grid1(uint64_t n, int per = kT) {
  return dim3((unsigned)((n + per - 1) / per));
}
}  // namespace

// n_dev (nullable): the device-side op count, n its upper bound
__device__ __forceinline__ uint64_t dev_n(const uint64_t* n_dev, uint64_t n) {
  return n_dev ? *n_dev : n;
}

// ---- two-launch tile scans ---------------------------------------------------
// A tile is kSegTile = 1024 elements, 4 consecutive per thread of a 256-thread
// block.  Pass 1 stores each tile's sum; pass 2 adds the sums of the tiles
// before it (<= n / 1024 words, read by the whole block) to a block scan.  No
// look-back state to initialise, no temp storage, two launches in all.
namespace {
constexpr int kScanPer = (int)kSegTile / kT;
static_assert(kScanPer * kT == (int)kSegTile, "tile shape");

// exclusive scan of v over the block's 256 threads; *total = the block sum
template <class T>
__device__ __forceinline__ T block_scan(T v, T* total) {
  __shared__ T ws[kT / kWave];
  T incl = v;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const T y = __shfl_up(incl, off);
    if (lane_id() >= off) incl += y;
  }
  const int w = threadIdx.x / kWave;
  if (lane_id() == kWave - 1) ws[w] = incl;
  __syncthreads();
  T base = 0, sum = 0;
#pragma unroll
  for (int i = 0; i < kT / kWave; ++i) {
    base += i < w ? ws[i] : T(0);
    sum += ws[i];
  }
  __syncthreads();
  *total = sum;
  return base + incl - v;
}

}  // namespace


// One launch: every 1024-op tile counts its staged heads, publishes the
// count in its tagged word (chunk tag << 32 | count), sums the words of the
// tiles before it (tile index = blockIdx, or a ticket when the tree passes a
// counter, lookback_index; tree.cpp lb_ctr says which and why), and fills its
// segments: seg_start / seg_page at each staged head, seg_end at its run's
// last op (the count of staged heads up to and including that op is the
// segment's position + 1).

__global__ __launch_bounds__(kT) void k_seg_fill(const uint64_t* page, uint64_t n,
                                                 const uint64_t* n_dev, uint64_t* lbw,
                                                 uint32_t* seg_start, uint32_t* seg_end,
                                                 uint64_t* seg_page, uint32_t* num_seg,
                                                 const uint8_t* pnew, uint32_t tag,
                                                 const uint32_t* any_new, uint32_t* err,
                                                 UpperArgs q, int has_q, uint32_t* ids,
                                                 uint32_t self_after, const uint64_t* ndel_src,
                                                 uint64_t* ndel_dst) {
  // the chunk's delete count into UpperCtl (k_upper's copy), before anything
  // of this chunk publishes its op buffers free (below, or k_upper)
  if (ndel_dst && blockIdx.x == 0 && threadIdx.x == 0) *ndel_dst = *ndel_src;
  if (any_new && *any_new != tag) {  // no op of this chunk marked a page (every block)
    if (blockIdx.x == 0) {
      if (threadIdx.x == 0) *num_seg = 0;
      if (has_q) seg_complete_unchanged(q);
    }
    return;
  }
  // the look-back's tile: a ticket, taken by every block past the check above
  const uint32_t b = lookback_index(ids);
  const uint64_t nv = dev_n(n_dev, n);
  if ((uint64_t)b * kSegTile >= nv) {  // past the device count (the grid covers n)
    if (nv == 0 && b == 0 && threadIdx.x == 0) *num_seg = 0;
    return;
  }
  segt::seg_tile(page, nv, b, lbw, seg_start, seg_end, seg_page, num_seg, pnew, tag, self_after);
}

void launch_segment(const uint64_t* page, uint64_t n, const uint64_t* n_dev, uint64_t* lbw,
                    uint32_t* seg_start, uint32_t* seg_end, uint64_t* seg_page,
                    uint32_t* num_seg, const uint8_t* pnew, uint32_t tag,
                    const uint32_t* any_new, uint32_t* err, hipStream_t s,
                    const UpperArgs* quick, uint32_t* ids, uint32_t self_after,
                    const uint64_t* ndel_src, uint64_t* ndel_dst) {
  const UpperArgs q = quick ? *quick : UpperArgs{};
  const int has_q = quick && any_new ? 1 : 0;
  // at least one block: block 0 copies the delete count even for no ops
  const uint64_t tiles = n ? seg_tiles(n) : 1;
  hipLaunchKernelGGL(k_seg_fill, dim3((unsigned)tiles), dim3(kT), 0, s, page, n, n_dev, lbw,
                     seg_start, seg_end, seg_page, num_seg, pnew, tag, any_new, err, q, has_q, ids,
                     self_after, ndel_src, ndel_dst);
}

// Exclusive scan of u64 counts in one launch: every 1024-element tile
// publishes its sum in a tagged word (tag << 48 | sum: a range scan's
// counts total < 2^48), sums the words of the tiles before it (as
// k_seg_fill) and writes its offsets; the thread holding n - 1 writes
// tot = {total, *err} (nullable).
__global__ __launch_bounds__(kT) void k_scan_u64(const uint64_t* in, uint64_t n, uint64_t* lbw,
                                                 uint32_t tag, uint64_t* out,
                                                 const uint32_t* err, uint64_t* tot,
                                                 uint32_t* err_out, uint32_t* ids) {
  __shared__ uint64_t s_pre[kT / kWave];
  const uint32_t b = lookback_index(ids);  // the tile
  const uint64_t i0 = (uint64_t)b * kSegTile + (uint64_t)threadIdx.x * kScanPer;
  uint64_t v[kScanPer], c = 0;
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    v[j] = i0 + j < n ? in[i0 + j] : 0;
    c += v[j];
  }
  uint64_t total;
  const uint64_t local = block_scan<uint64_t>(c, &total);
  constexpr uint64_t kMask = (1ull << 48) - 1;
  const uint64_t tg = (uint64_t)(tag & 0xFFFFu) << 48;
  if (threadIdx.x == 0)
    __hip_atomic_store(lbw + b, tg | (total & kMask), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t pre = 0;
  for (uint32_t x = threadIdx.x; x < b; x += kT) {
    uint64_t w = 0;
    for (uint32_t spin = 0;; ++spin) {
      w = __hip_atomic_load(lbw + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((w & ~kMask) == tg) break;
      if (spin > (1u << 24)) {
        atomicOr(err_out, kErrScanSpin);
        w = tg;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    pre += w & kMask;
  }
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) pre += __shfl_xor(pre, o);
  if (lane_id() == 0) s_pre[threadIdx.x / kWave] = pre;
  __syncthreads();
  uint64_t pos = local;
#pragma unroll
  for (int w = 0; w < kT / kWave; ++w) pos += s_pre[w];
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    if (i0 + j < n) out[i0 + j] = pos;
    pos += v[j];
    if (tot && i0 + j + 1 == n) {
      tot[0] = pos;
      tot[1] = *err;
    }
  }
}

void launch_scan_u64_total(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* lbw,
                           uint32_t tag, const uint32_t* err, uint64_t* tot, uint32_t* err_out,
                           uint32_t* ids, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_scan_u64, dim3((unsigned)seg_tiles(n)), dim3(kT), 0, s, in, n, lbw, tag, out,
                     err, tot, err_out, ids);
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

// keys[i] = to_key(ids[i]) for an arbitrary id array (zipf streams)
__global__ void k_hash_ids(const uint64_t* ids, uint64_t n, uint64_t keyspace,
                           uint64_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = cityhash64_u64(ids[i]) + 1;
  out[i] = keyspace ? h % keyspace : h;
}
void launch_hash_ids(const uint64_t* ids, uint64_t n, uint64_t keyspace, uint64_t* out,
                     hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_hash_ids, grid1(n), dim3(kT), 0, s, ids, n, keyspace, out);
}

// ---- multi-GPU routing: shard s owns [s*2^64/P, (s+1)*2^64/P) -------------
__device__ __forceinline__ uint32_t owner_of(uint64_t k, uint32_t shards) {
  return (uint32_t)__umul64hi(k, (uint64_t)shards);
}
constexpr int kRouteMaxShards = 64;
constexpr int kRoutePer = 4;  // keys per thread
constexpr int kRouteTile = kT * kRoutePer;

// Stable bucketing by owner (keys_out keeps input order inside each shard,
// which insert routing needs for last-writer-in-batch-order semantics):
//   count   : per-tile shard counts            -> cm[tile][shard]
//   scan    : per shard, exclusive over tiles  -> cm = tile bases, counts_out
//   scatter : per tile, ranks in index order from wave ballots
//   (keymax, nullable: a routed insert's batch -- a kKeyMax key sets the
//   flag, and the scan then rejects the batch whole: every count 0, the
//   error bit kErrKeyMax, as a local insert rejects its chunk)
__global__ __launch_bounds__(kT) void k_route_count(const uint64_t* __restrict__ keys,
                                                    uint64_t n, uint32_t shards,
                                                    uint32_t* __restrict__ cm,
                                                    uint32_t* keymax) {
  __shared__ uint32_t c[kRouteMaxShards];
  if (threadIdx.x < kRouteMaxShards) c[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kRouteTile;
  bool bad = false;
#pragma unroll
  for (int r = 0; r < kRoutePer; ++r) {
    const uint64_t i = base + (uint64_t)r * kT + threadIdx.x;
    if (i < n) {
      const uint64_t k = keys[i];
      bad |= k == kKeyMax;
      atomicAdd(&c[owner_of(k, shards)], 1u);
    }
  }
  if (keymax && ballot(bad) && lane_id() == 0) atomicOr(keymax, 1u);
  __syncthreads();
  if (threadIdx.x < shards) cm[(uint64_t)blockIdx.x * shards + threadIdx.x] = c[threadIdx.x];
}

__global__ __launch_bounds__(1024) void k_route_scan(uint32_t* __restrict__ cm, uint32_t tiles,
                                                     uint32_t shards,
                                                     uint64_t* __restrict__ counts_out,
                                                     uint32_t* keymax, uint32_t* err) {
  __shared__ uint32_t part[1024];
  __shared__ uint32_t off[kRouteMaxShards];
  const uint32_t t = threadIdx.x;
  const uint32_t Q = 1024 / shards;  // tile slices
  const uint32_t q = t / shards, sh = t % shards;
  const bool live = q < Q;
  const uint32_t b0 = live ? (uint32_t)(((uint64_t)tiles * q) / Q) : 0;
  const uint32_t b1 = live ? (uint32_t)(((uint64_t)tiles * (q + 1)) / Q) : 0;
  uint32_t sum = 0;
  for (uint32_t b = b0; b < b1; ++b) sum += cm[(uint64_t)b * shards + sh];
  if (live) part[q * shards + sh] = sum;
  __syncthreads();
  // per shard, inclusive scan of the slice sums over q (log2 Q steps)
  uint32_t incl = sum;
  for (uint32_t d = 1; d < Q; d <<= 1) {
    const uint32_t add = (live && q >= d) ? part[(q - d) * shards + sh] : 0u;
    __syncthreads();
    if (live) part[q * shards + sh] = (incl += add);
    __syncthreads();
  }
  if (live && q == Q - 1) off[sh] = incl;  // shard total for now
  __syncthreads();
  if (t == 0) {
    const bool reject = keymax && *keymax;
    if (reject) {
      *keymax = 0;
      atomicOr(err, kErrKeyMax);
    }
    uint32_t acc = 0;
    for (uint32_t x = 0; x < shards; ++x) {
      const uint32_t v = off[x];
      counts_out[x] = reject ? 0u : v;
      off[x] = acc;
      acc += v;
    }
  }
  __syncthreads();
  if (live) {
    uint32_t run = off[sh] + incl - sum;
    for (uint32_t b = b0; b < b1; ++b) {
      const uint64_t o = (uint64_t)b * shards + sh;
      const uint32_t v = cm[o];
      cm[o] = run;
      run += v;
    }
  }
}

__global__ __launch_bounds__(kT) void k_route_scatter(const uint64_t* __restrict__ keys,
                                                      uint64_t n, uint32_t shards,
                                                      const uint32_t* __restrict__ cm,
                                                      uint64_t* __restrict__ keys_out,
                                                      uint32_t* __restrict__ perm) {
  constexpr int kW = kT / kWave;
  __shared__ uint32_t wc[kRoutePer][kW][kRouteMaxShards];
  const int t = threadIdx.x, w = t >> 6, lane = lane_id();
  for (int j = t; j < kRoutePer * kW * kRouteMaxShards; j += kT) (&wc[0][0][0])[j] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kRouteTile;
  uint64_t kk[kRoutePer];
  uint32_t own[kRoutePer], rank[kRoutePer];
#pragma unroll
  for (int r = 0; r < kRoutePer; ++r) {
    const uint64_t i = base + (uint64_t)r * kT + t;
    const bool valid = i < n;
    kk[r] = valid ? keys[i] : 0;
    own[r] = valid ? owner_of(kk[r], shards) : ~0u;
    rank[r] = 0;
    uint64_t pending = ballot(valid);
    while (pending) {  // one pass per distinct owner in this wave
      const uint32_t o = rl32(own[r], ctz64(pending));
      const uint64_t m = ballot(own[r] == o);
      if (own[r] == o) rank[r] = popc64(m & lanemask_lt());
      if (lane == 0) wc[r][w][o] = popc64(m);
      pending &= ~m;
    }
  }
  __syncthreads();
  if ((uint32_t)t < shards) {  // index order = (round, wave, lane)
    uint32_t run = cm[(uint64_t)blockIdx.x * shards + t];
    for (int r = 0; r < kRoutePer; ++r)
      for (int x = 0; x < kW; ++x) {
        const uint32_t v = wc[r][x][t];
        wc[r][x][t] = run;
        run += v;
      }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRoutePer; ++r) {
    if (own[r] == ~0u) continue;
    const uint32_t o = wc[r][w][own[r]] + rank[r];
    keys_out[o] = kk[r];
    perm[o] = (uint32_t)(base + (uint64_t)r * kT + t);
  }
}

uint64_t route_scratch_words(uint64_t n_max) {
  return ((n_max + kRouteTile - 1) / kRouteTile) * kRouteMaxShards;
}

void launch_route_bucket(const uint64_t* keys, uint64_t n, uint32_t shards,
                         uint64_t* counts, uint64_t* keys_out, uint32_t* perm,
                         uint32_t* cm, uint32_t* keymax, uint32_t* err, hipStream_t s) {
  const uint32_t tiles = (uint32_t)((n + kRouteTile - 1) / kRouteTile);
  if (n)
    hipLaunchKernelGGL(k_route_count, dim3(tiles), dim3(kT), 0, s, keys, n, shards, cm, keymax);
  hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, s, cm, tiles, shards, counts, keymax,
                     err);
  if (n)
    hipLaunchKernelGGL(k_route_scatter, dim3(tiles), dim3(kT), 0, s, keys, n, shards,
                       (const uint32_t*)cm, keys_out, perm);
}

// out[i] = in[perm[i]] (apply the bucket permutation to a companion array)
__global__ void k_permute(const uint64_t* in, const uint32_t* perm, uint64_t n,
                          uint64_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[perm[i]];
}
void launch_permute(const uint64_t* in, const uint32_t* perm, uint64_t n, uint64_t* out,
                    hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_permute, grid1(n), dim3(kT), 0, s, in, perm, n, out);
}

// found (nullable): found[perm[i]] = in[i] != kValueNull (Tree.cpp:445-448)
__global__ void k_unpermute(const uint64_t* in, const uint32_t* perm,
                            uint64_t n, uint64_t* out, uint8_t* found) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const uint64_t v = in[i];
    const uint32_t p = perm[i];
    out[p] = v;
    if (found) found[p] = v != kValueNull ? 1 : 0;
  }
}
void launch_unpermute(const uint64_t* in, const uint32_t* perm, uint64_t n,
                      uint64_t* out, uint8_t* found, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_unpermute, grid1(n), dim3(kT), 0, s, in, perm, n, out, found);
}

// ---- fixed-capacity get exchange (shard.cpp): no host-known counts ------------
// Peer p's keys go to slot run [p * cap, (p + 1) * cap) of the send buffer,
// the rest of the run kKeyMax (a get of kKeyMax finds nothing).  A key's
// place in its run comes from a per-peer cursor (one atomic per peer present
// in a block), so no bucketing pass, scan or pack is needed; the order inside
// a run does not matter, since spos[i] records where input i went and the
// results are gathered back from the same places.  cursor[p] ends as the
// number of keys routed to peer p (a run's overflow included), cursor[P] as
// the number of overflowed keys.
// kKeyMax padding of the P runs of cap slots (run `own` in own_out when
// non-null) and the cursors zeroed
__global__ __launch_bounds__(kT) void k_route_fill(uint64_t* out, uint64_t cap, uint32_t* cursor,
                                                   uint32_t P, uint32_t own, uint64_t* own_out) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i == 0)
    for (uint32_t p = 0; p <= P; ++p) cursor[p] = 0;
  if (i >= (uint64_t)P * cap) return;
  const uint32_t p = (uint32_t)(i / cap);
  if (own_out && p == own)
    own_out[i - (uint64_t)p * cap] = kKeyMax;
  else
    out[i] = kKeyMax;
}

// A block of 1024 threads places 4096 keys (4 per thread): per round and
// wave, ranks among the lanes of one owner by ballots (as k_route_scatter);
// per owner, ONE global claim for the whole block.  Sixteen waves per block,
// four per SIMD (round 5's 256-thread blocks of 16 keys per thread left one
// wave per SIMD waiting on its loads and its block's claim).  The claim words
// sit on lines of their own (ctr, kCtrStride words apart): a returning
// device-scope atomic on one word saturates at ~88 per us (MI355X_MICROARCH
// "dequeue"), and the 2048 claims of a 2^20-key batch at P = 8 on one line
// took ~20 us (tools/route_p8.py); per line they are 256.  The last block
// to finish copies the counts to cursor[0..P] (P runs, then the overflow
// count: what the exchange and the host read) and returns the claim words
// to zero, so no launch resets them.
// A key past its run's capacity goes to the overflow list (ovk[j] = key,
// ovi[j] = its input position; one claim per wave and round) and the
// shard's second round returns its value (shard.cpp); without an overflow
// list (ovk == nullptr) it finds nothing and kErrOverflow is reported.
constexpr int kSlotT = 1024;

template <int kSlotPer>
__global__ __launch_bounds__(kSlotT) void k_route_slots(const uint64_t* __restrict__ keys,
                                                        uint64_t n, uint32_t P, uint64_t cap,
                                                        uint32_t* __restrict__ cursor,
                                                        uint32_t* __restrict__ ctr,
                                                        uint64_t* __restrict__ out,
                                                        uint32_t* __restrict__ spos, uint64_t* ovk,
                                                        uint32_t* ovi, uint32_t* err, uint32_t own_p,
                                                        uint64_t* own_out) {
  constexpr int kW = kSlotT / kWave;
  constexpr int kSlotTile = kSlotT * kSlotPer;
  __shared__ uint32_t wc[kSlotPer][kW][kRouteMaxShards];
  __shared__ uint32_t last;
  const int t = threadIdx.x, w = t >> 6, lane = lane_id();
  for (int j = t; j < kSlotPer * kW * kRouteMaxShards; j += kSlotT) (&wc[0][0][0])[j] = 0;
  const uint64_t base = (uint64_t)blockIdx.x * kSlotTile;
  uint64_t kk[kSlotPer];
#pragma unroll
  for (int r = 0; r < kSlotPer; ++r) {
    const uint64_t i = base + (uint64_t)r * kSlotT + t;
    kk[r] = i < n ? keys[i] : 0;
  }
  __syncthreads();
  // ranks among the wave's lanes of one owner from the owner's bit planes:
  // one ballot per bit (3 at P = 8), each lane keeping the lanes that agree
  // with its owner on every bit, and lane o < P the lanes whose owner is o
  // (its count).  A pass per owner present in the wave (readlane, ballot,
  // LDS store per pass) took 5-6 of the kernel's 12.4 us at P = 8
  // (tools/route_p8.py, the passes skipped: 6.8 us)
  const int nb = P > 1 ? 32 - __clz((int)(P - 1)) : 0;
  uint32_t own[kSlotPer], rank[kSlotPer];
#pragma unroll
  for (int r = 0; r < kSlotPer; ++r) {
    const bool valid = base + (uint64_t)r * kSlotT + t < n;
    own[r] = valid ? owner_of(kk[r], P) : ~0u;
    const uint64_t vm = ballot(valid);
    uint64_t mine = vm, mine_o = vm;
    for (int b = 0; b < nb; ++b) {
      const uint64_t bb = ballot(valid && ((own[r] >> b) & 1u));
      mine &= ((own[r] >> b) & 1u) ? bb : ~bb;
      mine_o &= ((lane >> b) & 1) ? bb : ~bb;
    }
    rank[r] = valid ? popc64(mine & lanemask_lt()) : 0u;
    if ((uint32_t)lane < P) wc[r][w][lane] = popc64(mine_o);
  }
  __syncthreads();
  // one wave per owner: its 64 (round, wave) counts scanned across the
  // lanes, the block's one claim on the owner's run, the bases written back
  // (a thread per owner summing them in turn spent ~3 us in LDS latency)
  constexpr int kQ = kSlotPer * kW;  // (round, wave) counts per owner
  static_assert(kQ < kWave || kQ % kWave == 0, "whole lanes per (round, wave)");
  constexpr int kE = kQ >= kWave ? kQ / kWave : 1;  // per lane
  for (uint32_t p = (uint32_t)w; p < P; p += kW) {
    uint32_t v[kE], sum = 0;
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      const int q = lane * kE + e;
      v[e] = q < kQ ? wc[q / kW][q % kW][p] : 0u;
      sum += v[e];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)incl, off);
      if (lane >= off) incl += y;
    }
    const uint32_t tot = rl32(incl, kWave - 1);
    uint32_t run = 0;
    if (lane == 0 && tot) run = atomicAdd(ctr + p * kCtrStride, tot);
    run = rl32(run, 0) + incl - sum;
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      const int q = lane * kE + e;
      if (q < kQ) wc[q / kW][q % kW][p] = run;
      run += v[e];
    }
  }
  __syncthreads();
  bool over = false;
#pragma unroll
  for (int r = 0; r < kSlotPer; ++r) {
    const uint64_t i = base + (uint64_t)r * kSlotT + t;
    bool ov = false;
    if (own[r] != ~0u) {
      const uint32_t pos = wc[r][w][own[r]] + rank[r];
      if (pos < cap) {
        const uint64_t x = (uint64_t)own[r] * cap + pos;
        if (own_out && own[r] == own_p)
          own_out[pos] = kk[r];  // this rank's run: straight to the local get
        else
          out[x] = kk[r];
        spos[i] = (uint32_t)x;
      } else {  // this peer's run is full
        spos[i] = ~0u;
        ov = true;
      }
    }
    const uint64_t om = ballot(ov);  // wave-uniform
    if (om && ovk) {
      uint32_t ob = 0;
      if (lane == 0) ob = atomicAdd(ctr + P * kCtrStride, (uint32_t)popc64(om));
      ob = rl32(ob, 0);
      if (ov) {
        const uint32_t j = ob + (uint32_t)popc64(om & lanemask_lt());
        ovk[j] = kk[r];
        ovi[j] = (uint32_t)i;
      }
    }
    over |= ov;
  }
  if (over && !ovk) atomicOr(err, kErrOverflow);
  // every claim of this block returned: the last block publishes the counts
  __syncthreads();
  if (t == 0) last = atomicAdd(ctr + (P + 1) * kCtrStride, 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (last && (uint32_t)t <= P + 1) {
    // read and reset in one atomic, at the point every claim went through
    const uint32_t v = atomicExch(ctr + t * kCtrStride, 0u);
    if ((uint32_t)t <= P) cursor[t] = v;
  }
}

// fill: pad the runs with kKeyMax first (a slot's first batch, or one whose
// capacity changed); otherwise the runs' tails keep the keys an earlier
// batch placed there at the same capacity -- keys of the same owner's
// range, searched and never gathered, exactly as padding.  ctr: (P + 2) *
// kCtrStride words, zero at rest (route_ctr_words)
void launch_route_slots(const uint64_t* keys, uint64_t n, uint32_t P, uint64_t cap,
                        uint32_t* cursor, uint32_t* ctr, uint64_t* out, uint32_t* spos,
                        uint64_t* ovk, uint32_t* ovi, uint32_t* err, hipStream_t s, uint32_t own,
                        uint64_t* own_out, bool fill) {
  const uint64_t slots = (uint64_t)P * cap;
  if (fill)
    hipLaunchKernelGGL(k_route_fill, grid1(slots + 1), dim3(kT), 0, s, out, cap, cursor, P, own,
                       own_out);
  // four keys per thread: 256 blocks for 2^20 keys (one or two keys per
  // thread, or eight, measured no better at P = 8: tools/route_p8.py)
  if (n)
    hipLaunchKernelGGL(k_route_slots<4>, grid1(n, kSlotT * 4), dim3(kSlotT), 0, s, keys, n, P,
                       cap, cursor, ctr, out, spos, ovk, ovi, err, own, own_out);
  else if (!fill)
    (void)hipMemsetAsync(cursor, 0, sizeof(uint32_t) * (P + 1), s);
}

// out[i] = in[spos[i]] (0 for a key cut by a full run: the overflow round
// fills it afterwards), found[i] = out[i] != 0 (Tree.cpp:445-448).  Four
// inputs per thread when the buffers allow 16 B accesses: one spos load, four
// gathers in flight, two 16 B value stores and one 4 B found store
__device__ __forceinline__ uint64_t gather_one(const uint64_t* in, uint32_t x, uint64_t own_lo,
                                               uint64_t cap, const uint64_t* own_src) {
  if (x == ~0u) return kValueNull;
  return own_src && x - own_lo < cap ? own_src[x] : in[x];
}
__global__ void k_route_gather(const uint64_t* in, const uint32_t* spos, uint64_t n,
                               uint64_t* out, uint8_t* found, uint64_t own_lo, uint64_t cap,
                               const uint64_t* own_src) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t v = gather_one(in, spos[i], own_lo, cap, own_src);
  out[i] = v;
  if (found) found[i] = v != kValueNull ? 1 : 0;
}
__global__ void k_route_gather4(const uint64_t* in, const uint32_t* spos, uint64_t n4,
                                uint64_t* out, uint8_t* found, uint64_t own_lo, uint64_t cap,
                                const uint64_t* own_src) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n4) return;
  const uint4 x = reinterpret_cast<const uint4*>(spos)[j];
  const uint64_t v0 = gather_one(in, x.x, own_lo, cap, own_src);
  const uint64_t v1 = gather_one(in, x.y, own_lo, cap, own_src);
  const uint64_t v2 = gather_one(in, x.z, own_lo, cap, own_src);
  const uint64_t v3 = gather_one(in, x.w, own_lo, cap, own_src);
  ulonglong2* o = reinterpret_cast<ulonglong2*>(out) + 2 * j;
  o[0] = make_ulonglong2(v0, v1);
  o[1] = make_ulonglong2(v2, v3);
  if (found)
    reinterpret_cast<uint32_t*>(found)[j] = (v0 != kValueNull ? 1u : 0u) |
                                            (v1 != kValueNull ? 1u << 8 : 0u) |
                                            (v2 != kValueNull ? 1u << 16 : 0u) |
                                            (v3 != kValueNull ? 1u << 24 : 0u);
}
void launch_route_gather(const uint64_t* in, const uint32_t* spos, uint64_t n, uint64_t* out,
                         uint8_t* found, hipStream_t s, uint32_t own, uint64_t cap,
                         const uint64_t* own_src) {
  if (!n) return;
  const uint64_t lo = (uint64_t)own * cap;
  const bool vec = ((reinterpret_cast<uintptr_t>(spos) | reinterpret_cast<uintptr_t>(out)) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(found) & 3) == 0;
  const uint64_t n4 = vec ? n / 4 : 0;
  if (n4)
    hipLaunchKernelGGL(k_route_gather4, grid1(n4), dim3(kT), 0, s, in, spos, n4, out, found, lo,
                       cap, own_src);
  if (n > 4 * n4)
    hipLaunchKernelGGL(k_route_gather, grid1(n - 4 * n4), dim3(kT), 0, s, in, spos + 4 * n4,
                       n - 4 * n4, out + 4 * n4, found ? found + 4 * n4 : nullptr, lo, cap,
                       own_src);
}

// the overflow round's results: out[ovi[perm[j]]] = in[j] (perm: the
// overflow list's bucketing permutation), found likewise
__global__ void k_route_ov_scatter(const uint64_t* in, const uint32_t* perm, const uint32_t* ovi,
                                   uint64_t m, uint64_t* out, uint8_t* found) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint32_t i = ovi[perm[j]];
  const uint64_t v = in[j];
  out[i] = v;
  if (found) found[i] = v != kValueNull ? 1 : 0;
}
void launch_route_ov_scatter(const uint64_t* in, const uint32_t* perm, const uint32_t* ovi,
                             uint64_t m, uint64_t* out, uint8_t* found, hipStream_t s) {
  if (m)
    hipLaunchKernelGGL(k_route_ov_scatter, grid1(m), dim3(kT), 0, s, in, perm, ovi, m, out, found);
}

// Routed insert: the stably bucketed keys (and values) of peer p, run
// [sum(cnt[< p]), + cnt[p]), packed into slot run [p * cap, (p + 1) * cap):
// the first min(cnt[p], cap) in bucket (= input) order, the rest kKeyMax
// padding (the receiver's insert skips it).  The overflow (cnt[p] > cap)
// stays in kb / vb for the shard's second round.
__global__ __launch_bounds__(kT) void k_route_pack(const uint64_t* kb, const uint64_t* vb,
                                                   const uint64_t* cnt, uint32_t P, uint64_t cap,
                                                   uint64_t* pk, uint64_t* pv, uint32_t own,
                                                   uint64_t* own_k, uint64_t* own_v) {
  const uint64_t x = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (x >= (uint64_t)P * cap) return;
  const uint32_t p = (uint32_t)(x / cap);
  const uint64_t j = x - (uint64_t)p * cap;
  uint64_t off = 0;
  for (uint32_t q = 0; q < p; ++q) off += cnt[q];
  const bool real = j < cnt[p];
  const bool mine = own_k && p == own;  // this rank's run: straight to the local insert
  (mine ? own_k + j : pk + x)[0] = real ? kb[off + j] : kKeyMax;
  (mine ? own_v + j : pv + x)[0] = real ? vb[off + j] : kValueNull;
}
void launch_route_pack(const uint64_t* kb, const uint64_t* vb, const uint64_t* cnt, uint32_t P,
                       uint64_t cap, uint64_t* pk, uint64_t* pv, hipStream_t s, uint32_t own,
                       uint64_t* own_k, uint64_t* own_v) {
  const uint64_t slots = (uint64_t)P * cap;
  if (slots)
    hipLaunchKernelGGL(k_route_pack, grid1(slots), dim3(kT), 0, s, kb, vb, cnt, P, cap, pk, pv,
                       own, own_k, own_v);
}

// ---- routed range scans (shard.cpp shm_shard_range_query) -------------------
// Piece (p, j) of the P x cap piece matrix = scan j's overlap with shard p,
// [max(from, lo_p), min(to, hi_p)], or empty (1, 0) where it misses the shard
// (or j >= n); row p goes to rank p.  bnd: shard p owns [bnd[p], bnd[p + 1]),
// bnd[P] = 0 standing for 2^64.
__global__ __launch_bounds__(kT) void k_range_pieces(const uint64_t* from, const uint64_t* to,
                                                     uint64_t n, uint64_t cap, uint32_t P,
                                                     ShardBounds bnd, uint64_t* plo,
                                                     uint64_t* phi) {
  const uint64_t x = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (x >= (uint64_t)P * cap) return;
  const uint32_t p = (uint32_t)(x / cap);
  const uint64_t j = x - (uint64_t)p * cap;
  uint64_t lo = 1, hi = 0;
  if (j < n) {
    const uint64_t f = from[j], t = to[j];
    const uint64_t slo = bnd.b[p];
    const uint64_t shi = p + 1 < P ? bnd.b[p + 1] - 1 : kKeyMax;  // inclusive top
    if (f <= t && f <= shi && t >= slo) {
      lo = f > slo ? f : slo;
      hi = t < shi ? t : shi;
    }
  }
  plo[x] = lo;
  phi[x] = hi;
}
void launch_range_pieces(const uint64_t* from, const uint64_t* to, uint64_t n, uint64_t cap,
                         uint32_t P, const ShardBounds& bnd, uint64_t* plo, uint64_t* phi,
                         hipStream_t s) {
  const uint64_t m = (uint64_t)P * cap;
  if (m) hipLaunchKernelGGL(k_range_pieces, grid1(m), dim3(kT), 0, s, from, to, n, cap, P, bnd, plo, phi);
}

// Sums after the counts came back: blocks [0, P) sum row r of rc (the values
// this rank, as scanner, sends rank r) into rw[r]; blocks [P, 2P) row p of
// bc (the values it receives from shard p) into rw[P + p]; the rest give
// counts[j] = sum over p of bc[p][j] for j < n (scan j's total).
__global__ __launch_bounds__(kT) void k_range_sums(const uint64_t* rc, const uint64_t* bc,
                                                   uint64_t n, uint64_t cap, uint32_t P,
                                                   uint64_t* rw, uint64_t* counts) {
  const uint32_t b = blockIdx.x;
  if (b < 2 * P) {
    const uint64_t* row = (b < P ? rc : bc) + (uint64_t)(b % P) * cap;
    uint64_t v = 0;
    for (uint64_t j = threadIdx.x; j < cap; j += kT) v += row[j];
    uint64_t tot;
    (void)block_scan<uint64_t>(v, &tot);
    if (threadIdx.x == 0) rw[b] = tot;
    return;
  }
  const uint64_t j = (uint64_t)(b - 2 * P) * kT + threadIdx.x;
  if (j >= n) return;
  uint64_t c = 0;
  for (uint32_t p = 0; p < P; ++p) c += bc[(uint64_t)p * cap + j];
  counts[j] = c;
}
void launch_range_sums(const uint64_t* rc, const uint64_t* bc, uint64_t n, uint64_t cap,
                       uint32_t P, uint64_t* rw, uint64_t* counts, hipStream_t s) {
  const uint32_t blocks = 2 * P + (uint32_t)((n + kT - 1) / kT);
  hipLaunchKernelGGL(k_range_sums, dim3(blocks), dim3(kT), 0, s, rc, bc, n, cap, P, rw, counts);
}

// Scan j's values, in shard order (= key order across shards): piece (p, j)
// holds bc[p][j] values at bv[bsc[p][j]] (bsc: exclusive scan of bc in
// row-major order, the layout of the received value runs; pitch != 0: row
// p's run starts at bv[p * pitch] and holds at most pitch values, the
// exchange without a host read-back); they go to vals[offsets[j] + sum of
// its earlier pieces], values past vals_cap dropped.  One wave per scan.
__global__ __launch_bounds__(kT) void k_range_assemble(const uint64_t* bv, const uint64_t* bc,
                                                       const uint64_t* bsc, uint64_t n,
                                                       uint64_t cap, uint32_t P,
                                                       const uint64_t* offsets, uint64_t* vals,
                                                       uint64_t vals_cap, uint64_t pitch) {
  const uint64_t j = ((uint64_t)blockIdx.x * kT + threadIdx.x) / kWave;
  if (j >= n) return;
  const int lane = lane_id();
  uint64_t dst = offsets[j];
  for (uint32_t p = 0; p < P; ++p) {
    const uint64_t c = bc[(uint64_t)p * cap + j];
    const uint64_t x = bsc[(uint64_t)p * cap + j];
    // pitched: the piece's place inside row p's run, cut at the run's end
    const uint64_t rel = pitch ? x - bsc[(uint64_t)p * cap] : 0;
    const uint64_t src = pitch ? (uint64_t)p * pitch + rel : x;
    const uint64_t cc = pitch ? (rel >= pitch ? 0 : c < pitch - rel ? c : pitch - rel) : c;
    for (uint64_t k = (uint64_t)lane; k < cc; k += kWave)
      if (dst + k < vals_cap) vals[dst + k] = bv[src + k];
    dst += c;
  }
}
void launch_range_assemble(const uint64_t* bv, const uint64_t* bc, const uint64_t* bsc,
                           uint64_t n, uint64_t cap, uint32_t P, const uint64_t* offsets,
                           uint64_t* vals, uint64_t vals_cap, hipStream_t s, uint64_t pitch) {
  if (n)
    hipLaunchKernelGGL(k_range_assemble, grid1(n * kWave), dim3(kT), 0, s, bv, bc, bsc, n, cap, P,
                       offsets, vals, vals_cap, pitch);
}

// The routed scan's value exchange without a host read-back: the scanner's
// packed values (row p = the values for rank p's scans, rw[p] of them, rows
// in order) copied to fixed runs of pitch values per peer, sent whole.  Block
// 0 also writes the batch's status for the caller: status[0] = its scans'
// total (rw[2P + 2]), status[1] = flags (1: a run to or from a peer passed
// pitch, 2: the scan pass dropped values past its buffer, 4: total > vals_cap,
// 8: a device error word of the scans).  Grid-stride copy, rows by blockIdx.y.
__global__ __launch_bounds__(kT) void k_range_pitch(const uint64_t* rvals, const uint64_t* rw,
                                                    uint32_t P, uint64_t pitch, uint64_t* out,
                                                    uint64_t rvcap, uint64_t vals_cap,
                                                    uint64_t* status) {
  const uint32_t p = blockIdx.y;
  uint64_t off = 0;
  for (uint32_t q = 0; q < p; ++q) off += rw[q];
  const uint64_t c = rw[p] < pitch ? rw[p] : pitch;
  for (uint64_t k = (uint64_t)blockIdx.x * kT + threadIdx.x; k < c; k += (uint64_t)gridDim.x * kT)
    if (off + k < rvcap) out[(uint64_t)p * pitch + k] = rvals[off + k];
  if (p == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
    uint64_t f = 0;
    for (uint32_t q = 0; q < P; ++q)
      if (rw[q] > pitch || rw[P + q] > pitch) f |= 1;
    if (rw[2 * P] > rvcap) f |= 2;
    if (rw[2 * P + 2] > vals_cap) f |= 4;
    if (rw[2 * P + 1] || rw[2 * P + 3] || rw[2 * P + 5]) f |= 8;
    status[0] = rw[2 * P + 2];
    status[1] = f;
  }
}
void launch_range_pitch(const uint64_t* rvals, const uint64_t* rw, uint32_t P, uint64_t pitch,
                        uint64_t* out, uint64_t rvcap, uint64_t vals_cap, uint64_t* status,
                        hipStream_t s) {
  uint64_t bx = (pitch + kT - 1) / kT;
  if (bx > 64) bx = 64;
  if (bx == 0) bx = 1;
  hipLaunchKernelGGL(k_range_pitch, dim3((unsigned)bx, P), dim3(kT), 0, s, rvals, rw, P, pitch,
                     out, rvcap, vals_cap, status);
}

// ---- Tree::lock_bench (src/Tree.cpp:310-321): take and release the lock word
// of each key, lock[CityHash64(key) % num_locks], as try_lock_addr /
// unlock_addr do (Tree.cpp:205-264) on the HBM lock table: a word is free
// when it holds <= tag (the epoch tags of the insert chunks, insert.hip),
// taken as tag | 1 by atomicCAS, released by storing tag.  Lanes of one wave
// that share a word take it in turn (a lane releases in the iteration it
// acquired, so the wave never waits on itself).  Spins are bounded.
__global__ __launch_bounds__(kT) void k_lock_bench(const uint64_t* keys, uint64_t n,
                                                   uint64_t* locks, uint32_t num_locks,
                                                   uint64_t tag, uint32_t* err) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  bool done = i >= n;
  unsigned long long* w = nullptr;
  if (!done)
    w = reinterpret_cast<unsigned long long*>(locks) + cityhash64_u64(keys[i]) % num_locks;
  const unsigned long long mine = (unsigned long long)(tag | 1ull);
  for (uint32_t spin = 0; spin < kMaxLockSpins; ++spin) {
    if (!done) {
      const unsigned long long cur = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur <= (unsigned long long)tag && atomicCAS(w, cur, mine) == cur) {
        __hip_atomic_store(w, (unsigned long long)tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        done = true;
      }
    }
    if (!ballot(!done)) return;
    __builtin_amdgcn_s_sleep(1);
  }
  if (!done) atomicOr(err, kErrLock);
}
void launch_lock_bench(const uint64_t* keys, uint64_t n, uint64_t* locks, uint32_t num_locks,
                       uint64_t tag, uint32_t* err, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_lock_bench, grid1(n), dim3(kT), 0, s, keys, n, locks, num_locks, tag, err);
}

// ---- diagnostics: a window marker for profiles (shm__mark) -------------------
// One empty wave whose dispatch names a window's edge in a kernel trace or a
// counter collection (tools/fold_roofline.py keeps the dispatches between
// tag 1 and tag 2).
__global__ void k_mark(uint32_t tag) { (void)tag; }
void launch_mark(uint32_t tag, hipStream_t s) {
  hipLaunchKernelGGL(k_mark, dim3(1), dim3(kWave), 0, s, tag);
}

// ---- diagnostics: a kernel that holds CUs (shm__hog) -----------------------------
// Each block declares a whole CU's LDS (160 KiB), so no other block that uses
// LDS fits its CU while it runs, and spins on the 100 MHz wall clock until
// `ticks` have passed since it started (bounded: every wave leaves).  n
// blocks therefore take n CUs away from the kernels of other streams for that
// long (tests/test_gpu_parity.py::test_split_insert_beside_cu_hog).
constexpr uint32_t kHogLdsWords = 160 * 1024 / 4;
__global__ __launch_bounds__(kWave) void k_hog(uint64_t ticks, uint32_t* sink) {
  __shared__ uint32_t s_pad[kHogLdsWords];
  s_pad[threadIdx.x] = threadIdx.x;
  const uint64_t t0 = wall_clock64();
  uint32_t spins = 0;
  while (wall_clock64() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
    ++spins;
  }
  // keep the LDS array alive; never true for a real run (spins > 0)
  if (spins == 0xFFFFFFFFu) sink[0] = s_pad[(threadIdx.x * 7) % kHogLdsWords];
}
void launch_hog(uint32_t n, uint64_t ticks, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_hog, dim3(n), dim3(kWave), 0, s, ticks, nullptr);
}

}  // namespace dev
}  // namespace shm
