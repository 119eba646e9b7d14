// isort.hip — ordering of an insert batch: sorted by key, one op per key
// (the last writer in batch order), as Tree::insert applied op after op
// leaves it (src/Tree.cpp:353-403, 878-889: a later insert of a key
// overwrites the earlier one).
//
//   1. k_tile_dedup   every 2048-op tile: an LDS hash table keeps each key's
//                     last op (atomic max of the op index), and the tile's
//                     survivors are compacted to its front (gcount).  Heavy
//                     hitters (zipf) shrink to one op per tile here.
//   2. coarse pass    partition.hip: 256 bins by the top 8 bits of the key's
//                     offset in the shard range, carrying the op index.
//   3. k_bin_unique   every bin: last writer per key, sorted (below); a bin
//                     over 6144 ops (clustered keys) is sorted by the same
//                     block with a stable LSD radix sort through global
//                     scratch, so every batch is ordered on the device.  The
//                     bin then finds its place among the bins (tagged count
//                     words, bin_prefix) and writes its survivors straight
//                     to uk / uv / dk.
#include "device_common.h"
#include "kernels.h"

namespace shm {
namespace dev {

namespace {

constexpr int kIT = 1024;  // threads per block

__device__ __forceinline__ bool pair_gt(uint64_t ka, uint32_t ia, uint64_t kb, uint32_t ib) {
  return ka > kb || (ka == kb && ia > ib);
}

// ascending bitonic sort of size `m` (power of two, <= capacity) in LDS
template <int PER>
__device__ __forceinline__ void lds_bitonic(uint64_t* key, uint32_t* idx, uint32_t m) {
  const int t = threadIdx.x;
  for (uint32_t k = 2; k <= m; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int r = 0; r < PER / 2; ++r) {
        const uint32_t p = (uint32_t)(r * kIT + t);  // pair index
        if (p < (m >> 1)) {
          const uint32_t i = 2 * j * (p / j) + (p % j);
          const uint32_t l = i + j;
          const bool up = (i & k) == 0;
          const uint64_t a = key[i], b = key[l];
          const uint32_t x = idx[i], y = idx[l];
          if (pair_gt(a, x, b, y) == up) {
            key[i] = b;
            key[l] = a;
            idx[i] = y;
            idx[l] = x;
          }
        }
      }
      __syncthreads();
    }
  }
}

// exclusive block scan of one u32 per thread (kIT threads)
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int t = threadIdx.x, l = lane_id(), w = t >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, off);
    if (l >= off) incl += y;
  }
  if (l == kWave - 1) wsum[w] = incl;
  __syncthreads();
  uint32_t base = 0, all = 0;
  for (int x = 0; x < kIT / kWave; ++x) {
    base += x < w ? wsum[x] : 0;
    all += wsum[x];
  }
  *total = all;
  __syncthreads();
  return base + incl - v;
}

}  // namespace

__global__ __launch_bounds__(kIT) void k_tile_dedup(const uint64_t* __restrict__ keys, uint64_t n,
                                                   uint64_t* __restrict__ keys_out,
                                                   uint32_t* __restrict__ idx_out,
                                                   uint32_t* __restrict__ gcount,
                                                   uint32_t* err, uint32_t* gate, uint32_t tag,
                                                   KeyRange kr, uint32_t* __restrict__ M,
                                                   uint32_t* __restrict__ S,
                                                   uint32_t* __restrict__ Mx, int skip_pad) {
  // LDS hash table of the tile's distinct keys: slot -> (key, 1 + last index)
  constexpr int kSlots = 2 * kIsortTile;
  constexpr int PER = kIsortTile / kIT;
  constexpr int SPT = kSlots / kIT;  // slots per thread in the compaction
  __shared__ unsigned long long hkey[kSlots];
  __shared__ uint32_t hidx[kSlots];
  __shared__ uint32_t wsum[kIT / kWave];
  __shared__ uint32_t hist[kCoarse];  // the coarse pass's tile histogram (M != nullptr)
  const int t = threadIdx.x;
  if (t < kCoarse) hist[t] = 0;
  const uint64_t base = (uint64_t)blockIdx.x * kIsortTile;
#pragma unroll
  for (int r = 0; r < SPT; ++r) {
    hkey[r * kIT + t] = kKeyMax;  // empty (kKeyMax is never a stored key)
    hidx[r * kIT + t] = 0;
  }
  __syncthreads();
  bool bad = false;
  uint64_t kin[PER];  // both keys requested before the first probe
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const uint64_t i = base + (uint64_t)(r * kIT + t);
    kin[r] = i < n ? keys[i] : kKeyMax;
  }
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const uint64_t i = base + (uint64_t)(r * kIT + t);
    if (i >= n) continue;
    const uint64_t k = kin[r];
    if (k == kKeyMax) {
      // kKeyMax cannot be stored (root highest is exclusive, Tree.h:150);
      // a routed insert's slot padding (skip_pad) is no op at all
      if (!skip_pad) bad = true;
      continue;
    }
    uint32_t h = (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> 50) & (kSlots - 1);
    for (int probe = 0; probe < kSlots; ++probe) {
      const unsigned long long o = atomicCAS(&hkey[h], (unsigned long long)kKeyMax,
                                             (unsigned long long)k);
      if (o == kKeyMax || o == k) {
        atomicMax(&hidx[h], (uint32_t)i + 1u);  // the last writer in batch order
        break;
      }
      h = (h + 1) & (kSlots - 1);
    }
  }
  if (bad) {
    // the chunk is rejected whole (k_bin_unique emits nothing) and reported
    atomicOr(err, kErrKeyMax);
    atomicCAS(err + 1, 0u, tag);  // the first chunk with an error names itself
    *gate = tag;
  }
  __syncthreads();
  if (Mx) {
    // Tile mode: the survivors sorted by coarse bin (a counting sort in LDS),
    // bin b's run of this tile at keys_out[tile base + Mx[tile][b] ...] with
    // M[tile][b] keys.  k_bin_unique gathers its bin's runs from every tile,
    // so no coarse scatter pass moves the survivors once more.
    __shared__ uint32_t lex[kCoarse];
    uint64_t kk[SPT];
    uint32_t ii[SPT], bn[SPT], rk[SPT];
#pragma unroll
    for (int r = 0; r < SPT; ++r) {
      kk[r] = hkey[SPT * t + r];
      ii[r] = hidx[SPT * t + r] - 1u;
      bn[r] = kk[r] != kKeyMax ? coarse_of(kk[r], kr) : 0u;
      rk[r] = kk[r] != kKeyMax ? atomicAdd(&hist[bn[r]], 1u) : 0u;
    }
    __syncthreads();
    const uint32_t c = t < kCoarse ? hist[t] : 0u;
    uint32_t total;
    const uint32_t ex = block_scan(c, wsum, &total);  // ends with a barrier
    if (t < kCoarse) {
      // bin-major ([bin][tile]): k_bin_unique reads its bin's row whole
      lex[t] = ex;
      M[(uint64_t)t * kMaxTiles + blockIdx.x] = c;
      Mx[(uint64_t)t * kMaxTiles + blockIdx.x] = ex;
      if (c) atomicAdd(&S[(blockIdx.x / 16) * kCoarse + t], c);
    }
    __syncthreads();  // lex set; every slot read into registers
#pragma unroll
    for (int r = 0; r < SPT; ++r)
      if (kk[r] != kKeyMax) {
        const uint32_t p = lex[bn[r]] + rk[r];
        hkey[p] = kk[r];
        hidx[p] = ii[r];
      }
    __syncthreads();
    for (uint32_t j = (uint32_t)t; j < total; j += kIT) {  // contiguous stores
      keys_out[base + j] = hkey[j];
      idx_out[base + j] = hidx[j];
    }
    if (t == 0) gcount[blockIdx.x] = total;
    return;
  }
  uint32_t keep = 0;
#pragma unroll
  for (int r = 0; r < SPT; ++r) keep += hkey[SPT * t + r] != kKeyMax ? 1u : 0u;
  uint32_t total;
  uint32_t pos = block_scan(keep, wsum, &total);
#pragma unroll
  for (int r = 0; r < SPT; ++r) {
    const uint64_t k = hkey[SPT * t + r];
    if (k != kKeyMax) {
      keys_out[base + pos] = k;
      idx_out[base + pos] = hidx[SPT * t + r] - 1u;
      ++pos;
      if (M) atomicAdd(&hist[coarse_of(k, kr)], 1u);
    }
  }
  if (t == 0) gcount[blockIdx.x] = total;
  if (M) {
    // this tile is one coarse-pass tile (batches of <= 256 tiles): its
    // histogram and group sums, as k_part_coarse_hist would write them
    __syncthreads();
    if (t < kCoarse) {
      const uint32_t c = hist[t];
      M[(uint64_t)blockIdx.x * kCoarse + t] = c;
      if (c) atomicAdd(&S[(blockIdx.x / 16) * kCoarse + t], c);
    }
  }
}

// ---- step 3 + 4 without the library scan: per-bin dedup, sort, emit --------
//
// k_bin_unique, one block per coarse bin (<= kUniqCap ops):
//   a. LDS hash table of the bin's keys keeping each key's last op (atomic
//      max of the op index); a key lives in exactly one bin, so the
//      survivors are the batch's last writers (Tree.cpp:878-889 applied in
//      batch order leaves exactly these);
//   b. counting sort of the survivors by the next 8 key bits (the bin's
//      keys share the top 8 bits of their offset in the shard range): the
//      op that claims a key's slot in a. takes the key's rank in its
//      sub-bucket, b. places the claimed keys at sub-bucket base + rank;
//   c. each survivor's place inside its sub-bucket by rank: the number of
//      the sub-bucket's keys below its own (keys are unique after a.; the
//      sub-bucket's keys are LDS broadcast reads for the lanes that share
//      it), its value fetched from `vals` meanwhile into LDS at that place.
//      A sub-bucket > 64 (skewed keys) sorts the whole bin with the LDS
//      bitonic network instead (values then fetched in d.);
//   d. each survivor's value classifies it as an upsert or a delete (value 0
//      = kValueNull, Tree.cpp:881); local ranks by one block scan.
// The bin's (upserts, deletes) give its place among the bins (bin_prefix),
// and its survivors go straight to uk / uv (upserts, key order) and dk
// (deletes); the last bin writes the totals to counts[0..1].
constexpr int kUniqSlots = 8192;  // LDS hash slots (96 KB with the op indices)
constexpr int kUniqCap = 6144;    // ops per bin handled here (load <= 0.75)
constexpr int kUniqPer = kUniqCap / kIT;


// ---- bins over kUniqCap ops: the same result through global scratch ---------
// Stable LSD radix sort of the bin's (key, op index) pairs by 8-bit digits,
// one block, ping-ponging between the bin's slots of keys1 / pay1 and the
// same slots of the scratch arrays; digits on which every key agrees are
// skipped (clustered keys need few passes).  Equal keys stay in op-index
// order (the input holds at most one op per key per 2048-op tile, tiles in
// order), so the last of each run is the batch's last writer.  Survivors
// are then compacted to the bin's front with their ranks, as in the LDS path.
// ldsw: >= 8 x 256 + 16 x 256 + 256 + 16 words of LDS.
__device__ void big_bin_unique(uint64_t* __restrict__ keys1, uint32_t* __restrict__ pay1,
                               uint64_t* __restrict__ kscr, uint32_t* __restrict__ iscr,
                               uint32_t start, uint32_t cnt, const uint64_t* __restrict__ vals,
                               uint32_t* __restrict__ lrank, uint32_t* cnt2,
                               uint32_t* ldsw) {
  constexpr int kW = kIT / kWave;  // 16 waves
  uint32_t* h8 = ldsw;                  // [8][256] digit histograms
  uint32_t* wc = ldsw + 8 * 256;        // [16][256] per-wave digit counts
  uint32_t* base = wc + kW * 256;       // [256] running digit offsets
  uint32_t* wsum = base + 256;          // [16]
  const int t = threadIdx.x, w = t >> 6;
  for (int j = t; j < 8 * 256; j += kIT) h8[j] = 0;
  __syncthreads();
  for (uint32_t e = (uint32_t)t; e < cnt; e += kIT) {
    const uint64_t k = keys1[start + e];
#pragma unroll
    for (int d = 0; d < 8; ++d) atomicAdd(&h8[d * 256 + ((k >> (8 * d)) & 255)], 1u);
  }
  __syncthreads();
  uint64_t* ka = keys1 + start;
  uint32_t* ia = pay1 + start;
  uint64_t* kb = kscr + start;
  uint32_t* ib = iscr + start;
  for (int d = 0; d < 8; ++d) {
    // skip a digit every key shares (block-uniform after the barrier)
    const uint32_t hv = t < 256 ? h8[d * 256 + t] : 0u;
    if (__syncthreads_or(hv == cnt)) continue;
    uint32_t tot;
    const uint32_t ex = block_scan(hv, wsum, &tot);
    if (t < 256) base[t] = ex;
    __syncthreads();
    for (uint32_t c0 = 0; c0 < cnt; c0 += kIT) {
      for (int j = t; j < kW * 256; j += kIT) wc[j] = 0;
      __syncthreads();
      const uint32_t e = c0 + (uint32_t)t;
      const bool valid = e < cnt;
      const uint64_t k = valid ? ka[e] : 0;
      const uint32_t ix = valid ? ia[e] : 0;
      const uint32_t dg = (uint32_t)(k >> (8 * d)) & 255u;
      // lanes of this wave holding the same digit: rank among them in lane order
      uint64_t m = ballot(valid);
#pragma unroll
      for (int bit = 0; bit < 8; ++bit) {
        const uint64_t on = ballot(valid && ((dg >> bit) & 1u));
        m &= ((dg >> bit) & 1u) ? on : ~on;
      }
      const uint32_t rk = (uint32_t)popc64(m & lanemask_lt());
      if (valid && rk == 0) wc[w * 256 + dg] = (uint32_t)popc64(m);
      __syncthreads();
      if (t < 256) {  // digit t: offsets of its elements per wave, in wave order
        uint32_t run = base[t];
        for (int x = 0; x < kW; ++x) {
          const uint32_t v = wc[x * 256 + t];
          wc[x * 256 + t] = run;
          run += v;
        }
        base[t] = run;
      }
      __syncthreads();
      if (valid) {
        const uint32_t p = wc[w * 256 + dg] + rk;
        kb[p] = k;
        ib[p] = ix;
      }
      __syncthreads();
    }
    uint64_t* tk = ka;
    ka = kb;
    kb = tk;
    uint32_t* ti = ia;
    ia = ib;
    ib = ti;
  }
  // survivors (last of each run of equal keys) compacted to keys1 / pay1 at
  // the bin's front; ranks among upserts / deletes (bit 31)
  uint32_t ru = 0, rd = 0, rs = 0;
  for (uint32_t c0 = 0; c0 < cnt; c0 += kIT) {
    const uint32_t e = c0 + (uint32_t)t;
    const bool valid = e < cnt;
    const uint64_t k = valid ? ka[e] : 0;
    const uint32_t ix = valid ? ia[e] : 0;
    const bool surv = valid && (e + 1 == cnt || ka[e + 1] != k);
    const bool del = surv && vals[ix] == kValueNull;
    uint32_t tu, td, ts;
    const uint32_t xu = block_scan(surv && !del ? 1u : 0u, wsum, &tu);
    const uint32_t xd = block_scan(del ? 1u : 0u, wsum, &td);
    const uint32_t xs = block_scan(surv ? 1u : 0u, wsum, &ts);
    // every read of this tile is done: positions < c0 + kIT, later tiles
    // read from c0 + kIT on
    __syncthreads();
    if (surv) {
      keys1[start + rs + xs] = k;
      pay1[start + rs + xs] = ix;
      lrank[start + rs + xs] = del ? (0x80000000u | (rd + xd)) : (ru + xu);
    }
    ru += tu;
    rd += td;
    rs += ts;
    __syncthreads();
  }
  if (t == 0) {
    cnt2[0] = ru;
    cnt2[1] = rd;
  }
  __syncthreads();
}

// Bin b's place among the bins: publish its (upserts, deletes) in its
// tagged word (chunk tag << 48 | upserts << 24 | deletes), then wave 0 waits
// for the words of bins < b and sums them (the last bin sums all of them into
// counts[0..1]).  b is the block's ticket (lookback_index): a bin waits only
// on bins taken before it by running blocks, whatever else holds the CUs.
__device__ void bin_prefix(uint64_t* lbw, uint32_t b, uint32_t tag, uint32_t ups, uint32_t dels,
                           uint32_t* red, uint32_t& bu, uint32_t& bd, uint64_t* counts,
                           uint32_t* err) {
  const uint64_t tg = (uint64_t)(tag & 0xFFFFu);
  if (threadIdx.x == 0)
    __hip_atomic_store(lbw + b, (tg << 48) | ((uint64_t)ups << 24) | dels, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < (unsigned)kWave) {
    const uint32_t lane = threadIdx.x;
    const bool last = b == (uint32_t)kCoarse - 1;
    const uint32_t lim = last ? (uint32_t)kCoarse : b;
    uint64_t su = 0, sd = 0, tu = 0, td = 0;
    for (uint32_t i = lane; i < lim; i += kWave) {
      uint64_t w = 0;
      for (uint32_t spin = 0;; ++spin) {
        w = __hip_atomic_load(lbw + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((w >> 48) == tg) break;
        if (spin > (1u << 24)) {
          atomicOr(err, kErrBinSpin);
          w = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      const uint64_t u = (w >> 24) & 0xFFFFFFu, d = w & 0xFFFFFFu;
      if (i < b) {
        su += u;
        sd += d;
      }
      tu += u;
      td += d;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      su += __shfl_xor(su, o);
      sd += __shfl_xor(sd, o);
      tu += __shfl_xor(tu, o);
      td += __shfl_xor(td, o);
    }
    if (lane == 0) {
      red[0] = (uint32_t)su;
      red[1] = (uint32_t)sd;
      if (last) {
        counts[0] = tu;
        counts[1] = td;
      }
    }
  }
  __syncthreads();
  bu = red[0];
  bd = red[1];
  __syncthreads();
}

__global__ __launch_bounds__(kIT) void k_bin_unique(uint64_t* __restrict__ keys1,
                                                   uint32_t* __restrict__ pay1,
                                                   const uint32_t* __restrict__ bins,
                                                   KeyRange kr,
                                                   const uint64_t* __restrict__ vals,
                                                   uint32_t* __restrict__ lrank,
                                                   uint64_t* __restrict__ lbw,
                                                   uint64_t* __restrict__ kscr,
                                                   uint32_t* __restrict__ iscr,
                                                   uint64_t* __restrict__ uk,
                                                   uint64_t* __restrict__ uv,
                                                   uint64_t* __restrict__ dk,
                                                   uint64_t* __restrict__ counts,
                                                   uint32_t* __restrict__ err,
                                                   uint32_t* __restrict__ S,
                                                   const uint32_t* gate, uint32_t tag,
                                                   uint64_t* __restrict__ stamps,
                                                   TileRuns tr, uint32_t* ids) {
  constexpr int SPT = kUniqSlots / kIT;  // hash slots per thread
  __shared__ unsigned long long hkey[kUniqSlots];  // hash, then the sorted keys
  __shared__ uint32_t hidx[kUniqSlots];            // 1 + op index, then op index
  __shared__ uint64_t hval[kUniqCap];               // the survivors' values in key order (c.)
  __shared__ uint32_t hist[kFine];
  __shared__ uint32_t wsum[kIT / kWave];
  __shared__ uint32_t s_big;
  __shared__ uint32_t s_cnt2[2];
  // tile mode: this bin's run in every tile (prefix of the run lengths over
  // the tiles, and where each run starts in the tiles' output)
  __shared__ uint32_t s_tpre[kMaxTiles + 1];
  __shared__ uint32_t s_tbase[kMaxTiles];
  const int t = threadIdx.x;
  const uint32_t b = lookback_index(ids);  // the bin (bin_prefix waits on smaller ones)
  const uint32_t tiles = tr.tiles;
  // the coarse pass is complete: clear its group sums for the next batch
  // (tile mode: the last bin, once every bin has read them, bin_prefix)
  if (b == 0 && !tiles)
    for (int j = t; j < kPartGroupWords; j += kIT) S[j] = 0;
  if (*gate == tag) {  // rejected chunk (kKeyMax): nothing to apply
    if (b == 0 && t == 0) counts[0] = counts[1] = 0;
    if (tiles && b == (uint32_t)kCoarse - 1)
      for (int j = t; j < kPartGroupWords; j += kIT) S[j] = 0;
    return;
  }
  // diagnostic phase clock (shm__upper_stamps): stamps[p * kCoarse + b]
  auto bstamp = [&](int p) {
    if (stamps && t == 0) stamps[p * kCoarse + b] = wall_clock64();
  };
  bstamp(0);
  uint32_t start = 0, cnt = 0;
  if (tiles) {
    const uint32_t c = (uint32_t)t < tiles ? tr.M[(uint64_t)b * kMaxTiles + t] : 0u;
    const uint32_t bx = (uint32_t)t < tiles ? tr.Mx[(uint64_t)b * kMaxTiles + t] : 0u;
    const uint32_t ex = block_scan(c, wsum, &cnt);  // ends with a barrier
    if ((uint32_t)t < tiles) {
      s_tpre[t] = ex;
      s_tbase[t] = (uint32_t)t * (uint32_t)kIsortTile + bx;
    }
    if (t == 0) s_tpre[tiles] = cnt;
    __syncthreads();
  } else {
    start = bins[2 * b];
    cnt = bins[2 * b + 1];
  }
  // tile mode: where bin element o lies in the tiles' output (the tile whose
  // run holds it: the last tile with prefix <= o, a binary search in LDS)
  auto src_of = [&](uint32_t o) -> uint32_t {
    uint32_t lo = 0, hi = tiles;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_tpre[mid] <= o)
        lo = mid;
      else
        hi = mid;
    }
    return s_tbase[lo] + (o - s_tpre[lo]);
  };
  if (cnt > (uint32_t)kUniqCap) {  // block-uniform
    if (tiles) {
      // the bin's own contiguous range of keys1 / pay1: its start is the sum
      // of the bins before it (the tiles' group sums S), then a copy
      uint32_t v = 0;
      if ((uint32_t)t < b)
        for (int g = 0; g < kPartGroupWords / kCoarse; ++g) v += S[g * kCoarse + t];
      uint32_t bt;
      (void)block_scan(v, wsum, &bt);
      start = bt;
      for (uint32_t o = (uint32_t)t; o < cnt; o += kIT) {
        const uint32_t q = src_of(o);
        keys1[start + o] = tr.keys[q];
        pay1[start + o] = tr.idx[q];
      }
      __threadfence_block();
      __syncthreads();
    }
    big_bin_unique(keys1, pay1, kscr, iscr, start, cnt, vals, lrank, s_cnt2,
                   reinterpret_cast<uint32_t*>(hkey));
    uint32_t bu, bd;
    bin_prefix(lbw, b, tag, s_cnt2[0], s_cnt2[1], wsum, bu, bd, counts, err);
    if (tiles && b == (uint32_t)kCoarse - 1)  // every bin has read S (bin_prefix)
      for (int j = t; j < kPartGroupWords; j += kIT) S[j] = 0;
    const uint32_t u = s_cnt2[0] + s_cnt2[1];
    for (uint32_t o = (uint32_t)t; o < u; o += kIT) {
      const uint32_t r = lrank[start + o];
      const uint64_t k = keys1[start + o];
      if (r & 0x80000000u) {
        dk[bd + (r & 0x7FFFFFFFu)] = k;
      } else {
        uk[bu + r] = k;
        uv[bu + r] = vals[pay1[start + o]];
      }
    }
    return;
  }
  // a. last writer per key
#pragma unroll
  for (int r = 0; r < SPT; ++r) {
    hkey[r * kIT + t] = kKeyMax;  // kKeyMax is never a stored key
    hidx[r * kIT + t] = 0;
  }
  if (t < kFine) hist[t] = 0;
  if (t == 0) s_big = 0;
  __syncthreads();
  // the op that claims a key's slot also takes the key's rank in its fine
  // sub-bucket, so b. touches only the claimed slots
  uint64_t ck[kUniqPer];
  uint32_t ch[kUniqPer], cr[kUniqPer];
  // every element's (key, op index) requested before the first hash probe:
  // one memory round trip, not one per element (the LDS atomics below keep
  // the compiler from moving later loads above them)
  uint64_t lk[kUniqPer];
  uint32_t li[kUniqPer];
#pragma unroll
  for (int r = 0; r < kUniqPer; ++r) {
    const uint32_t o = (uint32_t)(r * kIT + t);
    lk[r] = kKeyMax;
    li[r] = 0;
    if (o < cnt) {
      const uint32_t q = tiles ? src_of(o) : start + o;
      lk[r] = tiles ? tr.keys[q] : keys1[q];
      li[r] = tiles ? tr.idx[q] : pay1[q];
    }
  }
#pragma unroll
  for (int r = 0; r < kUniqPer; ++r) {
    ch[r] = ~0u;
    ck[r] = 0;
    cr[r] = 0;
    const uint32_t o = (uint32_t)(r * kIT + t);
    if (o >= cnt) continue;
    const uint64_t k = lk[r];
    const uint32_t ix = li[r];
    uint32_t h = (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> 51) & (kUniqSlots - 1);
    for (int probe = 0; probe < kUniqSlots; ++probe) {
      const unsigned long long old = atomicCAS(&hkey[h], (unsigned long long)kKeyMax,
                                               (unsigned long long)k);
      if (old == kKeyMax) {
        ch[r] = h;
        ck[r] = k;
        cr[r] = atomicAdd(&hist[fine_of(k, kr)], 1u);
      }
      if (old == kKeyMax || old == k) {
        atomicMax(&hidx[h], ix + 1u);
        break;
      }
      h = (h + 1) & (kUniqSlots - 1);
    }
  }
  __syncthreads();
  bstamp(1);
  // b. survivors placed by fine digit: sub-bucket base + the claim's rank
  const uint32_t hc = t < kFine ? hist[t] : 0u;
  if (hc > 64) s_big = 1;
  uint32_t u;
  const uint32_t hex = block_scan(hc, wsum, &u);  // ends with a barrier
  if (t < kFine) hist[t] = hex;
  uint32_t ci[kUniqPer];
#pragma unroll
  for (int r = 0; r < kUniqPer; ++r) ci[r] = ch[r] != ~0u ? hidx[ch[r]] - 1u : 0u;
  __syncthreads();  // every claimed slot read (and hist scanned) before the moves
#pragma unroll
  for (int r = 0; r < kUniqPer; ++r) {
    if (ch[r] != ~0u) {
      const uint32_t p = hist[fine_of(ck[r], kr)] + cr[r];
      hkey[p] = ck[r];
      hidx[p] = ci[r];
    }
  }
  __syncthreads();
  bstamp(2);
  // c. finish the order
  if (!s_big) {
    constexpr int RP = (kUniqCap + kIT - 1) / kIT;
    uint64_t mk[RP], mv[RP];
    uint32_t mi[RP], dst[RP];
#pragma unroll
    for (int r = 0; r < RP; ++r) {
      const uint32_t p = (uint32_t)(r * kIT + t);
      mk[r] = kKeyMax;
      mv[r] = 0;
      mi[r] = 0;
      dst[r] = 0;
      if (p < u) {
        mk[r] = hkey[p];
        mi[r] = hidx[p];
        mv[r] = vals[mi[r]];  // in flight during the rank loop
      }
    }
#pragma unroll
    for (int r = 0; r < RP; ++r) {
      const uint32_t p = (uint32_t)(r * kIT + t);
      if (p < u) {
        const uint32_t d = fine_of(mk[r], kr);
        const uint32_t bs = hist[d], be = d + 1 < (uint32_t)kFine ? hist[d + 1] : u;
        uint32_t rank = 0;
        for (uint32_t q = bs; q < be; ++q) rank += hkey[q] < mk[r] ? 1u : 0u;
        dst[r] = bs + rank;
      }
    }
    __syncthreads();  // every rank read before the first move
#pragma unroll
    for (int r = 0; r < RP; ++r) {
      if ((uint32_t)(r * kIT + t) < u) {
        hkey[dst[r]] = mk[r];
        hidx[dst[r]] = mi[r];
        hval[dst[r]] = mv[r];
      }
    }
    __syncthreads();
  } else {
    uint32_t m = 2;
    while (m < u) m <<= 1;
    for (uint32_t o = u + (uint32_t)t; o < m; o += kIT) {
      hkey[o] = kKeyMax;
      hidx[o] = ~0u;
    }
    __syncthreads();
    lds_bitonic<kUniqSlots / kIT>(reinterpret_cast<uint64_t*>(hkey), hidx, m);
  }
  bstamp(3);
  // d. classify and rank: thread t owns survivors [E t, E t + E); then the
  // bin's place among the bins, and its survivors straight to uk / uv / dk
  constexpr int E = (kUniqCap + kIT - 1) / kIT;
  const uint32_t o0 = (uint32_t)(E * t);
  uint32_t isdel = 0, nloc = 0;  // bit r: survivor o0 + r is a delete
  uint64_t ok[E], ov[E];
#pragma unroll
  for (int r = 0; r < E; ++r) {
    const uint32_t o = o0 + (uint32_t)r;
    ok[r] = 0;
    ov[r] = 0;
    if (o < u) {
      ok[r] = hkey[o];
      ov[r] = s_big ? vals[hidx[o]] : hval[o];
      if (ov[r] == kValueNull) isdel |= 1u << r;
      ++nloc;
    }
  }
  const uint32_t ndl = (uint32_t)__builtin_popcount(isdel);
  // one scan of (upserts << 16 | deletes): a bin holds <= 6144 survivors
  uint32_t tot;
  const uint32_t ex = block_scan(((nloc - ndl) << 16) | ndl, wsum, &tot);
  bstamp(4);
  uint32_t bu, bd;
  bin_prefix(lbw, b, tag, tot >> 16, tot & 0xFFFF, wsum, bu, bd, counts, err);
  if (tiles && b == (uint32_t)kCoarse - 1)  // every bin has read S (bin_prefix)
    for (int j = t; j < kPartGroupWords; j += kIT) S[j] = 0;
  bstamp(5);
  uint32_t ru = bu + (ex >> 16), rd = bd + (ex & 0xFFFF);
#pragma unroll
  for (int r = 0; r < E; ++r) {
    const uint32_t o = o0 + (uint32_t)r;
    if (o < u) {
      if ((isdel >> r) & 1u) {
        dk[rd++] = ok[r];
      } else {
        uk[ru] = ok[r];
        uv[ru++] = ov[r];
      }
    }
  }
  bstamp(6);
}

void launch_tile_dedup(const uint64_t* keys, uint64_t n, uint64_t* keys_out, uint32_t* idx_out,
                       uint32_t* gcount, uint32_t* err, uint32_t* gate, uint32_t tag,
                       uint64_t key_lo, uint32_t key_bits, uint32_t* M, uint32_t* S,
                       uint32_t* Mx, int skip_pad, hipStream_t s) {
  if (!n) return;
  const uint64_t tiles = (n + kIsortTile - 1) / kIsortTile;
  if (tiles > (uint64_t)kMaxTiles) M = S = Mx = nullptr;  // the coarse pass counts for itself
  if (!M || !S) Mx = nullptr;
  hipLaunchKernelGGL(k_tile_dedup, dim3((unsigned)tiles), dim3(kIT), 0, s, keys, n, keys_out,
                     idx_out, gcount, err, gate, tag, KeyRange{key_lo, key_bits}, M, S, Mx,
                     skip_pad);
}

void launch_bin_unique(uint64_t* keys1, uint32_t* pay1, const uint32_t* bins, uint64_t key_lo,
                       uint32_t key_bits, const uint64_t* vals, uint32_t* lrank, uint64_t* lbw,
                       uint64_t* kscr, uint32_t* iscr, uint64_t* uk, uint64_t* uv, uint64_t* dk,
                       uint64_t* counts, uint32_t* err, uint32_t* S, const uint32_t* gate,
                       uint32_t tag, uint64_t* stamps, const TileRuns& tr, uint32_t* ids,
                       hipStream_t s) {
  const KeyRange kr{key_lo, key_bits};
  hipLaunchKernelGGL(k_bin_unique, dim3(kCoarse), dim3(kIT), 0, s, keys1, pay1, bins, kr, vals,
                     lrank, lbw, kscr, iscr, uk, uv, dk, counts, err, S, gate, tag, stamps, tr,
                     ids);
}

}  // namespace dev
}  // namespace shm
