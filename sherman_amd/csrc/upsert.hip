// upsert.hip — in-place leaf upserts of a segmented insert batch, four
// segments per wave: the no-split branch of Tree::insert's leaf_page_store
// (src/Tree.cpp:828-920).
//
// The batch's sorted unique keys are grouped into segments, one per target
// leaf, and every segment's lock word lock[CityHash64(page) % num_locks] (the
// reference's on-chip lock word, Tree.cpp:832-842, 205-242) is taken with an
// epoch tag in the same round trip as the page's DMA.  A wave takes G = 4
// consecutive segments:
//   * stage: the G pages by LDS-DMA with their lock words
//     (lock_and_read_page, Tree.cpp:851-852), checked with check_consistent
//     (front == rear, Tree.cpp:857) and the fences of every key.
//   * apply: lane group q (16 lanes x 4 consecutive entries) holds slot q's
//     54 entries.  For each op of segment q in key order the valid slot
//     holding the key is overwritten, else the first empty slot is taken;
//     f_version++ and r_version = f_version, 4-bit (Tree.cpp:878-912).
//   * write back only the changed 18 B entries (the reference writes the
//     entry, not the page: write_page_and_unlock(update_addr, ...),
//     Tree.cpp:915-920); the words are released when the chunk retires.
// Overwrites of keys a page holds were applied in place by k_locate (oslot
// bit 31); the segment list holds only pages that get a new key
// (launch_segment), and a segment skips the overwrites in its op loop.
// A segment whose page would reach 54 entries (the split point,
// Tree.cpp:914) is left untouched and flagged seg_P = ceil(T / 36) for the
// k-way split of insert.hip (k_upper), which also learns here how many new
// pages each of its block ranges needs (UpperCtl.leaf_np / leaf_ns).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "device_common.h"
#include "kernels.h"
#include "lds_dma.h"
#include "leaf_chunk.h"

namespace shm {
namespace dev {

namespace {

}  // namespace

// Apply one group of G staged pages (buf: G x 1 KB in LDS; slot s = lanes
// [s L, s L + L)): versions and fences, the segment's ops in key order with
// the reference's slot rule, the changed entries written back, and the
// segment's split plan (seg_T / seg_P / seg_newpages / seg_ver).  page / pok
// are valid in lanes s < G; qst / qen / pk / pv per slot group.  Returns the
// error bits.
template <int G>
__device__ __forceinline__ uint32_t apply_group(const SegArgs& a, const uint32_t* buf,
                                                uint64_t g0, uint32_t num_seg, uint64_t page,
                                                bool pok, bool locked, uint32_t qst,
                                                uint32_t qen, uint64_t pk, uint64_t pv,
                                                uint32_t po) {
  constexpr int L = kWave / G;                       // lanes per page
  constexpr int E = (kLeafCardinality + L - 1) / L;  // entries per lane
  constexpr int CD = kLeafEntry * E / 4;             // dwords per lane chunk
  constexpr uint64_t kGroupMask = L == 64 ? ~0ull : ((1ull << (L & 63)) - 1);
  const int lane = lane_id();
  const int q = lane / L;
  const int li = lane % L;
  uint32_t err = 0;
  // ---- per slot q: header, entries ---------------------------------------------
  const uint32_t* hp = buf + q * kPageDwords;
  const uint32_t h2 = hp[2], h3 = hp[3], h4 = hp[4], h7 = hp[7], h8 = hp[8], h9 = hp[9],
                 h10 = hp[10], z = hp[kOffLeafRear / 4];
  const uint64_t leftmost = (uint64_t)((h2 >> 8) | (h3 << 24)) |
                            ((uint64_t)((h3 >> 8) | (h4 << 24)) << 32);
  const uint32_t fver = h2 & 0xFF;
  const uint64_t lowest = (uint64_t)h7 | ((uint64_t)h8 << 32);
  const uint64_t highest = (uint64_t)h9 | ((uint64_t)h10 << 32);
  const bool qpok = (shfl32(pok ? 1u : 0u, q) != 0) && locked;  // buf slot q holds it
  const bool cons = leftmost == 0 && fver == (z & 0xFF);
  if (ballot(qpok && !cons)) err |= kErrInconsistent;
  const uint64_t qpage = shfl64(page, q);
  bool live = qpok && cons;
  const uint32_t nops = live ? qen - qst : 0u;

  const int ebase = chunk_base<E>(li);
  uint32_t D[CD];
  {
    const uint32_t* ep = hp + (kOffRecords + kLeafEntry * ebase) / 4;
#pragma unroll
    for (int i = 0; i < CD; ++i) D[i] = ep[i];
  }
  uint64_t ek[E], ev[E];
  uint32_t ef[E], er[E];
  chunk_entries<E>(D, ek, ev, ef, er);
  bool mine[E], valid[E], dirty[E], fresh[E];  // fresh: a new key took the slot
  uint32_t cnt = 0;  // valid entries of slot q (the same in all its lanes)
#pragma unroll
  for (int j = 0; j < E; ++j) {
    mine[j] = ebase + j >= li * E;
    valid[j] = mine[j] && ev[j] != kValueNull;
    dirty[j] = false;
    fresh[j] = false;
    cnt += (uint32_t)popc64((ballot(valid[j]) >> (q * L)) & kGroupMask);
  }

  // ---- entries after the batch T = valid + new keys.  More than 53 ops can
  // never stay in place (T >= ops): count their hits by binary search, as the
  // plan kernel did, and skip the per-op loop; smaller segments count while
  // applying and discard the result if the page would fill ------------------------
  const bool big = nops > (uint32_t)(kLeafCardinality - 1);
  uint32_t T = cnt;
  if (ballot(big)) {
    uint32_t hits = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) {
      bool h = false;
      if (big && valid[j]) {
        const uint64_t x = lower_bound64(a.op_key, qst, qen, ek[j]);
        h = x < qen && a.op_key[x] == ek[j];
      }
      hits += (uint32_t)popc64((ballot(h) >> (q * L)) & kGroupMask);
    }
    if (big) T = cnt + nops - hits;
  }
  const uint32_t nloop = big ? 0u : nops;

  // ---- apply the ops in key order -------------------------------------------------
  bool bad = false;
  for (uint32_t t = 0; ballot(t < nloop); ++t) {
    const bool act = t < nloop && !bad;
    const int src = q * L + (t < (uint32_t)L ? (int)t : L - 1);
    const uint64_t sk = shfl64(pk, src), sv = shfl64(pv, src);
    const uint32_t so = shfl32(po, src);
    // an op k_locate applied in place: its key is already valid in the page
    const bool done = (t < (uint32_t)L ? so : (act ? a.oslot[qst + t] : 0u)) >> 31;
    const uint64_t kq = act ? (t < (uint32_t)L ? sk : a.op_key[qst + t]) : 0;
    const uint64_t vq = act ? (t < (uint32_t)L ? sv : a.op_val[qst + t]) : 0;
    if (ballot(act && done) == ballot(act)) continue;  // wave-uniform
    if (act && !done && (kq < lowest || kq >= highest)) bad = true;  // not this page's key
    const bool go = act && !bad && !done;
    int hj = -1;
#pragma unroll
    for (int j = E - 1; j >= 0; --j)
      if (valid[j] && ek[j] == kq) hj = j;
    const uint64_t mh = (ballot(go && hj >= 0) >> (q * L)) & kGroupMask;
    bool take = false;
    const bool isnew = go && !mh;
    int tj = -1;
    if (go && mh) {
      take = li == ctz64(mh);  // the valid slot holding the key
      tj = hj;
    } else if (go) {
      T += 1;  // a new key: the first empty slot (one exists while T <= 53)
      int fj = -1;
#pragma unroll
      for (int j = E - 1; j >= 0; --j)
        if (mine[j] && !valid[j]) fj = j;
      const uint64_t me = (ballot(fj >= 0) >> (q * L)) & kGroupMask;
      if (me) {
        take = li == ctz64(me);  // the first empty slot
        tj = fj;
      }
    }
#pragma unroll
    for (int j = 0; j < E; ++j) {
      if (take && tj == j) {
        ek[j] = kq;
        ev[j] = vq;
        const uint32_t f = ((ef[j] & 0xF) + 1) & 0xF;
        ef[j] = (ef[j] & 0xF0) | f;
        er[j] = (er[j] & 0xF0) | f;
        valid[j] = true;
        dirty[j] = true;
        fresh[j] = fresh[j] || isnew;
      }
    }
  }
  if (ballot(bad)) err |= kErrPlan;
  live = live && !bad;
  const bool over = T > (uint32_t)(kLeafCardinality - 1);

  // ---- write back the changed entries of in-place segments -----------------------
  if (live && !over) {
    uint8_t* pg = a.arena + ga_offset(qpage);
#pragma unroll
    for (int j = 0; j < E; ++j)
      if (dirty[j]) {
        put_leaf_entry(reinterpret_cast<uint32_t*>(pg), ebase + j, ek[j], ev[j], ef[j], er[j]);
        // the leaf summary: an overwrite keeps its key's fingerprint; a new
        // key in an empty slot sets it (one partial line write per page
        // that gained keys, none for pure updates)
        if (fresh[j]) set_leaf_fp(a.sum, ga_offset(qpage), ebase + j, ek[j]);
      }
  }
  if (a.leaf_hw) {
    // the page's occupancy bound after the batch: 1 + its last valid slot
    uint32_t hw = 0;
#pragma unroll
    for (int j = 0; j < E; ++j)
      if (valid[j]) hw = (uint32_t)(ebase + j + 1);
#pragma unroll
    for (int m = L / 2; m > 0; m >>= 1) {
      const uint32_t o = (uint32_t)__shfl_xor((int)hw, m);
      hw = o > hw ? o : hw;
    }
    if (live && !over && li == 0) a.leaf_hw[ga_offset(qpage) >> 10] = (uint8_t)hw;
  }
  const uint64_t gq = g0 + (uint64_t)q;
  const uint32_t P = (live && over) ? (T + kLeafSplitFill - 1) / kLeafSplitFill : 1u;
  if (li == 0 && q < G && gq < num_seg) {
    a.seg_T[gq] = live ? T : 0u;
    a.seg_P[gq] = P;
    a.seg_newpages[gq] = P - 1;
    a.seg_ver[gq] = live ? fver : ~0u;
    if (P > 1) {
      // k_upper block range of this segment (insert.hip block_range)
      const uint32_t r = (uint32_t)((gq * a.up_nb) / num_seg);
      atomicAdd(&a.ctl->leaf_np[a.par][r], P - 1);
      atomicAdd(&a.ctl->leaf_ns[a.par][r], 1u);
      if (P > kSmallSplit) atomicAdd(&a.ctl->leaf_nb[a.par][r], P - 1);
    }
  }
  return err;
}

// Software-pipelined: a grid of about one resident wave set; each wave loops
// over groups
// w, w + W, ... and, while it applies group g from one LDS buffer, the pages
// of group g + W are already landing in the other (LDS-DMA) and the segment
// records of g + 2W and the ops of g + W are in flight.  Per group the wave
// then pays about the apply time instead of two dependent HBM round trips.
template <int G>
__global__ __launch_bounds__(kBlock) void k_leaf_upsert_pipe(SegArgs a) {
  constexpr int L = kWave / G;
  __shared__ __attribute__((aligned(16))) uint32_t s_pg[kWavesPerBlock * 2 * G * kPageDwords];
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  const uint64_t W = (uint64_t)gridDim.x * kWavesPerBlock;
  const uint64_t w = (uint64_t)blockIdx.x * kWavesPerBlock + (uint64_t)wv;
  const uint32_t num_seg = *a.num_seg_dev;
  const uint64_t ngroups = ((uint64_t)num_seg + G - 1) / G;
  uint64_t g = w;
  if (g >= ngroups) return;  // wave-uniform
  const uint32_t* bufs = &s_pg[wv * 2 * G * kPageDwords];
  const uint32_t bufs_lds = lds_addr_of(bufs);
  const int q = lane / L;
  const int li = lane % L;
  uint32_t err = 0;

  // segment record of group gg for lane s < G (raw loads, used later)
  auto rec = [&](uint64_t gg, uint64_t& page, uint32_t& st, uint32_t& en) {
    const bool sl = gg < ngroups && lane < G && gg * G + (uint64_t)lane < num_seg;
    const uint64_t gs = sl ? gg * G + (uint64_t)lane : 0;
    page = sl ? a.seg_page[gs] : 0;
    st = sl ? a.seg_start[gs] : 0u;
    en = sl ? a.seg_end[gs] : 0u;
  };
  // a loaded record -> page validity, the page's lock word, slot ranges, op
  // prefetch, page DMAs.  lock_and_read_page (Tree.cpp:205-242, 851-852):
  // the word is taken with an atomic max of the chunk's epoch tag (insert.hip
  // take_word; a smaller value is a retired chunk's hold, the same tag a
  // shared hold) in the same round trip as the page DMA; its old value is
  // checked before the page is used
  auto stage = [&](uint64_t gg, uint64_t page, uint32_t st, uint32_t en, uint32_t b,
                   bool& pok, uint64_t& lkold, uint32_t& qst, uint32_t& qen, uint64_t& pk,
                   uint64_t& pv, uint32_t& po) {
    const bool sl = lane < G && gg * G + (uint64_t)lane < num_seg;
    const bool pgok = sl && ptr_ok(page, a.node, a.arena_bytes);
    if (ballot(sl && !pgok)) err |= kErrBadPtr;
    pok = pgok;
    lkold = 0;
    if (pgok)
      lkold = atomicMax(reinterpret_cast<unsigned long long*>(a.locks) +
                            cityhash64_u64(page) % a.num_locks,
                        (unsigned long long)a.tag);
    qst = shfl32(st, q);
    qen = shfl32(en, q);
    const bool pf = (uint32_t)li < qen - qst;
    pk = pf ? a.op_key[qst + (uint32_t)li] : 0;
    pv = pf ? a.op_val[qst + (uint32_t)li] : 0;
    po = pf ? a.oslot[qst + (uint32_t)li] : 0u;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // buffer b's reads are done
    const uint64_t dma = ballot(pgok);
#pragma unroll
    for (int s = 0; s < G; ++s)
      if ((dma >> s) & 1)
        glds16(a.arena + ga_offset(rl64(page, s)), bufs_lds + (uint32_t)((b * G + s) * kPageSize));
  };

  uint64_t c_page, n_page, c_lk;
  uint32_t c_st, c_en, n_st, n_en;
  bool c_pok;
  uint32_t c_qst, c_qen;
  uint64_t c_pk, c_pv;
  uint32_t c_po;
  rec(g, c_page, c_st, c_en);
  stage(g, c_page, c_st, c_en, 0, c_pok, c_lk, c_qst, c_qen, c_pk, c_pv, c_po);
  rec(g + W, n_page, n_st, n_en);
  for (uint32_t it = 0;; ++it) {
    wait_vm<0>();  // group g's pages, lock words and ops, group g + W's records
    const uint32_t b = it & 1u;
    const uint64_t gn = g + W;
    bool x_pok = false;
    uint64_t x_lk = 0;
    uint32_t x_qst = 0, x_qen = 0;
    uint64_t x_pk = 0, x_pv = 0;
    uint32_t x_po = 0;
    uint64_t m_page = 0;
    uint32_t m_st = 0, m_en = 0;
    // a word held by a later tag is not this chunk's to take (never in a
    // serialised tree: reported as a lock failure, the segment left as is)
    const bool held = c_lk <= a.tag;
    if (ballot(c_pok && !held)) err |= kErrLock;
    if (gn < ngroups) {  // wave-uniform
      stage(gn, n_page, n_st, n_en, b ^ 1u, x_pok, x_lk, x_qst, x_qen, x_pk, x_pv, x_po);
      rec(gn + W, m_page, m_st, m_en);
    }
    err |= apply_group<G>(a, bufs + b * G * kPageDwords, g * G, num_seg, c_page, c_pok && held,
                          true, c_qst, c_qen, c_pk, c_pv, c_po);
    if (gn >= ngroups) break;
    g = gn;
    c_page = n_page;
    c_pok = x_pok;
    c_lk = x_lk;
    c_qst = x_qst;
    c_qen = x_qen;
    c_pk = x_pk;
    c_pv = x_pv;
    c_po = x_po;
    n_page = m_page;
    n_st = m_st;
    n_en = m_en;
  }
  if (err) atomicOr(a.err, err);
}

void launch_leaf_upsert(const SegArgs& a, hipStream_t s) {
  constexpr int G = 4;
  if (!a.num_seg) return;
  static const unsigned blocks = [] {
    int per_cu = 0, cus = 0, dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_leaf_upsert_pipe<G>, kBlock, 0);
    return (unsigned)((per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 256));
  }();
  const uint64_t groups = (a.num_seg + G - 1) / G;
  const uint64_t need = (groups + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(k_leaf_upsert_pipe<G>, dim3((unsigned)std::min<uint64_t>(need, blocks)),
                     dim3(kBlock), 0, s, a);
}

}  // namespace dev
}  // namespace shm
