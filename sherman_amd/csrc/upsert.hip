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
#include "split_wave.h"

namespace shm {
namespace dev {

namespace {

// A block's work queue in LDS.  Groups: wave w of the block takes the
// block's next group k (k-th of b * 4 + (k & 3) + (k >> 2) * W, the same
// groups the static w, w + W, ... assignment gave the block), so a wave that
// spends time on an early split leaves its share to the block's other waves.
// Early splits (split_wave.h split_early): queued by the wave that found
// them (slot, fields, then its ready word), taken by any wave of the block
// after its next group or once it has no group left; more than kEarlyMax in
// a block: the rest go to k_upper as before.
constexpr uint32_t kEarlyMax = 64;
struct BlockQ {
  uint32_t next;    // the block's next unclaimed group
  uint32_t active;  // waves still taking groups
  uint32_t ealloc;  // early split slots handed out
  uint32_t eclaim;  // early splits taken
  uint32_t ready[kEarlyMax];
  EarlyItem item[kEarlyMax];
};
using EarlyList = BlockQ;

// one queued early split for the wave (lane-0 LDS atomics, broadcast); false
// when none is queued right now
__device__ __forceinline__ bool take_early(BlockQ* q, uint32_t& x) {
  uint32_t got = ~0u;
  if (lane_id() == 0) {
    for (;;) {
      const uint32_t c = __hip_atomic_load(&q->eclaim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      uint32_t n = __hip_atomic_load(&q->ealloc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      n = n < kEarlyMax ? n : kEarlyMax;
      if (c >= n) break;
      if (atomicCAS(&q->eclaim, c, c + 1) == c) {
        got = c;
        break;
      }
    }
    // its producer is a running wave of this block between taking the slot
    // and publishing it
    if (got != ~0u)
      while (__hip_atomic_load(&q->ready[got], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
        __builtin_amdgcn_s_sleep(1);
  }
  got = rl32(got, 0);
  x = got;
  return got != ~0u;
}

}  // namespace

// Apply one group of G staged pages (buf: G x 1 KB in LDS; slot s = lanes
// [s L, s L + L)): versions and fences, the segment's ops in key order with
// the reference's slot rule, the changed entries written back, and the
// segment's split plan (seg_T / seg_P / seg_newpages / seg_ver).  page / pok
// are valid in lanes s < G; qst / qen / pk / pv per slot group.  Returns the
// error bits.
// early: small splits go to the block's list el (u: the split arguments,
// cursor0 the superblock's next_page)
template <int G>
__device__ __forceinline__ uint32_t apply_group(const SegArgs& a, const uint32_t* buf,
                                                uint64_t g0, uint32_t num_seg, uint64_t page,
                                                bool pok, bool locked, uint32_t qst,
                                                uint32_t qen, uint64_t pk, uint64_t pv,
                                                uint32_t po, const UpperArgs& u, EarlyList* el,
                                                bool early, uint64_t cursor0) {
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
  uint32_t eop[E];  // the op that took slot j (fresh)
  uint32_t cnt = 0;  // valid entries of slot q (the same in all its lanes)
#pragma unroll
  for (int j = 0; j < E; ++j) {
    mine[j] = ebase + j >= li * E;
    valid[j] = mine[j] && ev[j] != kValueNull;
    dirty[j] = false;
    fresh[j] = false;
    eop[j] = 0;
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
        if (isnew) eop[j] = qst + t;
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
        if (fresh[j]) {
          set_leaf_fp(a.sum, ga_offset(qpage), ebase + j, ek[j]);
          // for the directory upkeep after the chunk (k_dir_upkeep)
          if (a.placed) a.placed[eop[j]] = kOpPlaced | (uint32_t)(ebase + j);
        }
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
    a.seg_ver[gq] = live ? fver : ~0u;
    // a small split when the block's list has room: its pages now (one
    // atomic while the in-place groups go on), built after them
    bool queued = false;
    if (early && P > 1 && P <= kSmallSplit) {
      const uint32_t x = atomicAdd(&el->ealloc, 1u);
      if (x < kEarlyMax) {
        queued = true;
        EarlyItem& it = el->item[x];
        it.page = qpage;
        it.first = cursor0 + atomicAdd(reinterpret_cast<unsigned long long*>(&u.ctl->ualloc[u.par][0]),
                                       (unsigned long long)(P - 1));
        it.hint1 = dir_hint_page(u, pk, 1);  // pk: the segment's first op key (li == 0)
        it.st = qst;
        it.nb = qen - qst;
        it.T = T;
        it.pv = P | (fver << 8);
        __hip_atomic_store(&el->ready[x], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    a.seg_newpages[gq] = queued ? 0u : P - 1;
    if (P > 1 && !queued) {
      a.ctl->late[a.par][0] = 1u;
      // k_upper block range of this segment (insert.hip block_range)
      const uint32_t r = (uint32_t)((gq * a.up_nb) / num_seg);
      atomicAdd(&a.ctl->leaf_np[a.par][r], P - 1);
      atomicAdd(&a.ctl->leaf_ns[a.par][r], 1u);
      if (P > kSmallSplit) atomicAdd(&a.ctl->leaf_nb[a.par][r], P - 1);
    }
  }
  return err;
}

// The in-place groups of wave w (its first group g).
// Software-pipelined: a grid of about one resident wave set; each wave loops
// over groups
// w, w + W, ... and, while it applies group g from one LDS buffer, the pages
// of group g + W are already landing in the other (LDS-DMA) and the segment
// records of g + 2W and the ops of g + W are in flight.  Per group the wave
// then pays about the apply time instead of two dependent HBM round trips.
template <int G>
__device__ __forceinline__ uint32_t upsert_groups(const SegArgs& a, const UpperArgs& u,
                                                  BlockQ* el, bool early, uint64_t cursor0,
                                                  uint64_t cap, uint64_t W, uint64_t ngroups,
                                                  uint32_t num_seg, uint32_t* s_pg, WaveLds& Lw) {
  constexpr int L = kWave / G;
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
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

  // the block's next group (>= ngroups: none left)
  auto claim = [&]() -> uint64_t {
    uint32_t k = 0;
    if (lane == 0) k = atomicAdd(&el->next, 1u);
    k = rl32(k, 0);
    return (uint64_t)(k >> 2) * W + (uint64_t)blockIdx.x * kWavesPerBlock + (k & 3u);
  };
  uint64_t g = claim();
  if (g >= ngroups) return err;
  uint64_t gn = claim();
  uint64_t c_page, n_page, c_lk;
  uint32_t c_st, c_en, n_st, n_en;
  bool c_pok;
  uint32_t c_qst, c_qen;
  uint64_t c_pk, c_pv;
  uint32_t c_po;
  rec(g, c_page, c_st, c_en);
  stage(g, c_page, c_st, c_en, 0, c_pok, c_lk, c_qst, c_qen, c_pk, c_pv, c_po);
  rec(gn, n_page, n_st, n_en);
  for (uint32_t it = 0;; ++it) {
    wait_vm<0>();  // group g's pages, lock words and ops, group gn's records
    const uint32_t b = it & 1u;
    uint64_t gm = ngroups;
    bool x_pok = false;
    uint64_t x_lk = 0;
    uint32_t x_qst = 0, x_qen = 0;
    uint64_t x_pk = 0, x_pv = 0;
    uint32_t x_po = 0;
    uint64_t m_page = 0;
    uint32_t m_st = 0, m_en = 0;
    // a word held by a later tag is not this chunk's to take (never in a
    // serialised tree: reported as a lock failure, the segment left as is)
    // (tag | 1: an internal page's exclusive hold by an early split that
    // shares the word, lock_index hashes pages of every level)
    const bool held = c_lk <= (a.tag | 1ull);
    if (ballot(c_pok && !held)) err |= kErrLock;
    if (gn < ngroups) {  // wave-uniform
      stage(gn, n_page, n_st, n_en, b ^ 1u, x_pok, x_lk, x_qst, x_qen, x_pk, x_pv, x_po);
      gm = claim();
      rec(gm, m_page, m_st, m_en);
    }
    err |= apply_group<G>(a, bufs + b * G * kPageDwords, g * G, num_seg, c_page, c_pok && held,
                          true, c_qst, c_qen, c_pk, c_pv, c_po, u, el, early, cursor0);
    if (gn >= ngroups) break;
    g = gn;
    gn = gm;
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
  return err;
}

// Early splits (u.early): a segment that would split into at most
// kSmallSplit pages is queued in the block's LDS queue instead of being left
// to k_upper, and a wave of the same block builds it and takes its separators
// up (split_wave.h split_early) between its groups or after them, so C5's
// splits run beside the in-place groups instead of in a kernel of their own.
// A block's waves are resident together: a wave without groups waits (LDS)
// for its block's last queued split, never for other blocks.
// A wave takes queued splits once the block's groups are all taken (taking
// them between groups, round 4's interleaved variant, needed more VGPRs than
// the pipelined loop leaves and measured slower).
template <int G>
__device__ __forceinline__ void upsert_body(const SegArgs& a, const UpperArgs& u) {
  __shared__ __attribute__((aligned(16))) uint32_t s_pg[kWavesPerBlock * 2 * G * kPageDwords];
  __shared__ __attribute__((aligned(16))) WaveLds s_wl[kWavesPerBlock];
  __shared__ BlockQ s_q;
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  const uint64_t W = (uint64_t)gridDim.x * kWavesPerBlock;
  const uint32_t num_seg = *a.num_seg_dev;
  if (num_seg == 0) return;  // every op applied in place (C3's chunks): the block's only load
  const uint64_t ngroups = ((uint64_t)num_seg + G - 1) / G;
  // early splits need a root above the leaves (a leaf root grows the tree:
  // k_upper) and the direct path (SHM_UPPER_LISTS=1 sends all to the lists)
  const Superblock* sb = reinterpret_cast<const Superblock*>(a.arena);
  const uint64_t cursor0 = sb->next_page;
  const uint64_t cap = sb->capacity_pages;
  const bool early = u.early && sb->root_level >= 1 && !u.no_direct;
  // diagnostic clocks (u.stamps, tools/upper_stamps.py)
  uint64_t* clk = u.stamps && blockIdx.x < 1024 && threadIdx.x == 0
                      ? u.stamps + kUpsertStamps + blockIdx.x
                      : nullptr;
  if (clk) clk[0] = wall_clock64();
  if (threadIdx.x < kEarlyMax) s_q.ready[threadIdx.x] = 0;
  if (threadIdx.x == 0) {
    s_q.next = 0;
    s_q.active = kWavesPerBlock;
    s_q.ealloc = 0;
    s_q.eclaim = 0;
  }
  __syncthreads();
  uint32_t err = upsert_groups<G>(a, u, &s_q, early, cursor0, cap, W, ngroups, num_seg, s_pg,
                                  s_wl[wv]);
  // this wave queues nothing more
  if (lane == 0) __hip_atomic_fetch_add(&s_q.active, ~0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (clk && early) clk[1024] = wall_clock64();
  if (early) {
    for (;;) {
      uint32_t x;
      if (take_early(&s_q, x)) {
        err |= split_early(u, s_wl[wv], s_q.item[x], cursor0, cap,
                           u.stamps && x == 0 && blockIdx.x < 1024
                               ? u.stamps + kUpsertStamps + 4 * 1024 + blockIdx.x
                               : nullptr);
        continue;
      }
      uint32_t act = 0;
      if (lane == 0) act = __hip_atomic_load(&s_q.active, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (rl32(act, 0) == 0) {
        if (take_early(&s_q, x)) {
          err |= split_early(u, s_wl[wv], s_q.item[x], cursor0, cap);
          continue;
        }
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  if (err && lane == 0) atomicOr(a.err, err);
  if (clk) {
    clk[2 * 1024] = wall_clock64();
    clk[3 * 1024] = s_q.ealloc;
  }
}

template <int G>
__global__ __launch_bounds__(kBlock) void k_leaf_upsert_pipe(SegArgs a, UpperArgs u) {
  upsert_body<G>(a, u);
}

void launch_leaf_upsert(const SegArgs& a, const UpperArgs& u, hipStream_t s) {
  constexpr int G = 4;
  if (!a.num_seg) return;
  static unsigned nb = 0;
  if (!nb) {
    int per_cu = 0, cus = 0, dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_leaf_upsert_pipe<G>, kBlock, 0);
    nb = (unsigned)((per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 256));
  }
  const uint64_t groups = (a.num_seg + G - 1) / G;
  const uint64_t need = (groups + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(k_leaf_upsert_pipe<G>, dim3((unsigned)std::min<uint64_t>(need, nb)), dim3(kBlock),
                     0, s, a, u);
}

}  // namespace dev
}  // namespace shm
