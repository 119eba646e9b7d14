// get.hip — batched Tree::search walk with grouped page resolution.
//
// Restates src/Tree.cpp:405-459 (search), 593-663 (page_search),
// 665-685 (internal_page_search) and 687-697 (leaf_page_search) for a batch.
//
// One wave64 owns 64 queries, sorted by key across its lanes (bitonic, in
// registers), so the queries waiting on one page form a run of lanes.  Each
// round, the run heads' pages are fetched G at a time: one
// global_load_lds_dwordx4 (1 KB LDS-DMA) per page into one of two G-page LDS
// buffers, so group g + 1 is in flight while group g is resolved.  A group is
// resolved by the whole wave at once, not page by page:
//   * query side (lane = query): every lane reads the header of its own
//     page's slot (per-lane LDS address; G distinct pages), checks versions
//     (Tree.cpp:616-618) and fences (k >= highest -> sibling, 626-629), and
//     for an internal page runs a 6-step branchless search over its page's
//     keys (child = #keys <= k, 665-685);
//   * entry side (lane = entries): the 64 lanes split into G groups of
//     L = 64 / G lanes, group q holding slot q's 54 leaf entries, E = 54 / L
//     consecutive entries per lane (one 18E-byte chunk).  Per step t, group q
//     compares its entries with the key of query (head_q + t) of its run and
//     the wave ballots the hits; the query lane takes the value of the first
//     valid slot (key == k && value != 0 && f == r, Tree.cpp:687-697) with one
//     lane permute.
// The per-page scalar work (waits, header broadcasts, per-key ballots) of a
// page-at-a-time walk is paid once per G pages.
#include "device_common.h"
#include <hip/hip_ext.h>

#include "kernels.h"
#include "lds_dma.h"
#include "leaf_chunk.h"

namespace shm {
namespace dev {

namespace {

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t lds_u64(const uint32_t* lp, int d) {
  return (uint64_t)lp[d] | ((uint64_t)lp[d + 1] << 32);
}

}  // namespace

template <int G, int NB, int WPB>
__global__ __launch_bounds__(WPB * kWave) void k_get(WalkArgs a) {
  constexpr int L = kWave / G;                               // lanes per page
  constexpr int E = (kLeafCardinality + L - 1) / L;          // entries per lane
  constexpr int CD = kLeafEntry * E / 4;                     // dwords per lane chunk
  static_assert(kLeafEntry * E % 4 == 0, "lane chunks must be dword multiples");
  static_assert(G * L == kWave, "G must divide 64");
  static_assert(NB >= 1 && NB <= 4, "1..4 group buffers");
  constexpr int kWaveRing = NB * G * kPageDwords;
  __shared__ __attribute__((aligned(16))) uint32_t s_ring[WPB * kWaveRing];

  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  const uint64_t n = a.n;
  // XCD-aware chunk order: blocks are dealt to the 8 XCDs round-robin
  // (block b -> XCD b % 8; placement only affects speed), so give each XCD a
  // contiguous run of chunks.  Neighbouring chunks share internal pages and
  // write their results into one fine-partition range, and both then stay in
  // one XCD's L2 instead of being fetched / partially written back by eight.
  const uint32_t nb = gridDim.x, bx = blockIdx.x;
  const uint32_t xcd = a.xcd_remap ? bx & 7u : 0u, per = nb >> 3, rem = nb & 7u;
  const uint32_t lblock = a.xcd_remap
                              ? xcd * per + (xcd < rem ? xcd : rem) + (bx >> 3)
                              : bx;
  const uint64_t wave_base = ((uint64_t)lblock * WPB + (uint64_t)wv) * kWave;
  if (wave_base >= n) return;  // wave-uniform
  const uint32_t nact = (uint32_t)(n - wave_base < (uint64_t)kWave ? n - wave_base : kWave);
  const uint32_t* ring = &s_ring[wv * kWaveRing];
  const uint32_t ring_lds = lds_addr_of(ring);

  // sort this wave's queries by key; tag = lane the query came from
  uint64_t k = (uint32_t)lane < nact ? a.keys[wave_base + lane] : kKeyMax;
  uint32_t tag = (uint32_t)lane;
  wave_sort64(k, tag);
  const bool active = tag < nact;

  // leaf directory: start at the leaf (or the covering internal page), else
  // at the root
  uint64_t ptr = a.root;
  if (a.dir) ptr = dir_start(a.dir, a.dir_lo, a.dir_shift, a.dir_n, a.node, k, ptr);
  // occupancy bound of my page (kLeafHwFull after a move: read it whole)
  uint32_t hw = kLeafHwFull;
  if (a.leaf_hw && ptr_ok(ptr, a.node, a.arena_bytes)) hw = a.leaf_hw[ga_offset(ptr) >> 10];
  // kKeyMax can never be stored (root highest is exclusive, Tree.h:150)
  bool done = !active || k == kKeyMax;
  uint64_t val = 0;
  uint32_t err = 0;
  int rounds = 0, retries = 0;

  // entry side: this lane holds entries [E*li, E*li + E) of slot q
  const int q = lane / L;
  const int li = lane % L;
  // chunks stay inside the page: the last lane's chunk is shifted down to end
  // at entry 53 and masks the entries its left neighbour owns; lanes past
  // 54 / E mask everything
  const int ebase = chunk_base<E>(li);
  const int chunk_dw = (kOffRecords + kLeafEntry * ebase) / 4;
  const uint64_t lanemask_le = ~0ull >> (63 - lane);

  for (;;) {
    const uint64_t pend = ballot(!done);
    if (pend == 0) break;
    if (++rounds > kMaxRounds) {
      err |= kErrGetHops;
      break;
    }
    // run heads: first lane of each run of equal page pointers
    const int pl = lane == 0 ? 0 : lane - 1;
    const uint64_t prev = shfl64(ptr, pl);
    const bool prev_pend = ((pend >> pl) & 1) != 0;
    const bool head = !done && (lane == 0 || !prev_pend || prev != ptr);
    const uint64_t H = ballot(head);
    const uint64_t Hle = H & lanemask_le;
    const int run = popc64(Hle) - 1;          // run index of this (pending) lane
    const int myhead = 63 - __builtin_clzll(Hle | 1ull);
    const int ng = (popc64(H) + G - 1) / G;
    // invalid pointers load the superblock (always mapped) and are rejected
    // when resolved; padding slots of a short group load it too, so every
    // group is exactly G DMAs and the waits below are constants
    const bool pok = ptr_ok(ptr, a.node, a.arena_bytes);
    const uint64_t pload = pok ? ptr : 0;
    uint64_t hi = H;  // heads still to load
    uint64_t hr = H;  // heads still to resolve

    auto issue = [&](int b) {
#pragma unroll
      for (int s = 0; s < G; ++s) {
        uint64_t off = 0;
        int nl = 1;  // padding: the superblock's first and last lanes
        if (hi) {
          const int h = ctz64(hi);
          off = ga_offset(rl64(pload, h));
          nl = hw_dma_lanes(rl32(hw, h));
          hi &= hi - 1;
        }
        // lanes past the page's last occupied slot skip their 16 B (the
        // last lane, rear_version, always loads: every DMA counts in vmcnt)
        if (lane < nl || lane == 63) {
          if (a.nt)
            glds16_nt(a.arena + off, ring_lds + (uint32_t)((b * G + s) * kPageSize));
          else
            glds16(a.arena + off, ring_lds + (uint32_t)((b * G + s) * kPageSize));
        }
      }
    };
#pragma unroll
    for (int b = 0; b < NB; ++b)
      if (b < ng) issue(b);

    for (int g = 0; g < ng; ++g) {
      // groups issued after g: min(NB - 1, ng - 1 - g), G DMAs each
      const int later = ng - 1 - g < NB - 1 ? ng - 1 - g : NB - 1;
      if (later >= 3)
        wait_vm<3 * G>();
      else if (later == 2)
        wait_vm<2 * G>();
      else if (later == 1)
        wait_vm<G>();
      else
        wait_vm<0>();
      const int b = g % NB;
      // head lane of each slot of this group (64 = padding)
      int hq[G];
#pragma unroll
      for (int s = 0; s < G; ++s) {
        hq[s] = hr ? ctz64(hr) : 64;
        hr &= hr - 1;
      }
      const uint32_t* buf = ring + b * G * kPageDwords;

      // ---- one LDS trip: my page's header (query side), my entry chunk of
      // slot q (entry side) and the key of slot q's first query --------------
      const int slot = run - g * G;
      const bool inq = !done && slot >= 0 && slot < G;
      const uint32_t* lp = buf + (inq ? slot : 0) * kPageDwords;
      const u32x4 A = *reinterpret_cast<const u32x4*>(lp);      // dwords 0..3
      const u32x4 B = *reinterpret_cast<const u32x4*>(lp + 4);  // dwords 4..7
      const u32x2 C = *reinterpret_cast<const u32x2*>(lp + 8);  // dwords 8..9
      const uint32_t C2 = lp[10];
      const u32x2 Z = *reinterpret_cast<const u32x2*>(lp + 254);
      uint32_t D[CD];
      int hsrc = hq[0];
      uint64_t kq = 0;
      uint32_t hwq = kLeafHwFull;  // slots of page q that were loaded
      {
        const uint32_t* ep = buf + q * kPageDwords + chunk_dw;
#pragma unroll
        for (int i = 0; i < CD; ++i) D[i] = ep[i];
#pragma unroll
        for (int s = 1; s < G; ++s) hsrc = q == s ? hq[s] : hsrc;
        kq = shfl64(k, hsrc < 63 ? hsrc : 63);
        hwq = shfl32(hw, hsrc < 63 ? hsrc : 63);
      }

      const uint64_t leftmost = (uint64_t)((A.z >> 8) | (A.w << 24)) |
                                ((uint64_t)((A.w >> 8) | (B.x << 24)) << 32);
      const uint64_t sibling = (uint64_t)((B.x >> 8) | (B.y << 24)) |
                               ((uint64_t)((B.y >> 8) | (B.z << 24)) << 32);
      const uint64_t lowest = (uint64_t)B.w | ((uint64_t)C.x << 32);
      const uint64_t highest = (uint64_t)C.y | ((uint64_t)C2 << 32);
      const int cnt = (int)(int16_t)(B.z >> 16) + 1;
      const bool is_leaf = leftmost == 0;
      const uint32_t rver = (is_leaf ? Z.x : Z.y) & 0xFF;
      const bool vok = (A.z & 0xFF) == rver;
      const bool live = inq && pok && vok;
      const bool right = live && k >= highest;  // turn right
      const bool low = live && k < lowest;      // mis-routed
      const bool here = live && !right && !low;
      const bool qint = here && !is_leaf;
      const bool qleaf = here && is_leaf;
      const uint64_t any_int = ballot(qint);
      // the buffer is no longer needed once no internal page is searched in
      // it: refill it now so the next group's pages land during the compute
      bool refilled = false;
      if (!any_int && g + NB < ng) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue(b);
        refilled = true;
      }
      if (ballot(inq && !pok)) err |= kErrBadPtr;
      if (ballot(inq && pok && !vok)) {
        // torn / in-flight page: its queries re-list it next round
        if (++retries > kMaxRetries) err |= kErrInconsistent;
      }
      if (ballot(low)) err |= kErrFence;

      // ---- internal pages: branchless search, lane = query ----------------
      if (any_int) {
        int pos = 0;  // number of keys <= k (keys strictly increase)
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
          const int idx = pos + step - 1;
          const int ci = idx < 60 ? idx : 60;
          const uint64_t kk = lds_u64(lp, 11 + 4 * ci);
          pos += (idx < cnt && kk <= k) ? step : 0;
        }
        const uint64_t child = lds_u64(lp, 13 + 4 * (pos > 0 ? pos - 1 : 0));
        ptr = qint ? (pos == 0 ? leftmost : child) : ptr;
        hw = qint ? kLeafHwFull : hw;
      }

      // ---- leaf pages: lane groups hold the entries -----------------------
      uint64_t lq = ballot(qleaf);
      if (lq) {
        uint64_t ekey[E], evalue[E];
        uint32_t efr[E], erv[E];
        chunk_entries<E>(D, ekey, evalue, efr, erv);
        bool eok[E];
#pragma unroll
        for (int j = 0; j < E; ++j)
          eok[j] = evalue[j] != kValueNull && ((efr[j] ^ erv[j]) & 0xF) == 0 &&
                   ebase + j >= li * E && (uint32_t)(ebase + j) < hwq;
        const int tl = lane - myhead;  // my position in my run
        const int sl = slot & (G - 1);
        for (int t = 0;; ++t) {
          bool hit = false;
          uint64_t hv = 0;
#pragma unroll
          for (int j = E - 1; j >= 0; --j) {  // lowest slot wins
            const bool h = eok[j] && ekey[j] == kq;
            hit = hit || h;
            hv = h ? evalue[j] : hv;
          }
          const uint64_t M = ballot(hit);
          const bool mine = qleaf && tl == t;
          const uint64_t mq = (M >> (sl * L)) & (L == 64 ? ~0ull : ((1ull << (L & 63)) - 1));
          const uint64_t v = shfl64(hv, sl * L + (mq ? ctz64(mq) : 0));
          val = mine ? (mq ? v : 0) : val;
          lq &= ~ballot(mine);
          if (!lq) break;
          const int src = hsrc + t + 1;
          kq = shfl64(k, src < 63 ? src : 63);
        }
      }

      ptr = right ? sibling : ptr;
      hw = right ? kLeafHwFull : hw;
      done = done || (inq && !pok) || low || (right && sibling == 0) || qleaf ||
             (qint && ptr == 0);
      if (!refilled && g + NB < ng) {
        // the buffer's LDS reads are complete before its next DMA lands
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue(b);
      }
    }
    if (retries > kMaxRetries) break;
  }
  if (err) atomicOr(a.err, err);
  if (active) {
    const uint64_t i = wave_base + tag;
    const uint64_t o = a.perm ? (uint64_t)a.perm[i] : i;
    a.out_val[o] = val;
    if (a.out_found) a.out_found[o] = val != kValueNull ? 1 : 0;
  }
}

// ---- the summary walk: lane = query ------------------------------------------
//
// Per get, three HBM lines instead of a 1 KB page: the leaf-directory entry,
// the leaf's 64 B summary line (layout.h: the highest fence, an 8-bit
// fingerprint per slot) and the entries whose fingerprint matches (false
// positives ~ 36 / 255 per get at C2's 36 keys per leaf).
// A stale directory is fixed by turning right on k >= highest from the
// summary (B-link).  Pages without a summary (internal pages: a directory
// miss, or no directory) are walked from their own bytes, lane by lane:
// check_consistent, fences, binary search of the records (Tree.cpp:593-685).
// The leaf search keeps Tree.cpp:687-697: the first slot (in slot order) with
// key == k, value != 0 and f == r.  Batches are serialised against inserts
// by the call order, so a page is never torn under a get; the entry-level
// f == r check stays.
//
// Without a directory the walk starts at the root, or — with the LDS
// replica of the top of the tree (a.top_n: every page of one upper level
// with its lowest fence, launch_top) — at the page of that level holding k,
// found by a binary search of the block's LDS copy (the north star's "upper
// tree levels replicated in LDS"; DESIGN §8 measures it against the
// directory).

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
  return v;
}

// 5 waves per SIMD (95 VGPRs, no scratch).  Round 4 capped it at 6 waves
// (80 VGPRs: C2 +2 % against 5 then); with the pair form and the shared
// rounds the cap spilled 28-48 B per lane into scratch on the candidate
// rounds: same box C2 18623 / 18631 and C3 12750 / 12903 at 6 waves against
// 19572 / 19611 and 14828 / 14986 at 5.
// PCHK (SHM_FLAG_PAGE_CHECK): the page-level version check on the fast
// path too -- a hit read from a page's entry also reads that page's
// front_version (byte 8) and rear_version (byte 1016) and reports a
// mismatch (kErrInconsistent: check_consistent, Tree.h:241-261, Tree.cpp:
// 616-618); two more lines per get (DESIGN §3.5 measures it)
template <int TPB, bool PCHK>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(5))) void k_get_sum(WalkArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_top[];  // top_n x (8 + 4) B
  const uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x;
  const uint32_t tn = a.top_n;
  uint64_t* tk = reinterpret_cast<uint64_t*>(s_top);
  uint32_t* tpg = reinterpret_cast<uint32_t*>(s_top + 8 * (uint64_t)tn);
  if (tn) {  // block-uniform: the replica into LDS
    for (uint32_t j = threadIdx.x; j < tn; j += TPB) {
      tk[j] = a.top_keys[j];
      tpg[j] = a.top_pages[j];
    }
    __syncthreads();
  }
  if (a.clk && threadIdx.x == 0) a.clk[blockIdx.x] = wall_clock64();
  const bool act = i < a.n;
  const uint64_t k = act ? a.keys[i] : kKeyMax;
  uint64_t val = 0;
  uint32_t err = 0;
  uint32_t c_int = 0, c_right = 0, c_hops = 0, c_ent = 0;
  bool hit = false;
  uint32_t pv_f = 0, pv_r = 0;  // PCHK: the hit page's front / rear versions
  if (k != kKeyMax) {  // never stored (root highest is exclusive, Tree.h:150)
    uint64_t ptr = a.root;
    uint64_t alt = 0;  // a tie's safe start (dir_start_e)
    bool done = false;  // val is the answer
    if (a.dir) {
      u32x4 e[4];
      bool fpform;
      ptr = dir_start_e(a.dir, a.dir_lo, a.dir_shift, a.dir_n, a.node, k, ptr, e, fpform, &alt);
      // A wave's gets take their slowest lane's number of dependent rounds,
      // so the lanes share rounds: after the directory entry, a lane in
      // fingerprint form reads its lowest candidate entry (the prefix lies
      // in one leaf and the entry holds its fingerprints: Tree.cpp:687-697's
      // first valid slot with the key) while a lane that needs the summary
      // line reads it -- before, the summary lanes waited for the whole
      // wave's candidate loop -- and then every lane reads one candidate per
      // round, lowest first, the summary lanes' first beside the fingerprint
      // lanes' second.  A stale copy, an absent key, a right turn, a tie's
      // safe start, an internal page go on below.  C3 +5-7 %, C2 +0.5 %
      // (same box, first form); reading two candidates per round was C2
      // -2 % (speculative requests) for about the same C3.
      const bool pok = ptr_ok(ptr, a.node, a.arena_bytes);
      const uint64_t off = ga_offset(ptr);
      const uint8_t* page = a.arena + off;
      const bool fp = fpform && pok;
      // a read phase's pair form: the prefix's own keys, in up to four leaves
      bool pu = false;
      const uint32_t pc = !fpform && pok ? dir_pair_cand(e, k, pu) : 0u;
      const bool sm = !fpform && pok && !pu;
      // an exact directory (built, then kept by every insert chunk since):
      // a usable entry names every key of its prefix, so a key it does not
      // lead to is absent -- no summary walk for a miss (a tie at a split
      // point, or more matching pairs than the lane queues, walks anyway)
      const bool exact_miss = a.dir_exact && ((fpform && pok) || (pu && alt == 0 &&
                                                                  __builtin_popcount(pc) <= 8));
      // pend: the lane's candidate slots of its leaf still to read, lowest
      // first; a pair lane's candidates instead as up to 8 packed bytes
      // (leaf << 6 | slot) in plist, with the leaves' pages in lpg (the
      // directory entry itself is dead past this point: held through the
      // rounds it spilled registers, C3 -15 %)
      uint64_t pend = fp ? dir_fp_cand(e, k) : 0;
      uint64_t plist = 0;
      uint32_t pn = 0;
      const uint32_t lpg[4] = {e[0].x, e[0].y, e[0].z, e[0].w};
      if (pu) {
#pragma unroll
        for (int j = 0; j < (int)kDirPairMax; ++j) {
          if (((pc >> j) & 1u) && pn < 8) {
            uint32_t pgi;
            int sl;
            dir_pair_slot(e, j, pgi, sl);
            const uint32_t leaf = pgi == lpg[0] ? 0u : pgi == lpg[1] ? 1u : pgi == lpg[2] ? 2u : 3u;
            plist |= (uint64_t)((leaf << 6) | (uint32_t)sl) << (8 * pn);
            ++pn;
          }
        }
      }
      // the next candidate -> its page and slot (false: a pair naming a bad
      // page); pops it
      const uint8_t* cp = page;
      int cs = 0;
      auto next = [&]() -> bool {
        if (pn == 0) {
          cp = page;
          cs = (int)ctz64(pend);
          pend &= pend - 1;
          return true;
        }
        const uint32_t b = (uint32_t)plist & 0xFFu;
        plist >>= 8;
        --pn;
        cs = (int)(b & 63u);
        const uint32_t li = b >> 6;
        const uint64_t ga = dir_page_ga(li == 0 ? lpg[0] : li == 1 ? lpg[1] : li == 2 ? lpg[2] : lpg[3],
                                        a.node);
        cp = a.arena + ga_offset(ga);
        return ptr_ok(ga, a.node, a.arena_bytes);
      };
      RawEntry r1;
      bool l1 = false;
      const bool any1 = pend || pn;
      if (any1) {
        l1 = next();
        if (l1) entry_load(cp, cs, r1);
      }
      u32x4 sraw[4];
      if (sm) sum_load(a.sum, off, sraw);
      uint64_t ek, ev;
      uint32_t ef, er;
      if (any1 && l1) {
        ++c_ent;
        entry_decode(r1, ek, ev, ef, er);
        if (entry_hit(ek, ev, ef, er, k)) {
          val = ev;
          hit = done = true;
          if (PCHK) {
            pv_f = cp[kOffFrontVer];
            pv_r = cp[kOffLeafRear];
          }
        }
      }
      // a summary lane in k's leaf (k >= highest turns right below) joins
      // the candidate rounds
      SumLine sl;
      const bool inleaf = sm && sum_decode(sraw, k, sl) && k < sl.highest;
      if (inleaf) pend = sl.cand;
      while (!done && (pend || pn)) {  // one candidate per lane and round, lowest first
        if (next()) {
          ++c_ent;
          lane_entry(cp, cs, ek, ev, ef, er);
          if (entry_hit(ek, ev, ef, er, k)) {
            val = ev;
            done = true;
            hit = fp || pu;
            if (PCHK) {
              pv_f = cp[kOffFrontVer];
              pv_r = cp[kOffLeafRear];
            }
          }
        }
      }
      if (!done && exact_miss) done = true;  // absent (val stays 0)
      // not found: a fingerprint or pair lane takes the summary walk below
      // (absent key or stale copy); a summary lane's leaf does not hold k,
      // unless this was a tie's optimistic leaf (k may lie below its lowest
      // fence: walk again from the safe start)
      if (!done && inleaf) {
        if (alt) {
          ptr = alt;
          alt = 0;
        } else {
          done = true;
        }
      }
    } else if (tn) {
      // the last page of the level whose lowest fence is <= k (tk[0] = kKeyMin)
      uint32_t lo = 0, hi = tn;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (tk[mid] <= k)
          lo = mid;
        else
          hi = mid;
      }
      ptr = dir_page_ga(tpg[lo], a.node);
    }
    int retries = 0;
    for (int hop = 0; !done; ++hop) {
      if (hop > kMaxRounds) {
        err |= kErrGetHops;
        break;
      }
      if (!ptr_ok(ptr, a.node, a.arena_bytes)) {
        err |= kErrBadPtr;
        break;
      }
      const uint64_t off = ga_offset(ptr);
      const uint8_t* page = a.arena + off;
      SumLine sl;
      if (sum_read(a.sum, off, k, sl)) {
        if (k >= sl.highest) {  // turn right (Tree.cpp:626-629)
          const uint64_t sib = page_sibling(a.arena + off);
          if (!sib) {
            err |= kErrFence;
            break;
          }
          ptr = sib;
          ++c_right;
          continue;
        }
        uint64_t cand = sl.cand;
        while (cand) {
          uint64_t ek, ev;
          uint32_t ef, er;
          ++c_ent;
          lane_entry(page, ctz64(cand), ek, ev, ef, er);
          if (entry_hit(ek, ev, ef, er, k)) {
            val = ev;
            if (PCHK) {
              pv_f = page[kOffFrontVer];
              pv_r = page[kOffLeafRear];
            }
            break;
          }
          cand &= cand - 1;
        }
        if (val == kValueNull && alt) {
          // a tie's optimistic leaf does not hold k: k may lie below its
          // lowest fence, so walk again from the safe start
          ptr = alt;
          alt = 0;
          continue;
        }
        break;
      }
      // no summary: the page's own bytes
      if (hop == 0) c_int = 1;
      ++c_hops;
      const u32x4* pw = reinterpret_cast<const u32x4*>(page);
      const u32x4 A = pw[0], B = pw[1], C = pw[2];
      const uint64_t leftmost = (uint64_t)((A.z >> 8) | (A.w << 24)) |
                                ((uint64_t)((A.w >> 8) | (B.x << 24)) << 32);
      const uint64_t sibling = (uint64_t)((B.x >> 8) | (B.y << 24)) |
                               ((uint64_t)((B.y >> 8) | (B.z << 24)) << 32);
      const uint64_t lowest = (uint64_t)B.w | ((uint64_t)C.x << 32);
      const uint64_t highest = (uint64_t)C.y | ((uint64_t)C.z << 32);
      const int cnt = (int)(int16_t)(B.z >> 16) + 1;
      const bool leaf = leftmost == 0;
      const uint32_t* pd = reinterpret_cast<const uint32_t*>(page);
      const uint32_t rver = (leaf ? pd[kOffLeafRear / 4] : pd[kOffInternalRear / 4]) & 0xFF;
      if ((A.z & 0xFF) != rver) {  // torn page: read it again (Tree.cpp:616-618)
        if (++retries > kMaxRetries) {
          err |= kErrInconsistent;
          break;
        }
        continue;
      }
      if (k >= highest && sibling) {
        ptr = sibling;
        ++c_right;
        continue;
      }
      if (k < lowest && alt) {  // a tie's optimistic leaf: k lies to its left
        ptr = alt;
        alt = 0;
        continue;
      }
      if (k < lowest || k >= highest) {
        err |= kErrFence;
        break;
      }
      if (leaf) {  // every slot
        for (int sl = 0; sl < kLeafCardinality; ++sl) {
          uint64_t ek, ev;
          uint32_t ef, er;
          lane_entry(page, sl, ek, ev, ef, er);
          if (entry_hit(ek, ev, ef, er, k)) {
            val = ev;
            break;
          }
        }
        break;  // k >= lowest: this leaf is k's, found or not
      }
      // internal_page_search (Tree.cpp:665-685): child = #keys <= k
      int lo = 0, hi = cnt < kInternalCardinality ? cnt : kInternalCardinality;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const uint64_t km = (uint64_t)pd[11 + 4 * mid] | ((uint64_t)pd[12 + 4 * mid] << 32);
        if (km <= k)
          lo = mid + 1;
        else
          hi = mid;
      }
      ptr = lo == 0 ? leftmost
                    : ((uint64_t)pd[13 + 4 * (lo - 1)] | ((uint64_t)pd[14 + 4 * (lo - 1)] << 32));
    }
  }
  if (a.stats) {  // wave-uniform; every lane of the wave is here
    const uint32_t v[kIdxStats] = {wave_sum32(act && k != kKeyMax ? 1u : 0u), wave_sum32(c_int),
                                   wave_sum32(c_right), wave_sum32(c_hops), wave_sum32(c_ent),
                                   wave_sum32(act && val != kValueNull ? 1u : 0u),
                                   wave_sum32(hit ? 1u : 0u)};
    if (lane_id() == 0)
      for (int j = 0; j < kIdxStats; ++j)
        if (v[j]) atomicAdd(reinterpret_cast<unsigned long long*>(a.stats + j), v[j]);
  }
  if (PCHK && pv_f != pv_r) err |= kErrInconsistent;  // a torn page under a get
  if (err) atomicOr(a.err, err);
  if (act) {
    a.out_val[i] = val;
    if (a.out_found) a.out_found[i] = val != kValueNull ? 1 : 0;
  }
  if (a.clk && lane_id() == 0)
    a.clk[gridDim.x + blockIdx.x * (TPB / kWave) + (threadIdx.x / kWave)] = wall_clock64();
}

uint64_t get_sum_blocks(uint64_t n) { return (n + kGetSumTPB - 1) / kGetSumTPB; }

void launch_get_sum(const WalkArgs& a, uint64_t n, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  if (n == 0) {
    // the profile's events still complete
    if (ev0) (void)hipEventRecord(ev0, s);
    if (ev1) (void)hipEventRecord(ev1, s);
    return;
  }
  constexpr int TPB = kGetSumTPB;
  const uint32_t lds = (uint32_t)a.top_n * 12;
  const dim3 grid((unsigned)((n + TPB - 1) / TPB));
  // ev0 / ev1 (the profile): the dispatch's own start and end
  if (a.page_check)
    hipExtLaunchKernelGGL((k_get_sum<TPB, true>), grid, dim3(TPB), lds, s, ev0, ev1, 0u, a);
  else
    hipExtLaunchKernelGGL((k_get_sum<TPB, false>), grid, dim3(TPB), lds, s, ev0, ev1, 0u, a);
}

// ---- the top of the tree for the LDS replica ---------------------------------
// One block, breadth first from the root: level by level, every page's
// children (leftmost, then the records' pointers) and their lowest fences
// (the parent's lowest for leftmost, the record key otherwise,
// Tree.cpp:665-685), in key order, until the next level would not fit max_n
// pages or the leaves are next.  scratch: 4 x max_n u64.
__global__ __launch_bounds__(1024) void k_top(const uint8_t* arena, uint64_t arena_bytes,
                                              uint16_t node, uint64_t root, uint32_t max_n,
                                              uint64_t* keys, uint32_t* pages,
                                              uint64_t* scratch, uint32_t* n_out,
                                              uint32_t* err) {
  __shared__ uint32_t s_n, s_ws[16], s_stop;
  const int t = threadIdx.x;
  uint64_t* cur_p = scratch;
  uint64_t* cur_k = scratch + max_n;
  uint64_t* nxt_p = scratch + 2 * (uint64_t)max_n;
  uint64_t* nxt_k = scratch + 3 * (uint64_t)max_n;
  if (t == 0) {
    cur_p[0] = root;
    cur_k[0] = kKeyMin;
    s_n = 1;
    s_stop = 0;
  }
  __syncthreads();
  for (int level = 0; level < kMaxLevelOfTree; ++level) {
    const uint32_t n = s_n;
    // children per page of the current level (0: a leaf level; stop)
    uint32_t total = 0;
    for (uint32_t base = 0; base < n; base += 1024) {
      const uint32_t j = base + t;
      uint32_t c = 0;
      if (j < n) {
        const uint64_t p = cur_p[j];
        if (!ptr_ok(p, node, arena_bytes)) {
          atomicOr(err, kErrBadPtr);
          atomicOr(&s_stop, 1u);
        } else {
          const uint8_t* pg = arena + ga_offset(p);
          const uint32_t* d = reinterpret_cast<const uint32_t*>(pg);
          const uint64_t leftmost = (uint64_t)((d[2] >> 8) | (d[3] << 24)) |
                                    ((uint64_t)((d[3] >> 8) | (d[4] << 24)) << 32);
          const int cnt = (int)(int16_t)(pg[kOffLastIndex] | (pg[kOffLastIndex + 1] << 8)) + 1;
          c = leftmost ? 1u + (uint32_t)(cnt < 0 ? 0 : cnt) : 0u;
          if (!leftmost || pg[kOffLevel] <= 1) atomicOr(&s_stop, 1u);  // children are leaves
        }
      }
      total += c;
    }
    // block total of children
    uint32_t v = total;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    if ((t & 63) == 0) s_ws[t >> 6] = v;
    __syncthreads();
    uint32_t all = 0;
    for (int w = 0; w < 16; ++w) all += s_ws[w];
    const bool stop = s_stop != 0 || all > max_n || all == 0;
    __syncthreads();
    if (stop) break;
    // children in order: one pass per 1024 pages, an exclusive scan of counts
    uint32_t run = 0;
    for (uint32_t base = 0; base < n; base += 1024) {
      const uint32_t j = base + t;
      uint32_t c = 0;
      uint64_t leftmost = 0, lowest = 0;
      const uint8_t* pg = nullptr;
      if (j < n) {
        pg = arena + ga_offset(cur_p[j]);
        const uint32_t* d = reinterpret_cast<const uint32_t*>(pg);
        leftmost = (uint64_t)((d[2] >> 8) | (d[3] << 24)) |
                   ((uint64_t)((d[3] >> 8) | (d[4] << 24)) << 32);
        const int cnt = (int)(int16_t)(pg[kOffLastIndex] | (pg[kOffLastIndex + 1] << 8)) + 1;
        c = 1u + (uint32_t)(cnt < 0 ? 0 : cnt);
        lowest = cur_k[j];
      }
      uint32_t incl = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
        if ((t & 63) >= o) incl += y;
      }
      if ((t & 63) == 63) s_ws[t >> 6] = incl;
      __syncthreads();
      uint32_t wb = 0, bt = 0;
      for (int w = 0; w < 16; ++w) {
        wb += w < (t >> 6) ? s_ws[w] : 0u;
        bt += s_ws[w];
      }
      const uint32_t pos = run + wb + incl - c;
      if (c) {
        nxt_p[pos] = leftmost;
        nxt_k[pos] = lowest;
        const uint32_t* d = reinterpret_cast<const uint32_t*>(pg);
        for (uint32_t r = 0; r + 1 < c; ++r) {
          const uint32_t w0 = (kOffRecords + kInternalEntry * r) / 4;
          nxt_k[pos + 1 + r] = (uint64_t)d[w0] | ((uint64_t)d[w0 + 1] << 32);
          nxt_p[pos + 1 + r] = (uint64_t)d[w0 + 2] | ((uint64_t)d[w0 + 3] << 32);
        }
      }
      run += bt;
      __syncthreads();
    }
    // swap
    uint64_t* x = cur_p;
    cur_p = nxt_p;
    nxt_p = x;
    x = cur_k;
    cur_k = nxt_k;
    nxt_k = x;
    if (t == 0) s_n = all;
    __syncthreads();
  }
  const uint32_t n = s_n;
  for (uint32_t j = t; j < n; j += 1024) {
    keys[j] = cur_k[j];
    pages[j] = dir_page_index(cur_p[j]);
  }
  if (t == 0) *n_out = n;
}

void launch_top(const uint8_t* arena, uint64_t arena_bytes, uint16_t node, uint64_t root,
                uint32_t max_n, uint64_t* keys, uint32_t* pages, uint64_t* scratch,
                uint32_t* n_out, uint32_t* err, hipStream_t s) {
  hipLaunchKernelGGL(k_top, dim3(1), dim3(1024), 0, s, arena, arena_bytes, node, root, max_n,
                     keys, pages, scratch, n_out, err);
}

// summaries of a loaded image: one wave per page
__global__ __launch_bounds__(256) void k_sum_rebuild(const uint8_t* arena, uint64_t pages,
                                                     uint8_t* sum) {
  const uint64_t pg = 1 + ((uint64_t)blockIdx.x * 256 + threadIdx.x) / kWave;
  if (pg >= pages) return;  // wave-uniform
  const int lane = lane_id();
  const uint8_t* page = arena + pg * kPageSize;
  const u32x4* pw = reinterpret_cast<const u32x4*>(page);
  const u32x4 A = pw[0], B = pw[1], C = pw[2];
  const uint64_t leftmost = (uint64_t)((A.z >> 8) | (A.w << 24)) |
                            ((uint64_t)((A.w >> 8) | (B.x << 24)) << 32);
  const uint64_t highest = (uint64_t)C.y | ((uint64_t)C.z << 32);
  if (leftmost != 0) {  // internal page: no summary
    if (lane == 0) clear_leaf_sum(sum, pg * kPageSize);
    return;
  }
  uint32_t fp = 0;
  if (lane < kLeafCardinality) {
    uint64_t ek, ev;
    uint32_t ef, er;
    lane_entry(page, lane, ek, ev, ef, er);
    fp = ev != kValueNull ? key_fp(ek) : 0u;
  }
  put_leaf_sum(sum, pg * kPageSize, highest, fp);
}

void launch_sum_rebuild(const uint8_t* arena, uint64_t pages, uint8_t* sum, hipStream_t s) {
  if (pages <= 1) return;
  const uint64_t waves = pages - 1;
  hipLaunchKernelGGL(k_sum_rebuild, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, arena,
                     pages, sum);
}

// G = 4 pages per group, NB = 1 group buffer, 4 waves per block: 16 KB of
// LDS per block, 24-28 waves per CU (deeper buffers lost
// occupancy and measured 2-8 % slower)
void launch_get(const WalkArgs& a, uint64_t n, hipStream_t s) {
  if (n == 0) return;
  constexpr int G = 4, NB = 1, WPB = 4;
  const uint64_t waves = (n + kWave - 1) / kWave;
  hipLaunchKernelGGL((k_get<G, NB, WPB>), dim3((unsigned)((waves + WPB - 1) / WPB)),
                     dim3(WPB * kWave), 0, s, a);
}

}  // namespace dev
}  // namespace shm
