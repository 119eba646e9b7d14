// insert.hip — split propagation and deletes of a batched insert, driven by
// the device (no host read-back between the levels).
//
// Restates src/Tree.cpp:828-991 (leaf_page_store's split half), 699-826
// (internal_page_store), 126-149 (update_new_root) and 993-1057
// (leaf_page_del) for a sorted, de-duplicated batch.  The in-place half of
// leaf_page_store (the common case) is upsert.hip; what it leaves behind is a
// set of flagged leaf segments (seg_P > 1: the page would reach 54 entries)
// whose per-range new-page counts it accumulated in UpperCtl.
//
// k_upper is one launch per chunk that finishes the batch.  Work is split
// into phases (the leaf level, then each internal level, then the deletes);
// a phase whose results a later one reads hands its tasks out by ticket and
// ends at a hand-off (see "phase tickets and hand-offs" below), so no phase
// needs the launch's blocks to be resident together:
//   leaf level     per block: ordered scan of the per-range new-page counts;
//                  waves build new right siblings (k-way split, ceil(T / 36)
//                  pages) and rewrite page 0 of each split in place
//                  (set_consistent: front++, rear = front) once every sibling
//                  builder has read the old page (a per-segment counter);
//                  small splits take their separators up at once (propagate)
//                  --- hand-off, when a later phase needs the leaves ---
//   level L >= 1   block tasks: runs of separators with one parent, one wave
//                  per run under the parent's exclusive lock word: merged in
//                  place if T <= 60, else split into ceil((T + 1) / 41) pages
//                  --- hand-off ---
//   deletes        every wave: Tree::del of the chunk's deletes
// Lock words are epoch tagged (lock_excl below).
// Pages come from a device bump cursor (the superblock's next_page; the
// reference's LocalAllocator bump, include/LocalAllocator.h:21-43), checked
// against the arena capacity before each level.  The root page never moves:
// when the root splits, its left half is written to a fresh page X and the
// root page itself becomes the new internal root {leftmost = X} one level up
// (update_new_root, Tree.cpp:126-149, without the root-pointer CAS and the
// NEW_ROOT broadcast, Tree.cpp:116-124: every reader already starts there).
// Separators come out sorted (segment order = key order) and become the next
// level's batch.  Nothing here waits for the host; the superblock and a
// mapped host mirror are updated at the end of the launch.
#include "device_common.h"
#include "kernels.h"
#include "split_wave.h"
#include "upper_quick.h"

namespace shm {
namespace dev {

// Chunk r of level `level`'s separators (emitted unordered by the level
// below; chunks of `per` <= kLvlSort), sorted by key in LDS, cut into runs
// of one parent hint, one wave per run.  With per = ceil(n / nb) the few
// separators of C5's upper levels spread over as many blocks.
constexpr uint32_t kLvlSort = 1024;
struct LvlLds {
  uint64_t key[kLvlSort];
  uint64_t ptr[kLvlSort];
  uint64_t hint[kLvlSort];
  uint32_t head[kLvlSort];
};
__device__ __forceinline__ uint32_t level_per(uint32_t n, uint32_t nb) {
  const uint32_t share = (n + nb - 1) / nb;
  return share < kLvlSort ? share : kLvlSort;
}
__device__ __forceinline__ void upper_chunk(const UpperArgs& a, WaveLds& L, LvlLds& S, uint32_t* red,
                            uint32_t n, uint32_t per, uint32_t r, uint32_t level, uint64_t base,
                            uint64_t cap, uint32_t& err) {
  const int t = threadIdx.x, wv = t >> 6;
  const bool odd = (level & 1) != 0;
  const uint64_t* gk = odd ? a.sep_key[1] : a.sep_key[0];
  const uint64_t* gp = odd ? a.sep_ptr[1] : a.sep_ptr[0];
  const uint64_t* gh = odd ? a.ipage[1] : a.ipage[0];
  {
    const uint32_t c0 = r * per;
    const uint32_t cnt = n - c0 < per ? n - c0 : per;
    uint32_t m2 = 1;
    while (m2 < cnt) m2 <<= 1;
    for (uint32_t j = t; j < m2; j += kUpT) {
      const bool v = j < cnt;
      S.key[j] = v ? gk[c0 + j] : kKeyMax;
      S.ptr[j] = v ? gp[c0 + j] : 0;
      S.hint[j] = v ? gh[c0 + j] : 0;
    }
    __syncthreads();
    // bitonic sort by key (keys of one level are distinct)
    for (uint32_t k = 2; k <= m2; k <<= 1)
      for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
        for (uint32_t i = t; i < m2; i += kUpT) {
          const uint32_t l = i ^ jj;
          if (l > i) {
            const bool up = (i & k) == 0;
            const uint64_t x = S.key[i], y = S.key[l];
            if ((x > y) == up) {
              S.key[i] = y;
              S.key[l] = x;
              const uint64_t p = S.ptr[i], q = S.hint[i];
              S.ptr[i] = S.ptr[l];
              S.hint[i] = S.hint[l];
              S.ptr[l] = p;
              S.hint[l] = q;
            }
          }
        }
        __syncthreads();
      }
    // runs of one parent hint
    uint32_t nh = 0;
    for (uint32_t base_i = 0; base_i < cnt; base_i += kUpT) {
      const uint32_t i = base_i + t;
      const bool hd = i < cnt && (i == 0 || S.hint[i] != S.hint[i - 1]);
      uint32_t th;
      const uint32_t x = block_scan(hd ? 1u : 0u, red, &th);
      if (hd) S.head[nh + x] = i;
      nh += th;
      __syncthreads();
    }
    for (uint32_t hx = wv; hx < nh; hx += kUpWaves) {
      const uint32_t hs = S.head[hx];
      const uint32_t he = hx + 1 < nh ? S.head[hx + 1] : cnt;
      apply_run(a, L, S.key, S.ptr, hs, he, S.hint[hs], level, base, cap, err);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_upper: one launch per insert chunk, one 512-thread block per CU at most;
// no phase needs the blocks to be resident together (tickets and hand-offs
// above).
//   prologue  per-range prefix sums of the upsert kernel's new-page counts
//   leaf      phase 0 (large splits only): their sibling pages, four per
//             ticket; phase 1, every split: a small one (<= kSmallSplit
//             pages) built whole by one wave, siblings first and page 0 last
//             (it holds the old page's survivors, so no fan-in); a large
//             one's page 0 after the fan-in of its sibling builders
//   direct    (every split small, C5's chunks) the wave then takes its
//             split's separators up itself (propagate): parents under their
//             exclusive words, a parent's split going one level further, the
//             root growing in place -- no list and, unless deletes follow,
//             no hand-off: splits are then dealt statically (wave w takes
//             w, w + W, ...)
//   otherwise each new leaf's separator goes to position (its global
//             new-page index) of level 1's list: key order
//   --- hand-off (phases 0 and 1) ---
//   level 1   block tasks: separator range r of nb, runs of one parent, one
//             wave per run: the parent's epoch lock word, its survivors and
//             the run merged, rewritten in place or split (pages by an
//             atomic bump past the leaf level's), new separators to level 2
//   --- hand-off ---
//   level >=2 block tasks: chunks of the level's separators (emitted
//             unordered), sorted in LDS, runs of one parent under its
//             exclusive word; a hand-off after every level
//   deletes   Tree::del of the chunk's deletes, after every split
//   last      the last block to finish: if a hand-off gave up, it runs the
//             levels and the deletes again alone (idempotent); then the
//             superblock and its host mirror
// 4 waves per SIMD (<= 128 VGPRs): two blocks fit a CU.
// (3 waves per SIMD: 144 VGPRs and no scratch; at 4 the cap spilled 68 B
// per lane.  One 512-thread block per CU either way; C5 / C3 within noise)
__global__ __launch_bounds__(kUpT) __attribute__((amdgpu_waves_per_eu(3))) void k_upper(
    UpperArgs a) {
  __shared__ __attribute__((aligned(16))) WaveLds s_l[kUpWaves];
  __shared__ uint32_t s_red[kUpWaves];
  __shared__ uint32_t s_flag;
  __shared__ uint32_t s_tk;  // the block's ticket
  __shared__ uint32_t s_list[kUpT];  // segment heads of one separator chunk
  __shared__ __attribute__((aligned(16))) LvlLds s_lvl;  // levels >= 2: one chunk
  // completed by the segmentation kernel (no new key, no delete)
  if (a.ctl->skip[a.par][0] == a.batch) return;
  const int t = threadIdx.x, lane = lane_id(), wv = t >> 6;
  const uint32_t b = blockIdx.x, nb = gridDim.x;
  const uint64_t W = (uint64_t)nb * kUpWaves;
  const uint64_t wid = (uint64_t)b * kUpWaves + (uint64_t)wv;
  const uint64_t T = (uint64_t)nb * kUpT, tid = (uint64_t)b * kUpT + (uint64_t)t;
  WaveLds& L = s_l[wv];
  UpperCtl* ctl = a.ctl;
  uint32_t nstamp = 1;
  auto stamp = [&]() {
    if (a.stamps && b == 0 && t == 0 && nstamp < (uint32_t)kUpperStamps) {
      a.stamps[nstamp++] = wall_clock64();
      a.stamps[0] = nstamp;
    }
  };
  stamp();
  // per-block clocks (diagnostic): this block's start, and its end below
  uint64_t* bclk = a.stamps && b < 256 && t == 0 ? a.stamps + kUpperStamps + 8 * 256 + b : nullptr;
  if (bclk) bclk[0] = wall_clock64();
  Superblock* sb = reinterpret_cast<Superblock*>(a.arena);
  const uint32_t par = a.par;
  // the superblock as the chunk found it (the last block derives the new one
  // from it and the chunk's counters)
  const uint64_t cursor0 = sb->next_page;
  const uint64_t splits0 = sb->splits;
  uint32_t root_level = (uint32_t)sb->root_level;
  const uint64_t cap = sb->capacity_pages;
  uint32_t err = 0;
  const uint32_t ns = *a.ns_dev;
  // the counts the earlier kernels left, requested before the stores below
  // (which the compiler cannot move them past): one round trip at the start
  const uint32_t v_np = (uint32_t)t < nb ? ctl->leaf_np[par][t] : 0u;
  const uint32_t v_ns = (uint32_t)t < nb ? ctl->leaf_ns[par][t] : 0u;
  const uint32_t v_nb = (uint32_t)t < nb ? ctl->leaf_nb[par][t] : 0u;
  // the delete count: the segmentation kernel's copy in UpperCtl, not the
  // ordering's count, which chunk tag + 2's ordering (another stream) may
  // rewrite as soon as block 0 below publishes the op buffers free while
  // another block of this launch has not started
  const uint64_t n_del = ctl->ndel[par][0];
  if (a.prof && b == 0 && t == 0) {  // the chunk's counts (profiling)
    atomicAdd(reinterpret_cast<unsigned long long*>(a.prof), (unsigned long long)a.n_del[-1]);
    atomicAdd(reinterpret_cast<unsigned long long*>(a.prof) + 1, (unsigned long long)n_del);
    atomicAdd(reinterpret_cast<unsigned long long*>(a.prof) + 2, (unsigned long long)ns);
  }
  const uint32_t late = ctl->late[par][0];
  // pages the upsert kernel's early splits took from next_page on (theirs
  // come first; failed takes past the capacity used no page)
  const uint64_t ua = ctl->ualloc[par][0];
  // block 0's thread 0, for the fast path below: the root growth of the early
  // splits and the error bits of the chunk's earlier kernels, both final at
  // launch (in the same round trip as the loads above)
  uint32_t rn0 = 0, err0 = 0;
  if (b == 0 && t == 0) {
    rn0 = __hip_atomic_load(&ctl->root_new[par][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    err0 = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // no split left to k_upper and no delete (C5's chunks once their splits
  // are early): the blocks skip the count scans and block 0 alone writes the
  // superblock below
  const bool quick = late == 0 && n_del == 0 && !a.force_abort;
  upper_zero_next(ctl, par, tid, T);
  // leaf level: the upsert kernel left per-range new-page / split counts
  __shared__ uint32_t s_pnp[kMaxUpper + 1], s_pns[kMaxUpper + 1];
  uint32_t total = 0, nsplit = 0, nbig = 0;
  if (!quick) {
    const uint32_t xnp = block_scan(v_np, s_red, &total);
    const uint32_t xns = block_scan(v_ns, s_red, &nsplit);
    nbig = block_sum(v_nb, s_red);
    if ((uint32_t)t < nb) {
      s_pnp[t] = xnp;
      s_pns[t] = xns;
    }
    if (t == 0) {
      s_pnp[nb] = total;
      s_pns[nb] = nsplit;
    }
    __syncthreads();
  }
  const uint64_t cursor0e = cursor0 + ua < cap ? cursor0 + ua : cap;
  // nothing left to split and nothing to delete (every op applied in place,
  // C3's chunks, or every split early, C5's): only the batch count and the
  // early splits' pages and root growth change, so block 0 writes the
  // superblock and no block waits for the others (no fan-in on `done`)
  if (total == 0 && n_del == 0 && !a.force_abort) {
    if (b == 0 && t == 0) {
      // the error attribution first: no load or returning atomic after the
      // host mirror's stores (each would wait for their PCIe writes)
      if (err0 & ~kErrKeyMax) atomicCAS(a.err + 1, 0u, (uint32_t)a.batch);
      if (cursor0e != cursor0) {
        if (rn0 > root_level) root_level = rn0;
        sb->next_page = cursor0e;
        sb->root_level = root_level;
        sb->splits = splits0 + (cursor0e - cursor0);
        if (a.pub) {
          __hip_atomic_store(a.pub + 1, cursor0e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(a.pub + 2, (uint64_t)root_level, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(a.pub + 3, splits0 + (cursor0e - cursor0), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
      // the chunk's tag: with new pages, or whenever the host asks (its
      // directory is behind the tree: tree.cpp dir_stale's quiet rule)
      if (a.pub && (cursor0e != cursor0 || a.pub_always))
        __hip_atomic_store(a.pub + 0, a.batch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      sb->batches = a.batch;
      // no block of this launch reads the op buffers or the ordering's
      // counts on this path
      if (a.pub)
        __hip_atomic_store(a.pub + kPubApplied, a.batch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
    stamp();
    if (bclk) bclk[256] = wall_clock64();
    return;
  }
  bool ok = true;
  // every split small (C5's chunks): each wave takes its separators up
  // itself (propagate), no level list
  const bool direct = nbig == 0 && !a.no_direct;
  const bool grow0 = root_level == 0;  // the root is a leaf: its split grows the tree
  const bool fits = cursor0e + total + (grow0 ? 1u : 0u) <= cap;
  // pages past the leaf level's: the internal levels' bump allocator
  const uint64_t base = cursor0e + total + (grow0 ? 1u : 0u);
  // a later phase reads the leaf level's results (level 1's list, or the
  // deletes its pages): its tasks go by ticket and end at a hand-off
  const bool wait_leaf = !direct || n_del != 0 || a.force_abort != 0;
  uint32_t mine = 0;  // lane 0: the wave's finished tasks of the current phase
  if (total && !fits) {
    // arena exhausted: the flagged segments stay unapplied (reported)
    err |= kErrNoMem;
  } else if (total) {
    stamp();
    const uint64_t first = cursor0e;          // arena page of global new page 0
    const uint64_t xroot = cursor0e + total;  // the root's left half (grow0)
    const uint32_t ftag = fan_tag(a.batch, 0);
    // phase 0: sibling pages of the large splits (none in C5), four per
    // ticket (nbig > 0 implies wait_leaf: always by ticket)
    constexpr uint32_t kStepA = 4;
    for (uint32_t g0 = nbig ? wave_claim(&ctl->tk[par][0][0], kStepA) : total; g0 < total;
         g0 = wave_claim(&ctl->tk[par][0][0], kStepA)) {
      for (uint32_t gp = g0; gp < g0 + kStepA && gp < total; ++gp) {
        if (lane == 0) ++mine;
        const uint32_t r = last_le(s_pnp, nb, gp);
        uint32_t r0, r1, g, before;
        block_range(ns, r, nb, r0, r1);
        find_seg(a.seg_np, r0, r1, gp - s_pnp[r], false, g, before);
        if (g >= r1) {
          err |= kErrPlan;
          continue;
        }
        if (a.seg_P[g] <= kSmallSplit) continue;  // built whole in phase 1
        const uint32_t pb = s_pnp[r] + before;
        const int p = (int)(gp - pb) + 1;
        const Ops o0{a.op_key, a.op_val, a.seg_start[g], a.seg_end[g] - a.seg_start[g]};
        const u32x4 w = load_page_slice(a.arena, ga_offset(a.seg_page[g]));
        const Hdr h = parse_hdr(w);
        stage_page(L.page, w);
        wave_lds_sync();
        const Ops o = stage_ops(L, o0);
        const int na = leaf_survivors(L, o);
        // the old page 0 has been read: its rewrite may go ahead
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) fan_arrive(a.leaf_rd + g, ftag);
        const SplitPage sp{p, (int)a.seg_P[g], a.seg_T[g], first + pb,
                           new_ga(a.node, first + pb, p)};
        const uint64_t low = build_leaf_page(a, L, h, na, o, sp);
        const uint64_t par_pg = grow0 ? a.root : parent_of(a, low, 1, &err);
        if (lane == 0) {
          a.sep_key[1][gp] = low;
          a.sep_ptr[1][gp] = sp.dest;
          a.ipage[1][gp] = par_pg;
        }
      }
    }
    // phase 1: every split -- a small one whole (siblings, then page 0), a
    // large one's page 0 once its sibling builders have read the old page
    uint32_t k = wait_leaf ? wave_claim(&ctl->tk[par][1][0], 1u) : (uint32_t)wid;
    for (; k < nsplit; k = wait_leaf ? wave_claim(&ctl->tk[par][1][0], 1u) : k + (uint32_t)W) {
      if (lane == 0) ++mine;
      const uint32_t r = last_le(s_pns, nb, k);
      uint32_t r0, r1, g, before;
      block_range(ns, r, nb, r0, r1);
      find_seg(a.seg_np, r0, r1, k - s_pns[r], true, g, before);
      if (g >= r1) {
        err |= kErrPlan;
        continue;
      }
      const uint32_t pb = s_pnp[r] + before;
      const int P = (int)a.seg_P[g];
      const uint64_t page = a.seg_page[g];
      const bool small = (uint32_t)P <= kSmallSplit;
      if (!small && !fan_in(a.leaf_rd + g, (uint32_t)(P - 1), ftag)) err |= kErrFanIn;
      const Ops o0{a.op_key, a.op_val, a.seg_start[g], a.seg_end[g] - a.seg_start[g]};
      // the page and the segment's ops (<= 64 of them) requested together
      const bool few = o0.nb <= (uint32_t)kWave;
      uint64_t ok0 = 0, ov0 = 0;
      if (few && (uint32_t)lane < o0.nb) {
        ok0 = o0.key[o0.st + lane];
        ov0 = o0.val[o0.st + lane];
      }
      const u32x4 w = load_page_slice(a.arena, ga_offset(page));
      const uint64_t first_key = few ? rl64(ok0, 0) : o0.key[o0.st];
      // the level-1 parent (the directory's hint for the first op key), and
      // in the direct path its exclusive word, taken while the leaf pages are
      // built: one atomic whose result is looked at after the builds
      const uint64_t hint1 = direct ? dir_hint_page(a, first_key, 1) : 0ull;
      const bool pre = direct && !grow0 && hint1 != 0 &&
                       ptr_ok(hint1, a.node, a.arena_bytes);
      unsigned long long lk_old = ~0ull;
      if (pre && lane == 0)
        lk_old = atomicMax(reinterpret_cast<unsigned long long*>(a.locks) +
                               lock_index(hint1, a.num_locks),
                           (unsigned long long)(a.tag | 1ull));
      const Hdr h = parse_hdr(w);
      if (h.fver != a.seg_ver[g] || h.fver != h.rver_leaf) err |= kErrPlan;
      stage_page(L.page, w);
      if (few && (uint32_t)lane < o0.nb) {
        L.o_key[lane] = ok0;
        L.o_val[lane] = ov0;
      }
      wave_lds_sync();
      const Ops o = few ? Ops{L.o_key, L.o_val, 0, o0.nb} : o0;
      const int na = leaf_survivors(L, o);
      if (small) {
        for (int p = 1; p < P; ++p) {
          const SplitPage sp{p, P, a.seg_T[g], first + pb, new_ga(a.node, first + pb, p)};
          const uint64_t low = build_leaf_page(a, L, h, na, o, sp);
          if (direct) {  // the wave's run for level 1
            if (lane == 0) {
              L.r_key[p - 1] = low;
              L.r_ptr[p - 1] = sp.dest;
            }
            continue;
          }
          const uint64_t par_pg = grow0 ? a.root : parent_of(a, low, 1, &err);
          if (lane == 0) {
            const uint32_t gp = pb + (uint32_t)(p - 1);
            a.sep_key[1][gp] = low;
            a.sep_ptr[1][gp] = sp.dest;
            a.ipage[1][gp] = par_pg;
          }
        }
      }
      const uint64_t dest = grow0 ? ga_make(a.node, xroot * kPageSize) : page;
      (void)build_leaf_page(a, L, h, na, o, SplitPage{0, P, a.seg_T[g], first + pb, dest});
      if (grow0) write_new_root(a, L, dest, 1, h.fver);
      // the word taken above: a free value came back exactly when it was taken
      // (lock_excl's rule); otherwise apply_run spins for it as usual
      const bool held = pre && rl64((uint64_t)lk_old, 0) <= a.tag;
      if (direct) propagate(a, L, (uint32_t)(P - 1), 1, base, cap, err, grow0 ? 0ull : hint1, held);
    }
    stamp();
    if (wait_leaf)
      ok = handoff(ctl, par, 0, mine, (nbig ? total : 0u) + nsplit, a.force_abort != 0, s_red,
                   &s_flag);
    stamp();
  }

  // ---- internal levels: block tasks ------------------------------------------
  // solo: the launch's last block alone, every task in order, no tickets or
  // hand-offs (it completes what the hand-offs of the others abandoned)
  auto run_levels = [&](bool solo) -> bool {
    bool okl = true;
    // level 1: runs of separators with one parent (range rr of nb)
    const uint64_t* skey = a.sep_key[1];
    const uint64_t* sptr = a.sep_ptr[1];
    const uint64_t* spg = a.ipage[1];
    const uint32_t nsep = total;
    uint32_t done1 = 0, seq = 0;  // thread 0: the block's finished tasks
    for (uint32_t rr = solo ? seq++ : block_claim(&ctl->tk[par][2][0], &s_tk); rr < nb;
         rr = solo ? seq++ : block_claim(&ctl->tk[par][2][0], &s_tk)) {
      if (t == 0) ++done1;
      uint32_t r0, r1;
      block_range(nsep, rr, nb, r0, r1);
      for (uint32_t c0 = r0; c0 < r1; c0 += kUpT) {
        const uint32_t i = c0 + (uint32_t)t;
        const bool head = i < r1 && (i == 0 || spg[i] != spg[i - 1]);
        uint32_t th;
        const uint32_t x = block_scan(head ? 1u : 0u, s_red, &th);
        __syncthreads();
        if (head) s_list[x] = i;
        __syncthreads();
        for (uint32_t hx = (uint32_t)wv; hx < th; hx += kUpWaves) {
          const uint32_t hi = s_list[hx];
          const uint64_t page = spg[hi];
          // the run's end: first index past hi whose page differs
          uint32_t e = hi + 1;
          for (;;) {
            const uint32_t j = e + (uint32_t)lane;
            const uint64_t m = ballot(j >= nsep || spg[j] != page);
            if (m) {
              e += (uint32_t)ctz64(m);
              break;
            }
            e += kWave;
          }
          if (!ptr_ok(page, a.node, a.arena_bytes)) {
            err |= kErrBadPtr;
            continue;
          }
          // the run under the parent's exclusive word, B-link right moves as
          // at the upper levels (a solo pass finds parents that split since
          // the hint was taken); a short run staged in the wave's LDS
          const uint32_t nr = e - hi;
          if (nr <= (uint32_t)kWave) {
            if ((uint32_t)lane < nr) {
              L.o_key[lane] = skey[hi + lane];
              L.o_val[lane] = sptr[hi + lane];
            }
            wave_lds_sync();
            apply_run(a, L, L.o_key, L.o_val, 0, nr, page, 1, base, cap, err);
          } else {
            apply_run(a, L, skey, sptr, hi, e, page, 1, base, cap, err);
          }
        }
        __syncthreads();
      }
    }
    stamp();
    okl = solo ? block_fence() : handoff(ctl, par, 2, done1, nb, false, s_red, &s_flag);
    stamp();
    // levels >= 2: chunks of the level's separators
    for (uint32_t level = 2; okl; ++level) {
      const uint32_t n0 = __hip_atomic_load(&ctl->lvl_sep[par][level], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
      if (n0 == 0) break;
      if (level > (uint32_t)kMaxLevelOfTree) {
        err |= kErrRounds;
        break;
      }
      const uint32_t n = n0 < a.sep_cap ? n0 : (uint32_t)a.sep_cap;
      const uint32_t per = level_per(n, nb);
      const uint32_t nchunks = (n + per - 1) / per;
      uint32_t dl = 0, sq = 0;
      for (uint32_t rr = solo ? sq++ : block_claim(&ctl->tk[par][1 + level][0], &s_tk);
           rr < nchunks; rr = solo ? sq++ : block_claim(&ctl->tk[par][1 + level][0], &s_tk)) {
        if (t == 0) ++dl;
        upper_chunk(a, L, s_lvl, s_red, n, per, rr, level, base, cap, err);
      }
      stamp();
      okl = solo ? block_fence() : handoff(ctl, par, 1 + level, dl, nchunks, false, s_red, &s_flag);
      stamp();
    }
    return okl;
  };
  if (ok && total && fits && !direct) ok = run_levels(false);
  if (!ok) err |= kErrHandoff;
  // the chunk's deletes, after every split (Tree::del, Tree.cpp:542-591):
  // the keys are located afresh, so pages that moved right are followed; the
  // leaf level ended with a hand-off, so no leaf is still being written.
  // Nothing waits for them: dealt statically
  for (uint64_t i = wid; ok && i < n_del; i += W) delete_key(a, a.dk[i], L.page, err);
  if (err && lane == 0) atomicOr(a.err, err);
  err = 0;
  stamp();
  // the last block to finish writes the superblock: every block's
  // allocations and root growth are in the counters by then
  __syncthreads();
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the write-back before the arrival
    const uint32_t d = __hip_atomic_fetch_add(&ctl->done[par][0], 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    s_flag = (d == nb - 1 ? 1u : 0u) |
             (d == nb - 1 && __hip_atomic_load(&ctl->abort[par][0], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)
                  ? 2u
                  : 0u);
  }
  __syncthreads();
  const uint32_t last = s_flag;
  __syncthreads();
  if (last & 2u) {
    // A hand-off gave up (its wait bound, or force_abort).  Every block has
    // finished, so every task any block took is done: this block alone runs
    // the internal levels again from level 1 (re-inserting a separator a page
    // already holds rewrites it unchanged) and the deletes (deleting an absent
    // key changes nothing), so the chunk completes in this launch, before any
    // later call reads the tree -- nothing is dropped (the reference always
    // completes a parent insert, Tree.cpp:973-988).
    block_fence();
    if (total && fits && !direct) (void)run_levels(true);
    for (uint64_t i = (uint64_t)wv; i < n_del; i += kUpWaves) delete_key(a, a.dk[i], L.page, err);
    if (err && lane == 0) atomicOr(a.err, err);
    block_fence();
    if (t == 0) atomicAdd(a.err + 2, 1u);  // chunks completed this way (shm_last_error)
  }
  if (bclk) bclk[256] = wall_clock64();
  if ((last & 1u) && t == 0) {
    // superblock (device-authoritative) and its host mirror
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const uint64_t extra = total && fits ? __hip_atomic_load(&ctl->alloc[par][0], __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT)
                                         : 0ull;
    uint64_t cursor = total && fits ? base + extra : cursor0e;
    if (cursor > cap) cursor = cap;  // failed allocations used no page
    const uint32_t rn =
        __hip_atomic_load(&ctl->root_new[par][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (grow0 && total && fits) root_level = 1;
    if (rn > root_level) root_level = rn;
    const uint64_t made =
        (cursor0e - cursor0) +
        (total && fits ? (uint64_t)total + __hip_atomic_load(&ctl->made[par][0], __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT)
                       : 0ull);
    sb->next_page = cursor;
    sb->root_level = root_level;
    sb->splits = splits0 + made;
    sb->batches = a.batch;
    // the host mirror changes only with new pages.  Relaxed: the host reads
    // each word on its own (tree.cpp mirror) and relies on them only once the
    // stream is idle; a release here cost block 0 ~5 us (PCIe write waits)
    if (a.pub && cursor != cursor0) {
      __hip_atomic_store(a.pub + 1, cursor, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(a.pub + 2, (uint64_t)root_level, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(a.pub + 3, splits0 + made, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (a.pub && (cursor != cursor0 || a.pub_always))
      __hip_atomic_store(a.pub + 0, a.batch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // every block's error bits are in (released before its `done` arrival):
    // the first chunk to see a bit other than kErrKeyMax names itself
    if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~kErrKeyMax)
      atomicCAS(a.err + 1, 0u, (uint32_t)a.batch);
    // every block has finished (the `done` count): the op buffers are free
    if (a.pub)
      __hip_atomic_store(a.pub + kPubApplied, a.batch, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// LeafPage() + set_consistent (Tree.cpp:47-52)
__global__ void k_empty_leaf(uint8_t* arena, uint64_t off, uint8_t* sum) {
  __shared__ __attribute__((aligned(16))) uint32_t lp[kPageDwords + 8];
  init_page_image(lp, 1, 0, 0, 0, -1, kKeyMin, kKeyMax);
  wave_lds_sync();
  if (lane_id() == 0) lp[kOffLeafRear / 4] = 1;
  store_page(arena, off, lp);
  put_leaf_sum(sum, off, kKeyMax, 0);
}

__global__ void k_write_superblock(uint8_t* arena, Superblock sb) {
  if (threadIdx.x == 0) *reinterpret_cast<Superblock*>(arena) = sb;
}

// ---------------------------------------------------------------------------
uint32_t upper_blocks() {
  static const uint32_t nb = [] {
    int cus = 0, dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int n = cus > 0 ? cus : 256;
    return (uint32_t)(n < kMaxUpper ? n : kMaxUpper);
  }();
  return nb;
}

// a block of k_upper fits a CU at all (nothing more is needed: no phase
// waits for blocks that are not running)
bool upper_resident() {
  int nb = 0;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_upper, kUpT, 0) == hipSuccess &&
         nb >= 1;
}

void launch_upper(const UpperArgs& a, hipStream_t s) {
  // one block per CU (fewer may be resident: tickets and hand-offs, above);
  // 512 threads, ~66 KB of LDS
  hipLaunchKernelGGL(k_upper, dim3(upper_blocks()), dim3(kUpT), 0, s, a);
}

void launch_write_superblock(uint8_t* arena, const Superblock& sb, hipStream_t s) {
  hipLaunchKernelGGL(k_write_superblock, dim3(1), dim3(kWave), 0, s, arena, sb);
}
void launch_empty_leaf(uint8_t* arena, uint64_t off, uint8_t* sum, hipStream_t s) {
  hipLaunchKernelGGL(k_empty_leaf, dim3(1), dim3(kWave), 0, s, arena, off, sum);
}

}  // namespace dev
}  // namespace shm
