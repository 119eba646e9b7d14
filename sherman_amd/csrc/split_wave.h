// split_wave.h — wave-level leaf / internal split machinery shared by the
// upsert kernel (upsert.hip: small splits taken at once, "early") and
// k_upper (insert.hip).  See insert.hip for the algorithm and its
// reference citations.
#pragma once
#include "device_common.h"
#include "kernels.h"

namespace shm {
namespace dev {

namespace {

constexpr int kUpT = 512;                  // threads per k_upper block
constexpr int kUpWaves = kUpT / kWave;     // 8 waves
constexpr uint32_t kFanSpins = 1u << 22;

struct WaveLds {
  uint32_t page[kPageDwords + 8];
  uint64_t a_key[kWave];
  uint64_t a_val[kWave];
  uint32_t a_ver[kWave];
  uint64_t o_key[kWave];  // a segment's ops staged (stage_ops); propagate's run
  uint64_t o_val[kWave];
  uint64_t r_key[kWave];  // separators a direct propagation made (the next run)
  uint64_t r_ptr[kWave];
};

__device__ __forceinline__ uint32_t lock_index(uint64_t page, uint32_t n) {
  return (uint32_t)(cityhash64_u64(page) % n);
}

// Lock words (the reference's lock table, Tree.cpp:205-264) are epoch
// tagged: a word holding a value <= the chunk's tag (chunk number << 32) is
// free for the chunk.  An exclusive hold is tag | 1 (lock_excl: one
// atomicMax that returns a free value exactly when it took the word; the
// deletes: a CAS of a free value), bounded by kMaxLockSpins (kErrLock), and
// is handed back at the chunk's tag.  The next chunk's larger tag frees every
// word of this one, including the upsert kernel's shared holds (upsert.hip).
// the ops of one segment: keys [st, st + nb) of a sorted unique op array
struct Ops {
  const uint64_t* key;
  const uint64_t* val;
  uint32_t st, nb;
};

__device__ __forceinline__ bool op_contains(const Ops& o, uint64_t key) {
  const uint64_t i = lower_bound64(o.key, o.st, (uint64_t)o.st + o.nb, key);
  return i < (uint64_t)o.st + o.nb && o.key[i] == key;
}

// Surviving entries of the staged leaf (valid, not overwritten by an op),
// sorted by key into L.a_* ; returns their count.
__device__ __forceinline__ int leaf_survivors(WaveLds& L, const Ops& o) {
  const int lane = lane_id();
  const LeafEnt e = leaf_entry(L.page, lane < kLeafCardinality ? lane : 0);
  bool keep = lane < kLeafCardinality && e.val != kValueNull;
  if (keep && op_contains(o, e.key)) keep = false;
  uint64_t key = keep ? e.key : kKeyMax;
  uint32_t tag = (uint32_t)lane;
  wave_sort64(key, tag);
  const uint64_t v = shfl64(e.val, (int)tag);
  const uint32_t ver = shfl32(e.fraw | (e.rraw << 8), (int)tag);
  const int na = popc64(ballot(keep));
  L.a_key[lane] = key;
  L.a_val[lane] = v;
  L.a_ver[lane] = ver;
  wave_lds_sync();
  return na;
}

// Surviving records of an internal page (lane slice w), in key order.
__device__ __forceinline__ int internal_survivors(WaveLds& L, const u32x4 w, int cnt, const Ops& o) {
  const int lane = lane_id();
  const IntRec r = internal_record(w);
  bool keep = lane >= 3 && lane - 3 < cnt;
  if (keep && op_contains(o, r.key)) keep = false;
  const uint64_t km = ballot(keep);
  if (keep) {
    const int pos = popc64(km & lanemask_lt());
    L.a_key[pos] = r.key;
    L.a_val[pos] = r.ptr;
    L.a_ver[pos] = 0;
  }
  wave_lds_sync();
  return popc64(km);
}

// Element r of merge(A = survivors (na), B = ops); keys are disjoint.
// Merge-path binary search (distinct keys).
__device__ __forceinline__ void merged_elem(const WaveLds& L, int na, const Ops& o, uint32_t r,
                                            uint64_t& key, uint64_t& val, uint32_t& ver) {
  const uint32_t nb = o.nb, st = o.st;
  uint32_t lo = r > nb ? r - nb : 0;
  uint32_t hi = r < (uint32_t)na ? r : (uint32_t)na;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (L.a_key[mid] < o.key[st + r - mid - 1])
      lo = mid + 1;
    else
      hi = mid;
  }
  const uint32_t i = lo, j = r - lo;
  if (i < (uint32_t)na && (j >= nb || L.a_key[i] < o.key[st + j])) {
    key = L.a_key[i];
    val = L.a_val[i];
    ver = L.a_ver[i];
  } else {
    key = o.key[st + j];
    val = o.val[st + j];
    ver = 0;  // fresh LeafEntry() in the sibling (Tree.cpp:934, 944-948)
  }
}

// one page of a k-way split: page p of P of a segment with T entries after
// the batch; new page q >= 1 sits at arena page first_new + q - 1
struct SplitPage {
  int p, P;
  uint32_t T;
  uint64_t first_new;
  uint64_t dest;  // GlobalAddress written (page 0: the segment's page, or X)
};

__device__ __forceinline__ uint64_t new_ga(uint16_t node, uint64_t first_new, int q) {
  return ga_make(node, (first_new + (uint64_t)(q - 1)) * kPageSize);
}

// Write leaf page p of the split (survivors in L.a_*); returns its lowest
// fence (the separator of p > 0, copied up as in Tree.cpp:939-950).
__device__ __forceinline__ uint64_t build_leaf_page(const UpperArgs& a, WaveLds& L, const Hdr& h, int na,
                                    const Ops& o, const SplitPage& s) {
  const int lane = lane_id();
  const uint32_t base = s.T / (uint32_t)s.P, rem = s.T % (uint32_t)s.P;
  const uint32_t p = (uint32_t)s.p;
  const uint32_t c = base + (p < rem ? 1u : 0u);
  const uint32_t s0 = p * base + (p < rem ? p : rem);
  uint64_t key = 0, val = 0;
  uint32_t ver = 0;
  const bool has_next = s.p + 1 < s.P;
  if ((uint32_t)lane < c || ((uint32_t)lane == c && has_next))
    merged_elem(L, na, o, s0 + (uint32_t)lane, key, val, ver);
  const uint64_t lowest = s.p == 0 ? h.lowest : rl64(key, 0);
  const uint64_t highest = has_next ? rl64(key, (int)c) : h.highest;
  const uint64_t sibling = has_next ? new_ga(a.node, s.first_new, s.p + 1) : h.sibling;
  const uint32_t fver = s.p == 0 ? ((h.fver + 1) & 0xFF) : 1u;
  wave_lds_sync();
  init_page_image(L.page, fver, 0, sibling, 0, (int32_t)c - 1, lowest, highest);
  wave_lds_sync();
  if ((uint32_t)lane < c) put_leaf_entry(L.page, lane, key, val, ver & 0xFF, ver >> 8);
  if (lane == 0) L.page[kOffLeafRear / 4] = fver;  // rear_version, byte 1016
  store_page(a.arena, ga_offset(s.dest), L.page);
  if (a.leaf_hw && lane == 0) a.leaf_hw[ga_offset(s.dest) >> 10] = (uint8_t)c;  // slots [0, c)
  // every slot < c is valid (value != 0: deletes never reach a split page)
  put_leaf_sum(a.sum, ga_offset(s.dest), highest, (uint32_t)lane < c ? key_fp(key) : 0u);
  return lowest;
}

// An internal page written through to memory (8-B agent-scope relaxed
// atomic stores = global_store ... sc1, two per lane): waves on other XCDs
// read internal pages under the page's lock word (apply_run) or lock-free
// (parent_of), so their stores must not wait in this XCD's L2 for a
// release fence.  The writer drains them (s_waitcnt vmcnt(0)) before it
// hands the word back (unlock_excl) -- MI355X_MICROARCH.md "visibility",
// cdna_hip_programming.md §6 Guideline 16, R1 -- so unlocking needs no
// buffer_wbl2 of the whole L2.
__device__ __forceinline__ void store_page_wt(uint8_t* arena, uint64_t off, const uint32_t* lp) {
  wave_lds_sync();
  const int l = lane_id();
  const uint64_t* src = reinterpret_cast<const uint64_t*>(lp);
  uint64_t* dst = reinterpret_cast<uint64_t*>(arena + off);
  const uint64_t w0 = src[l], w1 = src[kWave + l];
  __hip_atomic_store(dst + l, w0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(dst + kWave + l, w1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The lane's 16 B of a page that other waves write through (store_page_wt)
// under its lock word: agent-scope relaxed loads (global_load ... sc1), so
// the locker needs no L1-invalidating acquire before reading the page
__device__ __forceinline__ u32x4 load_page_slice_wt(const uint8_t* arena, uint64_t off) {
  const uint64_t* p = reinterpret_cast<const uint64_t*>(arena + off + 16 * lane_id());
  const uint64_t x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t y = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return u32x4{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32)};
}

// Internal page p of the split: q = T - (P - 1) records stay, one record per
// extra page is pushed up (its ptr becomes that page's leftmost, its key the
// separator, Tree.cpp:779-793).  Returns the page's lowest fence.
__device__ __forceinline__ uint64_t build_internal_page(const UpperArgs& a, WaveLds& L, const Hdr& h, int na,
                                        const Ops& o, const SplitPage& s, uint32_t level) {
  const int lane = lane_id();
  const uint32_t q = s.T - (uint32_t)(s.P - 1);
  const uint32_t base = q / (uint32_t)s.P, rem = q % (uint32_t)s.P;
  const uint32_t p = (uint32_t)s.p;
  const uint32_t c = base + (p < rem ? 1u : 0u);
  const uint32_t s0 = p * base + (p < rem ? p : rem) + p;
  const bool has_next = s.p + 1 < s.P;
  uint64_t key = 0, val = 0;
  uint32_t ver = 0;
  bool want = false;
  uint32_t r = 0;
  if ((uint32_t)lane < c) {
    want = true;
    r = s0 + (uint32_t)lane;
  } else if (lane == 62 && s.p > 0) {
    want = true;
    r = s0 - 1;  // record pushed up to the parent; its ptr becomes leftmost
  } else if (lane == 63 && has_next) {
    want = true;
    r = s0 + c;  // next page's pushed-up key = this page's highest
  }
  if (want) merged_elem(L, na, o, r, key, val, ver);
  const uint64_t leftmost = s.p == 0 ? h.leftmost : rl64(val, 62);
  const uint64_t lowest = s.p == 0 ? h.lowest : rl64(key, 62);
  const uint64_t highest = has_next ? rl64(key, 63) : h.highest;
  const uint64_t sibling = has_next ? new_ga(a.node, s.first_new, s.p + 1) : h.sibling;
  const uint32_t fver = s.p == 0 ? ((h.fver + 1) & 0xFF) : 1u;
  wave_lds_sync();
  init_page_image(L.page, fver, leftmost, sibling, level, (int32_t)c - 1, lowest, highest);
  wave_lds_sync();
  if ((uint32_t)lane < c) {
    uint32_t* d = L.page + (kOffRecords + kInternalEntry * lane) / 4;
    d[0] = (uint32_t)key;
    d[1] = (uint32_t)(key >> 32);
    d[2] = (uint32_t)val;
    d[3] = (uint32_t)(val >> 32);
  }
  if (lane == 0) L.page[kOffInternalRear / 4] = fver;  // byte 1020
  store_page_wt(a.arena, ga_offset(s.dest), L.page);
  if (a.leaf_hw && lane == 0) a.leaf_hw[ga_offset(s.dest) >> 10] = kLeafHwFull;
  return lowest;
}

// The root page becomes the new internal root one level up, {leftmost = X}
// with no records (update_new_root, Tree.cpp:126-149); the level's separators
// are then inserted into it by the next level.
__device__ __forceinline__ void write_new_root(const UpperArgs& a, WaveLds& L, uint64_t x, uint32_t level,
                               uint32_t old_fver) {
  wave_lds_sync();
  init_page_image(L.page, (old_fver + 1) & 0xFF, x, 0, level, -1, kKeyMin, kKeyMax);
  wave_lds_sync();
  if (lane_id() == 0) L.page[kOffInternalRear / 4] = (old_fver + 1) & 0xFF;
  store_page_wt(a.arena, ga_offset(a.root), L.page);
  if (a.leaf_hw && lane_id() == 0) a.leaf_hw[ga_offset(a.root) >> 10] = kLeafHwFull;
  // the root page is internal now: its summary no longer describes a leaf
  if (lane_id() == 0) clear_leaf_sum(a.sum, ga_offset(a.root));
}

// The directory's page of `level` (1 or 2) on the path of k's prefix
// (k_leaf_dir records them), 0 when there is none: a B-link starting point
__device__ __forceinline__ uint64_t dir_hint_page(const UpperArgs& a, uint64_t k, uint32_t level) {
  if (!a.dir_hint || level < 1 || level > 2 || !dir_covers(a.dir_lo, a.dir_shift, a.dir_n, k))
    return 0;
  const uint32_t pg = a.dir_hint[(uint64_t)(level - 1) * a.dir_n + ((k - a.dir_lo) >> a.dir_shift)];
  return pg ? dir_page_ga(pg, a.node) : 0ull;
}

// The page of `level` whose fences hold k: header walk from the root with
// page_search's sibling rule (Tree.cpp:593-663) and internal_page_search
// (665-685), one wave.  0 on an inconsistency (error bits in *err).
// soft: a starting point only (the caller re-checks under the page's lock):
// a failure returns 0 without error bits
__device__ __forceinline__ uint64_t parent_of(const UpperArgs& a, uint64_t k, uint32_t level, uint32_t* err,
                              bool soft = false) {
  uint32_t scratch = 0;
  if (soft) err = &scratch;
  uint64_t ptr = a.root;
  // start at the level's page on the path of k's directory prefix (a page
  // keeps its lowest fence when it splits, so a stale hint is still a valid
  // B-link start); a hint whose page is no longer at `level` (the root page
  // grew a level) restarts from the root
  bool hinted = false;
  if (a.dir_hint && level >= 1 && level <= 2 && dir_covers(a.dir_lo, a.dir_shift, a.dir_n, k)) {
    const uint32_t pg = a.dir_hint[(uint64_t)(level - 1) * a.dir_n + ((k - a.dir_lo) >> a.dir_shift)];
    if (pg) {
      ptr = dir_page_ga(pg, a.node);
      hinted = true;
    }
  }
  int retries = 0;
  for (int hop = 0; hop < kMaxRounds; ++hop) {
    if (!ptr_ok(ptr, a.node, a.arena_bytes)) {
      *err |= kErrBadPtr;
      return 0;
    }
    const u32x4 w = load_page_slice(a.arena, ga_offset(ptr));
    const Hdr h = parse_hdr(w);
    const bool is_leaf = h.leftmost == 0;
    if (h.fver != (is_leaf ? h.rver_leaf : h.rver_internal)) {
      if (++retries > kMaxRetries) {
        *err |= kErrInconsistent;
        return 0;
      }
      // a page rewritten by another wave of this launch: drop cached lines
      // of it before reading again (L2 is per XCD and not coherent)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      continue;
    }
    if (hinted && (h.level != level || k < h.lowest)) {  // not this level's page any more
      hinted = false;
      ptr = a.root;
      continue;
    }
    if (k >= h.highest && h.sibling != 0) {  // turn right (Tree.cpp:626-629)
      ptr = h.sibling;
      continue;
    }
    if (k < h.lowest || k >= h.highest || h.level < level) {
      *err |= kErrFence;
      return 0;
    }
    if (h.level == level) return ptr;
    // child = #keys <= k (keys strictly increase; record j in lane j + 3)
    const IntRec r = internal_record(w);
    const int cnt = h.last_index + 1;
    const uint64_t le = ballot(lane_id() >= 3 && lane_id() - 3 < cnt && r.key <= k);
    const int pos = popc64(le);
    ptr = pos == 0 ? h.leftmost : rl64(r.ptr, pos + 2);
  }
  *err |= kErrRounds;
  return 0;
}

// ---- block / grid helpers (kUpT threads) ------------------------------------
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off);
  __syncthreads();
  if (lane_id() == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kUpWaves; ++i) s += red[i];
  return s;
}

// exclusive block scan; *total = block sum
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t* red, uint32_t* total) {
  uint32_t incl = v;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, off);
    if (lane_id() >= off) incl += y;
  }
  __syncthreads();
  if (lane_id() == kWave - 1) red[threadIdx.x >> 6] = incl;
  __syncthreads();
  uint32_t base = 0, all = 0;
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < kUpWaves; ++i) {
    base += i < w ? red[i] : 0u;
    all += red[i];
  }
  *total = all;
  return base + incl - v;
}

// ---- phase tickets and hand-offs ----------------------------------------------
// k_upper never needs its blocks to be resident together.  A phase whose
// results a later phase reads hands its tasks out by ticket: a running wave
// (or block) takes the next task of the phase with one atomic add, in
// dispatch order, and counts it finished when its stores are done.  A block
// that has run out of tickets waits at the hand-off until the phase's
// finished count reaches its task count.  Every task it waits for was taken
// by a wave that is running (tickets are only taken by running waves) and
// that finishes it without waiting on anything but lock words held by other
// running waves and, for a large split's page 0, the sibling builders of the
// previous phase (all of whose tasks were taken before any task of this phase
// was).  So the launch drains with any number of resident blocks, one
// included: beside another process's persistent kernels, RCCL kernels or a
// kernel holding most CUs (tests/test_gpu_parity.py::
// test_split_insert_beside_cu_hog) -- the reference's parent insert likewise
// waits only on a page lock (Tree.cpp:205-242, 973-988).  Phases nobody waits
// on (C5's direct propagation) keep the static wave-per-task assignment.

// the wave's next task: lane 0 takes `step` tickets of the phase at once
__device__ __forceinline__ uint32_t wave_claim(uint32_t* tk, uint32_t step) {
  uint32_t v = 0;
  if (lane_id() == 0) v = atomicAdd(tk, step);
  return rl32(v, 0);
}

// the block's next task (thread 0 takes the ticket; slot: LDS broadcast)
__device__ __forceinline__ uint32_t block_claim(uint32_t* tk, uint32_t* slot) {
  __syncthreads();  // every thread has read the previous ticket
  if (threadIdx.x == 0) *slot = atomicAdd(tk, 1u);
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(*slot);  // uniform: loops over it stay single loops
}

constexpr uint32_t kHandoffSpins = 1u << 22;

// the block's stores performed and released, then acquired by every thread
// (the solo pass of the last block, which waits for nobody)
__device__ __forceinline__ bool block_fence() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

// Phase hand-off: the block adds the tasks it finished (`mine`, summed over
// its threads' values) to the phase's count after its stores are performed
// and released, then waits until `want` tasks are finished; acquire.  False
// (every thread) when a wait gave up (kHandoffSpins, or another block gave
// up, or force): the abort word tells every block to leave at its next
// hand-off, and the launch's last block completes the chunk alone.
__device__ __forceinline__ bool handoff(UpperCtl* ctl, uint32_t par, uint32_t ph, uint32_t mine,
                                        uint32_t want, bool force, uint32_t* red,
                                        uint32_t* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint32_t sum = block_sum(mine, red);
  if (threadIdx.x == 0) {
    uint32_t* abort = &ctl->abort[par][0];
    uint32_t* d = &ctl->dn[par][ph][0];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the write-back before the count
    if (sum) __hip_atomic_fetch_add(d, sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t ok = force ? 0u : 1u;
    for (uint32_t spin = 0; ok; ++spin) {
      if (__hip_atomic_load(d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) break;
      if (__hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
          spin > kHandoffSpins)
        ok = 0;
      else
        __builtin_amdgcn_s_sleep(1);
    }
    if (ok && __hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ok = 0;
    if (!ok) __hip_atomic_store(abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    *flag = ok;
  }
  __syncthreads();
  return *flag != 0;
}

// last index s in [0, n) with base[s] <= x (base non-decreasing, base[0] = 0)
__device__ __forceinline__ uint32_t last_le(const uint32_t* base, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (base[mid] <= x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo - 1;
}

// [first, end) of block b's share of n items (the upsert kernel assigns item g
// to range g * nb / n, i.e. exactly these)
__device__ __forceinline__ void block_range(uint32_t n, uint32_t b, uint32_t nb, uint32_t& r0,
                                            uint32_t& r1) {
  r0 = (uint32_t)(((uint64_t)b * n + nb - 1) / nb);
  r1 = (uint32_t)(((uint64_t)(b + 1) * n + nb - 1) / nb);
}

// Segment of block range [r0, r1) holding the range's new page j (by_split
// false: the running sum of seg_np passes j) or being its j-th split
// (by_split: the j-th segment with seg_np > 0), one wave; before = the new
// pages of the range's segments ahead of it.  g = r1 if the counts disagree.
__device__ __forceinline__ void find_seg(const uint32_t* np, uint32_t r0, uint32_t r1, uint32_t j, bool by_split,
                         uint32_t& g, uint32_t& before) {
  const int lane = lane_id();
  uint32_t run_c = 0, run_np = 0;
  for (uint32_t c0 = r0; c0 < r1; c0 += kWave) {
    const uint32_t i = c0 + (uint32_t)lane;
    const uint32_t v = i < r1 ? np[i] : 0u;
    uint32_t ic = by_split ? (v ? 1u : 0u) : v, inp = v;  // inclusive scans over the wave
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint32_t yc = (uint32_t)__shfl_up((int)ic, o), yn = (uint32_t)__shfl_up((int)inp, o);
      if (lane >= o) {
        ic += yc;
        inp += yn;
      }
    }
    const uint64_t m = ballot(run_c + ic > j);
    if (m) {
      const int l = ctz64(m);
      g = c0 + (uint32_t)l;
      before = run_np + rl32(inp - v, l);
      return;
    }
    run_c += rl32(ic, kWave - 1);
    run_np += rl32(inp, kWave - 1);
  }
  g = r1;
  before = run_np;
}

// Fan-in counters (a split's sibling builders have read its page 0): one
// word per segment, tag << 32 | count, the tag naming the chunk and level.
// An arrival of a new tag restarts the count, so no word is ever reset and
// a launch that stopped early leaves nothing a later one could miscount.
__device__ __forceinline__ void fan_arrive(uint64_t* w, uint32_t tag) {
  unsigned long long* p = reinterpret_cast<unsigned long long*>(w);
  unsigned long long old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    const unsigned long long nv = (uint32_t)(old >> 32) == tag
                                      ? old + 1ull
                                      : (((unsigned long long)tag << 32) | 1ull);
    const unsigned long long prev = atomicCAS(p, old, nv);
    if (prev == old) return;
    old = prev;
  }
}
// wait until the word reads (tag, want); the builders it waits for took
// their tasks (phase 0 tickets) before this wave took its phase-1 one
__device__ __forceinline__ bool fan_in(uint64_t* cnt, uint32_t want, uint32_t tag) {
  const uint64_t target = ((uint64_t)tag << 32) | want;
  uint32_t ok = 1;
  if (lane_id() == 0) {
    ok = 0;
    for (uint32_t spin = 0; spin < kFanSpins; ++spin) {
      if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == target) {
        ok = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return rl32(ok, 0) != 0;
}
__device__ __forceinline__ uint32_t fan_tag(uint64_t batch, uint32_t level) {
  return (uint32_t)(batch << 3) | level;
}

// Tree::del of one key (leaf_page_del, Tree.cpp:993-1057), one wave: walk
// from the leaf directory (or the root) with page_search's sibling rule, lock
// the leaf's word, re-read it under the lock (turning right again if needed),
// clear the first valid slot holding the key (value = kValueNull, f++ ,
// r = f) and write back that 18 B entry, then release.  Keys are unique in a
// batch, so two waves never touch one entry; they may share a page and
// serialise on its word.
__device__ __forceinline__ void delete_key(const UpperArgs& a, uint64_t k, uint32_t* lp, uint32_t& err) {
  const int lane = lane_id();
  uint64_t ptr = a.root;
  if (a.dir) ptr = dir_start(a.dir, a.dir_lo, a.dir_shift, a.dir_n, a.node, k, ptr);
  bool locked = false;
  uint64_t lw = 0;
  int retries = 0;
  for (int hop = 0;; ++hop) {
    if (hop > kMaxRounds) {
      err |= kErrRounds;
      break;
    }
    if (!ptr_ok(ptr, a.node, a.arena_bytes)) {
      err |= kErrBadPtr;
      break;
    }
    const u32x4 w0 = load_page_slice(a.arena, ga_offset(ptr));
    const Hdr h0 = parse_hdr(w0);
    const bool leaf0 = h0.leftmost == 0;
    if (h0.fver != (leaf0 ? h0.rver_leaf : h0.rver_internal)) {
      if (++retries > kMaxRetries) {
        err |= kErrInconsistent;
        break;
      }
      // an internal page another wave rewrote: drop this XCD's stale lines
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      continue;
    }
    if (k >= h0.highest && h0.sibling != 0) {
      ptr = h0.sibling;
      continue;
    }
    if (k < h0.lowest || k >= h0.highest) {
      err |= kErrFence;
      break;
    }
    if (!leaf0) {
      const IntRec r = internal_record(w0);
      const int cnt = h0.last_index + 1;
      const int pos = popc64(ballot(lane >= 3 && lane - 3 < cnt && r.key <= k));
      ptr = pos == 0 ? h0.leftmost : rl64(r.ptr, pos + 2);
      continue;
    }
    // the leaf: lock_and_read_page (Tree.cpp:1014-1015)
    lw = (uint64_t)lock_index(ptr, a.num_locks);
    uint32_t got = 0;
    if (lane == 0) {
      // free for this delete: any value <= the chunk's tag (an earlier chunk's
      // hold or this chunk's upserts); tag | 1 = another delete of the chunk
      unsigned long long* wd = reinterpret_cast<unsigned long long*>(a.locks) + lw;
      const unsigned long long mine = (unsigned long long)(a.tag | 1ull);
      for (uint32_t spin = 0; spin < kMaxLockSpins; ++spin) {
        const unsigned long long cur =
            __hip_atomic_load(wd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur <= (unsigned long long)a.tag && atomicCAS(wd, cur, mine) == cur) {
          got = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    if (rl32(got, 0) == 0) {
      err |= kErrLock;
      break;
    }
    locked = true;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const u32x4 w = load_page_slice(a.arena, ga_offset(ptr));
    const Hdr h = parse_hdr(w);
    if (h.fver != h.rver_leaf) {
      err |= kErrInconsistent;
      break;
    }
    if (k >= h.highest && h.sibling != 0) {  // Tree.cpp:1028-1032
      if (lane == 0)
        __hip_atomic_store(a.locks + lw, a.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      locked = false;
      ptr = h.sibling;
      continue;
    }
    stage_page(lp, w);
    wave_lds_sync();
    LeafEnt e = leaf_entry(lp, lane < kLeafCardinality ? lane : 0);
    const uint64_t m = ballot(lane < kLeafCardinality && e.key == k && e.val != kValueNull);
    if (m && lane == ctz64(m)) {
      const uint32_t f = ((e.fraw & 0xF) + 1) & 0xF;
      put_leaf_entry(reinterpret_cast<uint32_t*>(a.arena + ga_offset(ptr)), lane, k, kValueNull,
                     (e.fraw & 0xF0) | f, (e.rraw & 0xF0) | f);
      clear_leaf_fp(a.sum, ga_offset(ptr), lane);  // empty
    }
    wave_lds_sync();
    break;
  }
  if (locked) {
    // write_page_and_unlock (Tree.cpp:1049-1052): the entry store first,
    // then the word back at the chunk's tag
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the write-back before the release
      __hip_atomic_store(a.locks + lw, a.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace

// ---- the restructured levels ----------------------------------------------------
// The segment's ops staged in the wave's LDS (<= 64 of them): the merge and
// the survivor test then read LDS instead of making dependent global loads.
__device__ __forceinline__ Ops stage_ops(WaveLds& L, const Ops& o) {
  if (o.nb > (uint32_t)kWave) return o;
  const int lane = lane_id();
  if ((uint32_t)lane < o.nb) {
    L.o_key[lane] = o.key[o.st + lane];
    L.o_val[lane] = o.val[o.st + lane];
  }
  wave_lds_sync();
  return Ops{L.o_key, L.o_val, 0, o.nb};
}

// n pages past the leaf level's (device bump allocation, one atomic per
// call; lane 0 result broadcast): the arena page of the first, or ~0 when
// the arena cannot hold them (kErrNoMem; the pages are not used)
__device__ __forceinline__ uint64_t alloc_pages(const UpperArgs& a, uint64_t base, uint64_t cap,
                                                uint32_t n, uint32_t& err) {
  uint64_t first = 0;
  if (lane_id() == 0) {
    // the upsert kernel's early splits bump their own counter from next_page
    // (base); k_upper's follow the leaf level's pages
    uint64_t* ctr = a.early ? &a.ctl->ualloc[a.par][0] : &a.ctl->alloc[a.par][0];
    first = base + atomicAdd(reinterpret_cast<unsigned long long*>(ctr), (unsigned long long)n);
    if (!a.early)
      atomicAdd(reinterpret_cast<unsigned long long*>(&a.ctl->made[a.par][0]),
                (unsigned long long)n);
  }
  first = rl64(first, 0);
  if (first + n > cap) {
    err |= kErrNoMem;
    return ~0ull;
  }
  return first;
}

// append separator (key, child) with its parent page to level `lvl`'s list
__device__ __forceinline__ void emit_sep(const UpperArgs& a, uint32_t lvl, uint64_t key,
                                         uint64_t child, uint64_t parent, uint32_t& err) {
  if (lane_id() != 0) return;
  const uint32_t j = atomicAdd(&a.ctl->lvl_sep[a.par][lvl], 1u);
  if ((uint64_t)j >= a.sep_cap) {
    err |= kErrPlan;
    return;
  }
  // selects, not a[lvl & 1]: a runtime index into the kernel argument
  // would copy it to scratch
  const bool odd = (lvl & 1) != 0;
  (odd ? a.sep_key[1] : a.sep_key[0])[j] = key;
  (odd ? a.sep_ptr[1] : a.sep_ptr[0])[j] = child;
  (odd ? a.ipage[1] : a.ipage[0])[j] = parent;
}

// the page's lock word held exclusively (tag | 1, as the deletes take it;
// free = any value <= the chunk's tag), released at the chunk's tag
__device__ __forceinline__ bool lock_excl(const UpperArgs& a, uint64_t page) {
  uint32_t got = 0;
  if (lane_id() == 0) {
    unsigned long long* wd =
        reinterpret_cast<unsigned long long*>(a.locks) + lock_index(page, a.num_locks);
    const unsigned long long mine = (unsigned long long)(a.tag | 1ull);
    // one round trip: max(word, tag | 1) returns a free value (<= tag: an
    // earlier chunk's, or this chunk's shared / handed-back hold) exactly
    // when this wave took it; tag | 1 back means another wave holds it
    for (uint32_t spin = 0; spin < kMaxLockSpins; ++spin) {
      if (atomicMax(wd, mine) <= (unsigned long long)a.tag) {
        got = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  // no acquire: the holder reads the page with sc1 loads (load_page_slice_wt)
  // and its previous holders wrote it through (store_page_wt)
  got = rl32(got, 0);
  return got != 0;
}
__device__ __forceinline__ void unlock_excl(const UpperArgs& a, uint64_t page) {
  // the page's write-through stores (store_page_wt) performed: the next
  // holder's sc1 loads (load_page_slice_wt) see them, no L2 write-back needed
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane_id() == 0)
    __hip_atomic_store(a.locks + lock_index(page, a.num_locks), a.tag, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// One internal page of `level` receives the ops o (sorted separators, their
// children), the survivors already in L.a_*: rewritten in place when they
// fit (T <= 60), else split into P pages, new right siblings first, page 0
// last (Tree.cpp:699-826 for a batch of separators), new separators emitted
// to the next level; the root splits into a fresh page X and becomes the new
// root one level up (update_new_root, Tree.cpp:126-149).
// direct (propagate): the new separators go to the wave's L.r_* from index
// nout on (the next level's run, in key order) instead of the level's list.
// Returns nout plus the separators it put there.
__device__ __forceinline__ uint32_t apply_internal(const UpperArgs& a, WaveLds& L, const Hdr& h, int na,
                                   const Ops& o, uint64_t page, uint32_t level, uint64_t base,
                                   uint64_t cap, uint32_t& err, bool direct = false,
                                   uint32_t nout = 0) {
  const uint32_t T2 = (uint32_t)na + o.nb;
  const uint32_t P = T2 <= (uint32_t)(kInternalCardinality - 1)
                         ? 1u
                         : (T2 + 1 + kInternalSplitFill) / (kInternalSplitFill + 1);
  if (P == 1) {
    (void)build_internal_page(a, L, h, na, o, SplitPage{0, 1, T2, 0, page}, level);
    return nout;
  }
  const bool grow = page == a.root;
  const uint64_t first = alloc_pages(a, base, cap, P - 1 + (grow ? 1u : 0u), err);
  if (first == ~0ull) return nout;  // no room: the page stays as it was (reported)
  for (uint32_t p = 1; p < P; ++p) {
    const SplitPage sp{(int)p, (int)P, T2, first, new_ga(a.node, first, (int)p)};
    const uint64_t low = build_internal_page(a, L, h, na, o, sp, level);
    if (direct) {
      if (nout >= (uint32_t)kWave) {
        err |= kErrPlan;  // cannot happen from runs of <= kSmallSplit - 1
      } else {
        if (lane_id() == 0) {
          L.r_key[nout] = low;
          L.r_ptr[nout] = sp.dest;
        }
        ++nout;
      }
      continue;
    }
    const uint64_t par = grow ? a.root : parent_of(a, low, level + 1, &err);
    emit_sep(a, level + 1, low, sp.dest, par, err);
  }
  const uint64_t dest0 = grow ? ga_make(a.node, (first + P - 1) * kPageSize) : page;
  // the new right siblings land before page 0 points at them (Tree.cpp:962:
  // the sibling is written before the relink), for lock-free parent walks
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  (void)build_internal_page(a, L, h, na, o, SplitPage{0, (int)P, T2, first, dest0}, level);
  if (grow) {
    write_new_root(a, L, dest0, level + 1, h.fver);
    if (lane_id() == 0) atomicMax(&a.ctl->root_new[a.par][0], level + 1);
  }
  return nout;
}

// Level >= 2: a run of separators (sorted keys [hs, he) of the block's LDS
// list, one parent hint) applied under the parent's exclusive word, as
// internal_page_store does (Tree.cpp:699-826: lock, read, turn right past
// the highest fence, insert, split at 61) for a batch.  Separators of one
// parent may sit in several blocks' lists: their runs serialise on the
// word.  The ops below the page's highest fence go in; the rest move right
// (B-link); a page no longer at `level` (the root grew, or a page another
// wave has just created is not visible yet) is found again from the root.
// direct: as apply_internal; returns the separators made (direct only).
// held: the caller already holds `page`'s exclusive word (a valid page)
__device__ __forceinline__ uint32_t apply_run(const UpperArgs& a, WaveLds& L, const uint64_t* keys,
                              const uint64_t* ptrs, uint32_t hs, uint32_t he, uint64_t page,
                              uint32_t level, uint64_t base, uint64_t cap, uint32_t& err,
                              bool direct = false, bool held = false) {
  uint32_t nout = 0;
  for (int hop = 0; hs < he; ++hop) {
    if (hop >= kMaxRounds) {
      err |= kErrRounds;
      if (held) unlock_excl(a, page);
      return nout;
    }
    if (!held && !ptr_ok(page, a.node, a.arena_bytes)) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      page = parent_of(a, keys[hs], level, &err, true);
      continue;
    }
    if (held) {
      held = false;  // taken by the caller for this first page
    } else if (!lock_excl(a, page)) {
      err |= kErrLock;
      return nout;
    }
    const u32x4 w = load_page_slice_wt(a.arena, ga_offset(page));
    const Hdr h = parse_hdr(w);
    const uint64_t k0 = keys[hs];
    if (h.leftmost == 0 || h.level != level || h.fver != h.rver_internal || k0 < h.lowest) {
      unlock_excl(a, page);
      page = parent_of(a, k0, level, &err, true);
      continue;
    }
    // ops of this page: keys below its highest fence (all if it is the last)
    uint32_t m = he;
    if (h.sibling != 0) {
      for (uint32_t c = hs; c < he; c += kWave) {
        const uint32_t j = c + (uint32_t)lane_id();
        const uint64_t mk = ballot(j < he && keys[j] >= h.highest);
        if (mk) {
          m = c + (uint32_t)ctz64(mk);
          break;
        }
      }
    }
    if (m > hs) {
      const Ops o{keys, ptrs, hs, m - hs};
      const int na = internal_survivors(L, w, h.last_index + 1, o);
      nout = apply_internal(a, L, h, na, o, page, level, base, cap, err, direct, nout);
    }
    unlock_excl(a, page);
    hs = m;
    page = h.sibling;  // Tree.cpp:737-743
  }
  return nout;
}

// Direct propagation (every split of the chunk small): the separators one
// wave made, L.r_*[0, n) in key order, go into `level` at once under the
// parents' exclusive words, and the separators that makes go one level up,
// by the same wave, until a level takes its run in place -- the reference's
// recursive internal_page_store (Tree.cpp:699-826, 804-812), a run at a time.
// No list and no grid barrier: waves meet only on a shared parent's word.
// A run of <= kSmallSplit - 1 separators splits each page it touches at most
// once, so every level's run stays that short (the 64-entry LDS bound).
// held1: the caller holds hint1's exclusive word (taken while it built the
// leaf pages, so the word's round trip is off the chain)
__device__ __forceinline__ void propagate(const UpperArgs& a, WaveLds& L, uint32_t n, uint32_t level,
                          uint64_t base, uint64_t cap, uint32_t& err, uint64_t hint1 = 0,
                          bool held1 = false) {
  for (; n; ++level) {
    if (level > (uint32_t)kMaxLevelOfTree) {
      err |= kErrRounds;
      return;
    }
    const int lane = lane_id();
    wave_lds_sync();
    if ((uint32_t)lane < n) {
      L.o_key[lane] = L.r_key[lane];
      L.o_val[lane] = L.r_ptr[lane];
    }
    wave_lds_sync();
    // the parent: level 1 starts straight at the directory's level-1 page
    // for the run's prefix (read before the leaf builds); otherwise a header
    // walk.  Either is a hint: apply_run re-checks it under the word and
    // moves right or relocates
    const uint64_t hint =
        level == 1 && hint1 ? hint1 : parent_of(a, L.o_key[0], level, &err, true);
    n = apply_run(a, L, L.o_key, L.o_val, 0, n, hint, level, base, cap, err, true,
                  level == 1 && held1);
  }
}

// ---- early splits (upsert.hip) ----------------------------------------------------
// A segment the upsert kernel found would split into P <= kSmallSplit pages,
// queued in its block's LDS and built by a wave of the same block once the
// block's in-place groups are done (Tree.cpp:922-991 for one leaf, its
// separators taken up at once as propagate does).  Its new pages were
// taken when it was queued: arena pages first .. first + P - 2.
struct EarlyItem {
  uint64_t page;   // the leaf (page 0 of the split, rewritten in place)
  uint64_t first;  // arena page of new page 1
  uint64_t hint1;  // the directory's level-1 page for the first op key (0: none)
  uint32_t st, nb;  // the segment's ops [st, st + nb)
  uint32_t T;       // entries after the batch
  uint32_t pv;      // P | front_version << 8 (as the upsert kernel read it)
};

// One early split, one wave (L: the wave's LDS); base = the superblock's
// next_page (early allocations count from it).  Returns error bits.
// clk (diagnostic, nullable): lane 0 records the wall clock at the start,
// once the page is staged, after the builds, once the parent's word is
// known and at the end, words 1024 apart
__device__ __forceinline__ uint32_t split_early(const UpperArgs& a, WaveLds& L,
                                                const EarlyItem& it, uint64_t base,
                                                uint64_t cap, uint64_t* clk = nullptr) {
  uint32_t err = 0;
  const int lane = lane_id();
  if (clk && lane == 0) clk[0] = wall_clock64();
  const int P = (int)(it.pv & 0xFFu);
  const uint32_t ver = it.pv >> 8;
  // the page, the ops (<= 64 staged) and the parent's word, in one round trip
  const bool few = it.nb <= (uint32_t)kWave;
  uint64_t ok0 = 0, ov0 = 0;
  if (few && (uint32_t)lane < it.nb) {
    ok0 = a.op_key[it.st + lane];
    ov0 = a.op_val[it.st + lane];
  }
  const u32x4 w = load_page_slice(a.arena, ga_offset(it.page));
  const bool pre = it.hint1 != 0 && ptr_ok(it.hint1, a.node, a.arena_bytes);
  unsigned long long lk_old = ~0ull;
  if (pre && lane == 0)
    lk_old = atomicMax(reinterpret_cast<unsigned long long*>(a.locks) +
                           lock_index(it.hint1, a.num_locks),
                       (unsigned long long)(a.tag | 1ull));
  const Hdr h = parse_hdr(w);
  const bool room = it.first + (uint64_t)(P - 1) <= cap;
  if (!room || h.fver != ver || h.fver != h.rver_leaf || P < 2) {
    // no room in the arena (the segment stays as it was, reported), or the
    // page is not the one the upsert kernel planned from (cannot happen)
    err |= room ? kErrPlan : kErrNoMem;
    if (pre && rl64((uint64_t)lk_old, 0) <= a.tag) unlock_excl(a, it.hint1);
    return err;
  }
  stage_page(L.page, w);
  if (few && (uint32_t)lane < it.nb) {
    L.o_key[lane] = ok0;
    L.o_val[lane] = ov0;
  }
  wave_lds_sync();
  if (clk && lane == 0) clk[1024] = wall_clock64();
  const Ops o = few ? Ops{L.o_key, L.o_val, 0, it.nb} : Ops{a.op_key, a.op_val, it.st, it.nb};
  const int na = leaf_survivors(L, o);
  for (int p = 1; p < P; ++p) {
    const SplitPage sp{p, P, it.T, it.first, new_ga(a.node, it.first, p)};
    const uint64_t low = build_leaf_page(a, L, h, na, o, sp);
    if (lane == 0) {
      L.r_key[p - 1] = low;
      L.r_ptr[p - 1] = sp.dest;
    }
  }
  (void)build_leaf_page(a, L, h, na, o, SplitPage{0, P, it.T, it.first, it.page});
  if (clk && lane == 0) clk[2 * 1024] = wall_clock64();
  const bool held = pre && rl64((uint64_t)lk_old, 0) <= a.tag;
  if (clk && lane == 0) clk[3 * 1024] = wall_clock64() | (held ? 1ull << 63 : 0ull);
  propagate(a, L, (uint32_t)(P - 1), 1, base, cap, err, it.hint1, held);
  if (clk && lane == 0) clk[4 * 1024] = wall_clock64();
  return err;
}

}  // namespace dev
}  // namespace shm
