// insert.hip — batched Tree::insert / Tree::del on HBM pages.
//
// Restates src/Tree.cpp:828-991 (leaf_page_store), 699-826
// (internal_page_store), 993-1057 (leaf_page_del) and 126-149
// (update_new_root) for a sorted, de-duplicated batch.  The host runtime
// (tree.cpp) groups the batch's keys into *segments* (runs of keys whose
// B-link walk ends at the same page) and runs, per tree level:
//
//   plan   (1 wave / segment, read-only): entries after the batch T and the
//          page count P (P = 1: applied in place; P > 1: k-way split into
//          ceil(T / fill) pages, fill = 36 leaf / 40 internal).
//   build  (1 wave / NEW page): new right siblings, written before anything
//          links to them (Sherman writes the sibling first, Tree.cpp:962).
//   update (1 wave / segment): lock the page in the HBM lock table
//          (atomicCAS 0 -> tag on lock[CityHash64(page) % num_locks], the
//          reference's on-chip lock word, Tree.cpp:205-242/832-842), re-read
//          it, check the front_version the plan saw (optimistic check), then
//          either apply the updates in place with the reference's slot rule
//          (update the valid slot with the key, else first empty slot; entry
//          versions f++ / r = f, Tree.cpp:878-912) or rewrite page 0 of the
//          split (set_consistent: front++ , rear = front), release the lock.
//
// A split page's new separators (first key of each new leaf / the pushed-up
// key of each new internal page) are emitted already sorted and become the
// next level's batch; a split root gets a new root above it.
#include "device_common.h"
#include "kernels.h"

namespace shm {
namespace dev {

namespace {

struct WaveLds {
  uint32_t page[kPageDwords + 8];
  uint64_t a_key[kWave];
  uint64_t a_val[kWave];
  uint32_t a_ver[kWave];
};

__device__ __forceinline__ uint64_t new_page_ga(const SegArgs& a, uint32_t g,
                                                int p) {
  const uint64_t idx = a.first_new_page + a.seg_pbase[g] + (uint64_t)(p - 1);
  return ga_make(a.node, idx * kPageSize);
}

__device__ __forceinline__ uint32_t lock_index(uint64_t page, uint32_t n) {
  return (uint32_t)(cityhash64_u64(page) % n);
}

// lane 0 spins on atomicCAS(0 -> tag); bounded (Tree.cpp:218-238)
__device__ __forceinline__ bool lock_page(const SegArgs& a, uint64_t page,
                                          uint64_t tag) {
  int ok = 0;
  if (lane_id() == 0) {
    unsigned long long* w =
        reinterpret_cast<unsigned long long*>(a.locks + lock_index(page, a.num_locks));
    for (uint32_t spin = 0; spin < kMaxLockSpins; ++spin) {
      if (atomicCAS(w, 0ull, (unsigned long long)tag) == 0ull) {
        ok = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  return rl32((uint32_t)ok, 0) != 0;
}

__device__ __forceinline__ void unlock_page(const SegArgs& a, uint64_t page) {
  // The page stores are performed (vmcnt(0)) before the lock word is cleared
  // (write_page_and_unlock batches "write page, then release", Tree.cpp:
  // 266-298).  No agent-scope release fence: within one batch every page is
  // written by exactly one wave (lock holders that collide on a lock word
  // touch other pages), and the next kernel on the stream sees all stores;
  // a release here costs an L2 write-back per segment (measured 11 ms per
  // 1 Mi-insert batch).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane_id() == 0) {
    __hip_atomic_store(a.locks + lock_index(page, a.num_locks), 0ull,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Does `key` occur among ops [st, en)?  (ops are sorted, unique)
__device__ __forceinline__ bool op_contains(const SegArgs& a, uint32_t st,
                                            uint32_t en, uint64_t key) {
  const uint64_t i = lower_bound64(a.op_key, st, en, key);
  return i < en && a.op_key[i] == key;
}

// Surviving entries of the staged leaf (valid, not overwritten by an op),
// sorted by key into L.a_* ; returns their count.
__device__ int leaf_survivors(const SegArgs& a, WaveLds& L, uint32_t st,
                              uint32_t en) {
  const int lane = lane_id();
  const LeafEnt e = leaf_entry(L.page, lane < kLeafCardinality ? lane : 0);
  bool keep = lane < kLeafCardinality && e.val != kValueNull;
  if (keep && op_contains(a, st, en, e.key)) keep = false;
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

// Surviving records of the staged internal page, in key order.
__device__ int internal_survivors(const SegArgs& a, WaveLds& L, const u32x4 w,
                                  int cnt, uint32_t st, uint32_t en) {
  const int lane = lane_id();
  const IntRec r = internal_record(w);
  bool keep = lane >= 3 && lane - 3 < cnt;
  if (keep && op_contains(a, st, en, r.key)) keep = false;
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

// Element r of merge(A = survivors (na), B = ops [st, st + nb)); keys are
// disjoint.  Merge-path binary search (distinct keys).
__device__ __forceinline__ void merged_elem(const SegArgs& a, const WaveLds& L,
                                            int na, uint32_t st, uint32_t nb,
                                            uint32_t r, uint64_t& key,
                                            uint64_t& val, uint32_t& ver) {
  uint32_t lo = r > nb ? r - nb : 0;
  uint32_t hi = r < (uint32_t)na ? r : (uint32_t)na;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (L.a_key[mid] < a.op_key[st + r - mid - 1])
      lo = mid + 1;
    else
      hi = mid;
  }
  const uint32_t i = lo, j = r - lo;
  if (i < (uint32_t)na && (j >= nb || L.a_key[i] < a.op_key[st + j])) {
    key = L.a_key[i];
    val = L.a_val[i];
    ver = L.a_ver[i];
  } else {
    key = a.op_key[st + j];
    val = a.op_val[st + j];
    ver = 0;  // fresh LeafEntry() in the sibling (Tree.cpp:934, 944-948)
  }
}

// Write page p (0 <= p < P) of a leaf k-way split of segment g into L.page and
// store it.  Survivors must already be in L.a_*.
__device__ void build_leaf_page(const SegArgs& a, WaveLds& L, uint32_t g,
                                const Hdr& h, int na, int p, int P,
                                uint32_t T, uint64_t page_ga) {
  const int lane = lane_id();
  const uint32_t st = a.seg_start[g], nb = a.seg_start[g + 1] - st;
  const uint32_t base = T / (uint32_t)P, rem = T % (uint32_t)P;
  const uint32_t c = base + ((uint32_t)p < rem ? 1u : 0u);
  const uint32_t s0 = (uint32_t)p * base + ((uint32_t)p < rem ? (uint32_t)p : rem);
  uint64_t key = 0, val = 0;
  uint32_t ver = 0;
  const bool has_next = p + 1 < P;
  if ((uint32_t)lane < c || ((uint32_t)lane == c && has_next))
    merged_elem(a, L, na, st, nb, s0 + (uint32_t)lane, key, val, ver);
  const uint64_t lowest = p == 0 ? h.lowest : rl64(key, 0);
  const uint64_t highest = has_next ? rl64(key, (int)c) : h.highest;
  const uint64_t sibling = has_next ? new_page_ga(a, g, p + 1) : h.sibling;
  const uint32_t fver = p == 0 ? ((h.fver + 1) & 0xFF) : 1u;
  wave_lds_sync();
  init_page_image(L.page, fver, 0, sibling, 0, (int32_t)c - 1, lowest, highest);
  wave_lds_sync();
  if ((uint32_t)lane < c) put_leaf_entry(L.page, lane, key, val, ver & 0xFF, ver >> 8);
  if (lane == 0) L.page[kOffLeafRear / 4] = fver;  // rear_version, byte 1016
  store_page(a.arena, ga_offset(page_ga), L.page);
  if (a.leaf_hw && lane == 0) a.leaf_hw[ga_offset(page_ga) >> 10] = (uint8_t)c;  // slots [0, c)
  if (p > 0 && lane == 0) {
    const uint64_t o = a.seg_pbase[g] + (uint64_t)(p - 1);
    a.sep_key[o] = lowest;
    a.sep_ptr[o] = page_ga;
  }
}

__device__ void build_internal_page(const SegArgs& a, WaveLds& L, uint32_t g,
                                    const Hdr& h, int na, int p, int P,
                                    uint32_t T, uint64_t page_ga) {
  const int lane = lane_id();
  const uint32_t st = a.seg_start[g], nb = a.seg_start[g + 1] - st;
  const uint32_t q = T - (uint32_t)(P - 1);  // records kept (non pushed-up)
  const uint32_t base = q / (uint32_t)P, rem = q % (uint32_t)P;
  const uint32_t c = base + ((uint32_t)p < rem ? 1u : 0u);
  const uint32_t s0 = (uint32_t)p * base + ((uint32_t)p < rem ? (uint32_t)p : rem) +
                      (uint32_t)p;
  const bool has_next = p + 1 < P;
  uint64_t key = 0, val = 0;
  uint32_t ver = 0;
  bool want = false;
  uint32_t r = 0;
  if ((uint32_t)lane < c) {
    want = true;
    r = s0 + (uint32_t)lane;
  } else if (lane == 62 && p > 0) {
    want = true;
    r = s0 - 1;  // record pushed up to the parent; its ptr becomes leftmost
  } else if (lane == 63 && has_next) {
    want = true;
    r = s0 + c;  // next page's pushed-up key = this page's highest
  }
  if (want) merged_elem(a, L, na, st, nb, r, key, val, ver);
  const uint64_t leftmost = p == 0 ? h.leftmost : rl64(val, 62);
  const uint64_t lowest = p == 0 ? h.lowest : rl64(key, 62);
  const uint64_t highest = has_next ? rl64(key, 63) : h.highest;
  const uint64_t sibling = has_next ? new_page_ga(a, g, p + 1) : h.sibling;
  const uint32_t fver = p == 0 ? ((h.fver + 1) & 0xFF) : 1u;
  wave_lds_sync();
  init_page_image(L.page, fver, leftmost, sibling, (uint32_t)a.level,
                  (int32_t)c - 1, lowest, highest);
  wave_lds_sync();
  if ((uint32_t)lane < c) {
    uint32_t* d = L.page + (kOffRecords + kInternalEntry * lane) / 4;
    d[0] = (uint32_t)key;
    d[1] = (uint32_t)(key >> 32);
    d[2] = (uint32_t)val;
    d[3] = (uint32_t)(val >> 32);
  }
  if (lane == 0) L.page[kOffInternalRear / 4] = fver;  // byte 1020
  store_page(a.arena, ga_offset(page_ga), L.page);
  if (p > 0 && lane == 0) {
    const uint64_t o = a.seg_pbase[g] + (uint64_t)(p - 1);
    a.sep_key[o] = lowest;
    a.sep_ptr[o] = page_ga;
  }
}

// segment index owning global new-page index gp (last s with pbase[s] <= gp)
__device__ __forceinline__ uint32_t seg_of_new_page(const SegArgs& a,
                                                    uint32_t gp) {
  uint32_t lo = 0, hi = a.num_seg;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a.seg_pbase[mid] <= gp)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo - 1;
}

}  // namespace

// ---------------------------------------------------------------------------
// leaf plan: T = valid + ops - overwritten; P = 1 if T <= 53 else ceil(T/36)
__global__ __launch_bounds__(kBlock) void k_leaf_plan(SegArgs a) {
  __shared__ __attribute__((aligned(16))) WaveLds s_l[kWavesPerBlock];
  const int lane = lane_id();
  const uint32_t g = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (g >= a.num_seg) return;
  WaveLds& L = s_l[threadIdx.x >> 6];
  const uint32_t st = a.seg_start[g], en = a.seg_start[g + 1];
  const uint64_t page = a.seg_page[g];
  if (!ptr_ok(page, a.node, a.arena_bytes)) {
    if (lane == 0) {
      atomicOr(a.err, kErrBadPtr);
      a.seg_T[g] = 0; a.seg_P[g] = 1; a.seg_newpages[g] = 0; a.seg_ver[g] = ~0u;
    }
    return;
  }
  const u32x4 w = load_page_slice(a.arena, ga_offset(page));
  const Hdr h = parse_hdr(w);
  stage_page(L.page, w);
  wave_lds_sync();
  const LeafEnt e = leaf_entry(L.page, lane < kLeafCardinality ? lane : 0);
  const bool valid = lane < kLeafCardinality && e.val != kValueNull;
  const bool hit = valid && op_contains(a, st, en, e.key);
  const uint32_t V = (uint32_t)popc64(ballot(valid));
  const uint32_t M = (uint32_t)popc64(ballot(hit));
  const uint32_t T = V + (en - st) - M;
  const uint32_t P = T <= (uint32_t)(kLeafCardinality - 1)
                         ? 1u
                         : (T + kLeafSplitFill - 1) / kLeafSplitFill;
  if (lane == 0) {
    a.seg_T[g] = T;
    a.seg_P[g] = P;
    a.seg_newpages[g] = P - 1;
    a.seg_ver[g] = h.fver;
    if (h.fver != h.rver_leaf || h.leftmost != 0) atomicOr(a.err, kErrInconsistent);
  }
}

// new right-sibling leaves of k-way splits (1 wave per new page)
__global__ __launch_bounds__(kBlock) void k_leaf_build(SegArgs a, uint32_t total) {
  __shared__ __attribute__((aligned(16))) WaveLds s_l[kWavesPerBlock];
  const uint32_t gp = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (gp >= total) return;
  WaveLds& L = s_l[threadIdx.x >> 6];
  const uint32_t g = seg_of_new_page(a, gp);
  const int p = (int)(gp - a.seg_pbase[g]) + 1;
  const int P = (int)a.seg_P[g];
  const uint32_t st = a.seg_start[g], en = a.seg_start[g + 1];
  const u32x4 w = load_page_slice(a.arena, ga_offset(a.seg_page[g]));
  const Hdr h = parse_hdr(w);
  stage_page(L.page, w);
  wave_lds_sync();
  const int na = leaf_survivors(a, L, st, en);
  build_leaf_page(a, L, g, h, na, p, P, a.seg_T[g], new_page_ga(a, g, p));
}

// lock, validate, apply in place or rewrite page 0, unlock (1 wave / segment)
__global__ __launch_bounds__(kBlock) void k_leaf_update(SegArgs a) {
  __shared__ __attribute__((aligned(16))) WaveLds s_l[kWavesPerBlock];
  const int lane = lane_id();
  const uint32_t g = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (g >= a.num_seg) return;
  WaveLds& L = s_l[threadIdx.x >> 6];
  const uint64_t page = a.seg_page[g];
  if (!ptr_ok(page, a.node, a.arena_bytes)) return;
  // after k_leaf_upsert only the segments it flagged for a split remain
  if (a.split_only && a.seg_P[g] == 1) return;
  const uint32_t st = a.seg_start[g], en = a.seg_start[g + 1];
  if (!lock_page(a, page, a.tag_base + g + 1)) {
    if (lane == 0) atomicOr(a.err, kErrLock);
    return;
  }
  const u32x4 w = load_page_slice(a.arena, ga_offset(page));
  const Hdr h = parse_hdr(w);
  if (h.fver != a.seg_ver[g] || h.fver != h.rver_leaf) {
    if (lane == 0) atomicOr(a.err, kErrPlan);
    unlock_page(a, page);
    return;
  }
  stage_page(L.page, w);
  wave_lds_sync();
  const int P = (int)a.seg_P[g];
  if (P == 1) {
    // in place, sequential in key order (Tree.cpp:875-912)
    LeafEnt e = leaf_entry(L.page, lane < kLeafCardinality ? lane : 0);
    const bool slot = lane < kLeafCardinality;
    bool dirty = false;
    for (uint32_t j = st; j < en; ++j) {
      const uint64_t kb = a.op_key[j];
      const uint64_t vb = a.op_val[j];
      uint64_t mm = ballot(slot && e.val != kValueNull && e.key == kb);
      bool fresh = false;
      if (!mm) {
        mm = ballot(slot && e.val == kValueNull);  // first empty slot
        fresh = true;
        if (!mm) {
          if (lane == 0) atomicOr(a.err, kErrOverflow);
          break;
        }
      }
      if (lane == ctz64(mm)) {
        if (fresh) e.key = kb;
        e.val = vb;
        const uint32_t f = ((e.fraw & 0xF) + 1) & 0xF;
        e.fraw = (e.fraw & 0xF0) | f;
        e.rraw = (e.rraw & 0xF0) | f;
        dirty = true;
      }
    }
    wave_lds_sync();
    if (dirty) put_leaf_entry(L.page, lane, e.key, e.val, e.fraw, e.rraw);
    store_page(a.arena, ga_offset(page), L.page);
    const uint64_t vm = ballot(slot && e.val != kValueNull);
    if (a.leaf_hw && lane == 0)
      a.leaf_hw[ga_offset(page) >> 10] = (uint8_t)(vm ? 64 - __builtin_clzll(vm) : 0);
  } else {
    const int na = leaf_survivors(a, L, st, en);
    build_leaf_page(a, L, g, h, na, 0, P, a.seg_T[g], page);
  }
  unlock_page(a, page);
}

// Tree::del on each segment (leaf_page_del, Tree.cpp:1037-1055)
__global__ __launch_bounds__(kBlock) void k_leaf_delete(SegArgs a) {
  __shared__ __attribute__((aligned(16))) WaveLds s_l[kWavesPerBlock];
  const int lane = lane_id();
  const uint32_t g = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (g >= a.num_seg) return;
  WaveLds& L = s_l[threadIdx.x >> 6];
  const uint64_t page = a.seg_page[g];
  if (!ptr_ok(page, a.node, a.arena_bytes)) return;
  const uint32_t st = a.seg_start[g], en = a.seg_start[g + 1];
  if (!lock_page(a, page, a.tag_base + g + 1)) {
    if (lane == 0) atomicOr(a.err, kErrLock);
    return;
  }
  const u32x4 w = load_page_slice(a.arena, ga_offset(page));
  const Hdr h = parse_hdr(w);
  if (h.fver != h.rver_leaf) {
    if (lane == 0) atomicOr(a.err, kErrInconsistent);
    unlock_page(a, page);
    return;
  }
  stage_page(L.page, w);
  wave_lds_sync();
  LeafEnt e = leaf_entry(L.page, lane < kLeafCardinality ? lane : 0);
  const bool hit = lane < kLeafCardinality && e.val != kValueNull &&
                   op_contains(a, st, en, e.key);
  if (ballot(hit)) {
    if (hit) {
      e.val = kValueNull;
      const uint32_t f = ((e.fraw & 0xF) + 1) & 0xF;
      e.fraw = (e.fraw & 0xF0) | f;
      e.rraw = (e.rraw & 0xF0) | f;
    }
    wave_lds_sync();
    if (hit) put_leaf_entry(L.page, lane, e.key, e.val, e.fraw, e.rraw);
    store_page(a.arena, ga_offset(page), L.page);
  }
  unlock_page(a, page);
}

// ---------------------------------------------------------------------------
// internal plan: T = cnt + ops - matched; P = 1 if T <= 60 else
// ceil((T + 1) / 41) (each extra page pushes one record up)
__global__ __launch_bounds__(kBlock) void k_int_plan(SegArgs a) {
  const int lane = lane_id();
  const uint32_t g = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (g >= a.num_seg) return;
  // a.num_seg may be an upper bound (num_seg_dev): zero the new-page counts
  // past the device-side count, which the scan after this kernel covers
  if (a.num_seg_dev && g >= *a.num_seg_dev) {
    if (lane == 0) a.seg_newpages[g] = 0;
    return;
  }
  const uint32_t st = a.seg_start[g], en = a.seg_start[g + 1];
  const uint64_t page = a.seg_page[g];
  if (!ptr_ok(page, a.node, a.arena_bytes)) {
    if (lane == 0) {
      atomicOr(a.err, kErrBadPtr);
      a.seg_T[g] = 0; a.seg_P[g] = 1; a.seg_newpages[g] = 0; a.seg_ver[g] = ~0u;
    }
    return;
  }
  const u32x4 w = load_page_slice(a.arena, ga_offset(page));
  const Hdr h = parse_hdr(w);
  const IntRec r = internal_record(w);
  const int cnt = h.last_index + 1;
  const bool valid = lane >= 3 && lane - 3 < cnt;
  const bool hit = valid && op_contains(a, st, en, r.key);
  const uint32_t M = (uint32_t)popc64(ballot(hit));
  const uint32_t T = (uint32_t)cnt + (en - st) - M;
  const uint32_t P = T <= (uint32_t)(kInternalCardinality - 1)
                         ? 1u
                         : (T + 1 + kInternalSplitFill) / (kInternalSplitFill + 1);
  if (lane == 0) {
    a.seg_T[g] = T;
    a.seg_P[g] = P;
    a.seg_newpages[g] = P - 1;
    a.seg_ver[g] = h.fver;
    if (h.fver != h.rver_internal || h.leftmost == 0 || (int)h.level != a.level)
      atomicOr(a.err, kErrInconsistent);
  }
}

__global__ __launch_bounds__(kBlock) void k_int_build(SegArgs a, uint32_t total) {
  __shared__ __attribute__((aligned(16))) WaveLds s_l[kWavesPerBlock];
  const uint32_t gp = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (gp >= total) return;
  WaveLds& L = s_l[threadIdx.x >> 6];
  const uint32_t g = seg_of_new_page(a, gp);
  const int p = (int)(gp - a.seg_pbase[g]) + 1;
  const uint32_t st = a.seg_start[g], en = a.seg_start[g + 1];
  const u32x4 w = load_page_slice(a.arena, ga_offset(a.seg_page[g]));
  const Hdr h = parse_hdr(w);
  const int na = internal_survivors(a, L, w, h.last_index + 1, st, en);
  build_internal_page(a, L, g, h, na, p, (int)a.seg_P[g], a.seg_T[g],
                      new_page_ga(a, g, p));
}

__global__ __launch_bounds__(kBlock) void k_int_update(SegArgs a) {
  __shared__ __attribute__((aligned(16))) WaveLds s_l[kWavesPerBlock];
  const int lane = lane_id();
  const uint32_t g = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (g >= a.num_seg) return;
  WaveLds& L = s_l[threadIdx.x >> 6];
  const uint64_t page = a.seg_page[g];
  if (!ptr_ok(page, a.node, a.arena_bytes)) return;
  const uint32_t st = a.seg_start[g], en = a.seg_start[g + 1];
  if (!lock_page(a, page, a.tag_base + g + 1)) {
    if (lane == 0) atomicOr(a.err, kErrLock);
    return;
  }
  const u32x4 w = load_page_slice(a.arena, ga_offset(page));
  const Hdr h = parse_hdr(w);
  if (h.fver != a.seg_ver[g] || h.fver != h.rver_internal) {
    if (lane == 0) atomicOr(a.err, kErrPlan);
    unlock_page(a, page);
    return;
  }
  const int na = internal_survivors(a, L, w, h.last_index + 1, st, en);
  build_internal_page(a, L, g, h, na, 0, (int)a.seg_P[g], a.seg_T[g], page);
  unlock_page(a, page);
}

// InternalPage(level) with leftmost = old root and no records; the level's
// separators are then inserted into it (update_new_root, Tree.cpp:126-149).
__global__ void k_new_root(uint8_t* arena, uint64_t off, uint64_t old_root,
                           uint32_t level) {
  __shared__ __attribute__((aligned(16))) uint32_t lp[kPageDwords + 8];
  init_page_image(lp, 1, old_root, 0, level, -1, kKeyMin, kKeyMax);
  wave_lds_sync();
  if (lane_id() == 0) lp[kOffInternalRear / 4] = 1;
  store_page(arena, off, lp);
}

// LeafPage() + set_consistent (Tree.cpp:47-52)
__global__ void k_empty_leaf(uint8_t* arena, uint64_t off) {
  __shared__ __attribute__((aligned(16))) uint32_t lp[kPageDwords + 8];
  init_page_image(lp, 1, 0, 0, 0, -1, kKeyMin, kKeyMax);
  wave_lds_sync();
  if (lane_id() == 0) lp[kOffLeafRear / 4] = 1;
  store_page(arena, off, lp);
}

__global__ void k_write_superblock(uint8_t* arena, Superblock sb) {
  if (threadIdx.x == 0) *reinterpret_cast<Superblock*>(arena) = sb;
}

// ---------------------------------------------------------------------------
static dim3 seg_grid(uint64_t waves) {
  return dim3((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock));
}
void launch_leaf_plan(const SegArgs& a, hipStream_t s) {
  if (a.num_seg) hipLaunchKernelGGL(k_leaf_plan, seg_grid(a.num_seg), dim3(kBlock), 0, s, a);
}
void launch_leaf_build(const SegArgs& a, uint32_t total, hipStream_t s) {
  if (total) hipLaunchKernelGGL(k_leaf_build, seg_grid(total), dim3(kBlock), 0, s, a, total);
}
void launch_leaf_update(const SegArgs& a, hipStream_t s) {
  if (a.num_seg) hipLaunchKernelGGL(k_leaf_update, seg_grid(a.num_seg), dim3(kBlock), 0, s, a);
}
void launch_leaf_delete(const SegArgs& a, hipStream_t s) {
  if (a.num_seg) hipLaunchKernelGGL(k_leaf_delete, seg_grid(a.num_seg), dim3(kBlock), 0, s, a);
}
void launch_int_plan(const SegArgs& a, hipStream_t s) {
  if (a.num_seg) hipLaunchKernelGGL(k_int_plan, seg_grid(a.num_seg), dim3(kBlock), 0, s, a);
}
void launch_int_build(const SegArgs& a, uint32_t total, hipStream_t s) {
  if (total) hipLaunchKernelGGL(k_int_build, seg_grid(total), dim3(kBlock), 0, s, a, total);
}
void launch_int_update(const SegArgs& a, hipStream_t s) {
  if (a.num_seg) hipLaunchKernelGGL(k_int_update, seg_grid(a.num_seg), dim3(kBlock), 0, s, a);
}
void launch_new_root(uint8_t* arena, uint64_t off, uint64_t old_root,
                     uint32_t level, hipStream_t s) {
  hipLaunchKernelGGL(k_new_root, dim3(1), dim3(kWave), 0, s, arena, off, old_root, level);
}
void launch_write_superblock(uint8_t* arena, const Superblock& sb, hipStream_t s) {
  hipLaunchKernelGGL(k_write_superblock, dim3(1), dim3(kWave), 0, s, arena, sb);
}
void launch_empty_leaf(uint8_t* arena, uint64_t off, hipStream_t s) {
  hipLaunchKernelGGL(k_empty_leaf, dim3(1), dim3(kWave), 0, s, arena, off);
}

}  // namespace dev
}  // namespace shm
