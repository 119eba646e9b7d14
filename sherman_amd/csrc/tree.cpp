// tree.cpp — host runtime behind the C-ABI (include/sherman_amd.h).
//
// Owns one shard's HBM page arena, lock table and batch workspace, and drives
// the kernels of walk.hip / insert.hip / util.hip.  The roles of the
// reference's DSM (include/DSM.h:33-176: remote read/write/CAS, alloc), the
// Directory's root publication (src/Directory.cpp:72-83) and the
// Local/GlobalAllocator (include/LocalAllocator.h, GlobalAllocator.h) are
// taken by: plain HBM pointers, a host-authoritative bump allocator over the
// arena (mirrored into the superblock in page 0) and a root register.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cstdio>
#include <mutex>
#include <vector>

#include "../../include/sherman_amd.h"
#include "kernels.h"
#include "layout.h"
#include "sort.h"

using namespace shm;

namespace {

constexpr uint64_t kSortMinGets = 8192;   // below this, walk in input order


constexpr uint32_t kDefaultSortBits = 16; // top key bits that order gets (8 + 8)
// get start table: 2^bits key prefixes (SHM_START_BITS, 8..22, default 16)
uint32_t start_bits() {
  static const uint32_t b = [] {
    const char* e = getenv("SHM_START_BITS");
    const int v = e ? atoi(e) : 16;
    return (uint32_t)(v < 8 ? 8 : v > 22 ? 22 : v);
  }();
  return b;
}
constexpr int kRedoOrder = -1000;          // internal: re-order with rocPRIM
constexpr uint32_t kRangeStage = 160;      // staged values per range scan
constexpr uint64_t kRangeStageBytes = 256ull << 20;  // staging budget
constexpr int kWalkDepth = 4;             // (ring depth is fixed in walk.hip)

}  // namespace

struct shm_tree {
  shm_config cfg{};
  hipStream_t stream = nullptr;
  uint8_t* arena = nullptr;
  uint64_t arena_bytes = 0;
  uint64_t cap_pages = 0;
  uint64_t* locks = nullptr;
  uint32_t* d_err = nullptr;
  uint64_t* d_counts = nullptr;  // 16 words of device scratch
  uint32_t* route_scratch = nullptr;
  // route_bucket scratch per stream (route_scratch serves the first one), so
  // routed batches on distinct streams bucket concurrently
  std::vector<std::pair<hipStream_t, uint32_t*>> route_ws;
  uint64_t* h_pin = nullptr;     // 16 words pinned host scratch (coherent, mapped)
  uint32_t* h_pin_dev = nullptr; // its device address (zero-copy read-backs)
  uint32_t rb_seq = 0;           // last zero-copy read-back sequence number
  uint64_t rb_nup = 0, rb_ndel = 0;  // ordering counts of the last read-back
  uint64_t* rstage = nullptr;    // range-scan value staging (RangeArgs.stage)
  uint64_t rstage_words = 0;
  // host-authoritative tree metadata (superblock mirror)
  uint64_t root = 0;
  uint32_t root_level = 0;
  uint64_t next_page = 0;
  uint64_t batches = 0;
  uint64_t splits = 0;
  uint32_t sticky_err = 0;
  // workspace (sized for cfg.max_batch)
  uint64_t nmax = 0, sep_cap = 0;
  uint64_t *ka = nullptr, *kb = nullptr;
  uint32_t *ia = nullptr, *ib = nullptr;
  uint64_t *flags = nullptr, *pos = nullptr;
  uint64_t *uk = nullptr, *uv = nullptr, *dk = nullptr;
  uint64_t* pages = nullptr;
  uint32_t *heads = nullptr, *hpos = nullptr;
  uint32_t* bsum = nullptr;  // per-tile sums of the two-launch scans
  uint64_t* bsum64 = nullptr;
  uint32_t* seg_start = nullptr;
  uint64_t* seg_page = nullptr;
  uint32_t *seg_T = nullptr, *seg_P = nullptr, *seg_np = nullptr,
           *seg_pbase = nullptr, *seg_ver = nullptr;
  uint8_t* leaf_hw = nullptr;   // per-page occupancy bound (layout.h kLeafHwFull)
  uint32_t* seg_lk = nullptr;  // lock words taken ahead per segment (k_seg_fill)
  uint64_t *sep_key[2] = {nullptr, nullptr}, *sep_ptr[2] = {nullptr, nullptr};
  void* temp = nullptr;
  size_t temp_bytes = 0;
  uint32_t* part_hist = nullptr;  // [kMaxTiles][kCoarse] coarse tile counts
  uint32_t* part_S = nullptr;     // coarse group sums (zero between batches)
  uint32_t* part_chunks = nullptr;  // fine-pass chunk table
  uint32_t* gcount = nullptr;       // insert ordering: survivors per 4096-op tile
  uint32_t* bins = nullptr;         // insert ordering: (start, count) per coarse bin
  // get start pages per key prefix (dev::launch_start_table); rebuilt before a
  // search when pages were added or the root moved since it was built
  uint64_t* start = nullptr;
  uint64_t start_np = ~0ull, start_root = ~0ull;
  // leaf directory (leafdir.hip): 2^dir_bits entries of 32 B over the whole
  // key space, rebuilt before a search once the tree grew by 1/32 since the
  // last build (stale entries only cost B-link right moves)
  bool err_pending = false;  // kernels ran since d_err was last read back
  uint64_t* dir = nullptr;
  uint32_t dir_bits = 0;
  uint64_t dir_np = 0;
  bool dir_valid = false;
  std::mutex mu;
  // profiling (shm_profile_*)
  bool prof_on = false;
  enum ProfKind { kProfGet = 0, kProfInsert = 1, kProfRange = 2 };
  // get: e0 order e1 walk e2; insert chunk: e0 .. e1 upsert e2 .. e3;
  // range launch: e0 kernel e1
  struct ProfRec {
    hipEvent_t e[4];
    uint64_t n;
    int kind;
    bool upsert_done;
  };
  std::vector<ProfRec> prof_pending;
  ProfRec* prof_ins = nullptr;  // the insert chunk being timed
  std::vector<hipEvent_t> event_pool;
  shm_profile_t prof_acc{};
  // ---- cross-stream ordering (Order below) --------------------------------
  // Searches are "shared" calls: they may run concurrently on distinct
  // streams.  An ordered search uses one of two get workspaces, alternating,
  // so the partition of one batch can overlap the walk of the previous one
  // on another stream.  Every other call that touches device state (inserts,
  // deletes, range scans, routing, a directory rebuild) is "exclusive": its
  // stream waits for every earlier call on the other streams.
  struct GetWs {
    uint64_t *keys1 = nullptr, *keys_out = nullptr;
    uint32_t *pos1 = nullptr, *src = nullptr, *M = nullptr, *S = nullptr, *chunks = nullptr;
  };
  GetWs gws[2];           // gws[0] aliases the insert workspace (ka, kb, ia, ib, part_*)
  int next_gws = 0;
  struct StreamEv {
    hipStream_t s;
    hipEvent_t ev;
  };
  std::vector<StreamEv> shared_ev;  // last shared call per stream
  hipEvent_t ex_ev = nullptr;       // last exclusive call
  hipStream_t ex_s = nullptr;
  bool ex_valid = false;
  hipEvent_t gws_ev[2] = {nullptr, nullptr};  // last user of each get workspace
  hipStream_t gws_s[2] = {nullptr, nullptr};
  bool gws_valid[2] = {false, false};
};

namespace {

#define HIP_OK(expr)                                                         \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess) {                                                  \
      fprintf(stderr, "sherman_amd: %s failed: %s (%s:%d)\n", #expr,         \
              hipGetErrorString(_e), __FILE__, __LINE__);                    \
      return SHM_EIO;                                                        \
    }                                                                        \
  } while (0)

template <class T>
int dalloc(T** p, uint64_t count) {
  if (count == 0) count = 1;
  if (hipMalloc((void**)p, sizeof(T) * count) != hipSuccess) {
    *p = nullptr;
    return SHM_ENOMEM;
  }
  return SHM_OK;
}

// stream argument of the C-ABI: NULL is the HIP null (default) stream, as for
// any HIP API; t->stream is used only for create / image transfers.
hipStream_t pick(shm_tree* t, void* s) {
  (void)t;
  return (hipStream_t)s;
}

hipEvent_t new_event() {
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  return e;
}

// Cross-stream ordering of one API call (shm_tree: shared / exclusive calls).
// Constructed under t->mu before the call's first launch; the destructor
// records the call's completion event on its stream.  Waits are skipped for
// events of the same stream (stream order already covers them).
struct Order {
  shm_tree* t;
  hipStream_t s;
  bool ex;
  int ws = -1;  // get workspace used by a shared call (-1: none)
  int rc = SHM_OK;
  Order(shm_tree* tt, hipStream_t ss, bool exclusive) : t(tt), s(ss), ex(exclusive) {
    if (t->ex_valid && t->ex_s != s) wait(t->ex_ev);
    if (ex) {
      for (const auto& r : t->shared_ev)
        if (r.s != s) wait(r.ev);
      for (int j = 0; j < 2; ++j)
        if (t->gws_valid[j] && t->gws_s[j] != s) wait(t->gws_ev[j]);
    }
  }
  // a shared call that turns exclusive (a directory rebuild)
  void make_exclusive() {
    if (ex) return;
    ex = true;
    for (const auto& r : t->shared_ev)
      if (r.s != s) wait(r.ev);
    for (int j = 0; j < 2; ++j)
      if (t->gws_valid[j] && t->gws_s[j] != s) wait(t->gws_ev[j]);
  }
  // take the next get workspace; returns its index
  int take_ws() {
    ws = t->next_gws;
    t->next_gws ^= 1;
    if (!ex && t->gws_valid[ws] && t->gws_s[ws] != s) wait(t->gws_ev[ws]);
    return ws;
  }
  void wait(hipEvent_t e) {
    if (hipStreamWaitEvent(s, e, 0) != hipSuccess) rc = SHM_EIO;
  }
  ~Order() {
    if (ex) {
      if (!t->ex_ev) t->ex_ev = new_event();
      if (t->ex_ev && hipEventRecord(t->ex_ev, s) == hipSuccess) {
        t->ex_s = s;
        t->ex_valid = true;
        // the waits above ordered this call after every earlier one
        for (auto& r : t->shared_ev) (void)hipEventDestroy(r.ev);
        t->shared_ev.clear();
        t->gws_valid[0] = t->gws_valid[1] = false;
      }
      return;
    }
    shm_tree::StreamEv* r = nullptr;
    for (auto& x : t->shared_ev)
      if (x.s == s) r = &x;
    if (!r) {
      hipEvent_t e = new_event();
      if (!e) return;
      t->shared_ev.push_back({s, e});
      r = &t->shared_ev.back();
    }
    (void)hipEventRecord(r->ev, s);
    if (ws >= 0) {
      if (!t->gws_ev[ws]) t->gws_ev[ws] = new_event();
      if (t->gws_ev[ws] && hipEventRecord(t->gws_ev[ws], s) == hipSuccess) {
        t->gws_s[ws] = s;
        t->gws_valid[ws] = true;
      }
    }
  }
};

// SHM_GET_KERNEL=walk selects the page-at-a-time walk (k_walk) for gets
// instead of the grouped one (k_get): an A/B switch for measurements.
bool get_kernel_v4() {
  static const bool v4 = [] {
    const char* e = getenv("SHM_GET_KERNEL");
    return e && strcmp(e, "walk") == 0;
  }();
  return v4;
}

// SHM_WALK_NT=0/1: leaf-page DMAs of the get walk with the default or the
// non-temporal cache policy (A/B knob; default 1: a leaf is read once per
// batch, and nt keeps it from displacing the directory: C2 +5 %)
// leaf DMA policy: ordered walks read each leaf once per batch (queries
// sharing it sit in one wave), so non-temporal loads keep the directory in
// L2 (C2 +5 %); an unordered walk reads a leaf once per wave that needs it,
// and under skew (C3, zipf 0.99) the cached policy serves the repeats from
// L2 (walk -9 %).  SHM_WALK_NT=0/1 forces either.
int walk_nt(bool ordered) {
  static const int v = [] {
    const char* e = getenv("SHM_WALK_NT");
    return e ? atoi(e) : -1;
  }();
  return v >= 0 ? v : (ordered ? 1 : 0);
}

// SHM_DEFER_COUNTS=0 reads the insert ordering's counts back before the
// leaf level (one more host synchronisation per batch; A/B knob)
bool deferred_counts() {
  static const bool v = [] {
    const char* e = getenv("SHM_DEFER_COUNTS");
    return !(e && strcmp(e, "0") == 0);
  }();
  return v;
}

// SHM_BIN_UNIQUE=0 orders insert batches with the per-bin bitonic sort and
// the mark / scan / compact passes instead of k_bin_unique (A/B knob)
bool bin_unique() {
  static const bool v = [] {
    const char* e = getenv("SHM_BIN_UNIQUE");
    return !(e && strcmp(e, "0") == 0);
  }();
  return v;
}

// SHM_GET_DIRECT=1: ordered gets carry each query's input index through the
// partition and the walk stores results in input order (no unpartition pass)
bool get_direct() {
  static const bool v = [] {
    const char* e = getenv("SHM_GET_DIRECT");
    return e && atoi(e) != 0;
  }();
  return v;
}

// SHM_GET_STAMPS=<file>: append the per-wave {start, end} s_memrealtime
// stamps (100 MHz) of every get walk launch to <file> (diagnostics only;
// synchronises the stream after each launch).
struct StampDump {
  uint64_t* d = nullptr;
  uint64_t n = 0;
  hipStream_t s;
  StampDump(dev::WalkArgs& a, uint64_t m, hipStream_t st) : s(st) {
    static const char* path = getenv("SHM_GET_STAMPS");
    if (!path) return;
    n = 2 * ((m + 63) / 64);
    if (hipMalloc((void**)&d, n * 8) != hipSuccess) d = nullptr;
    a.stamps = d;
  }
  ~StampDump() {
    if (!d) return;
    std::vector<uint64_t> h(n);
    if (hipMemcpyAsync(h.data(), d, n * 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
        hipStreamSynchronize(s) == hipSuccess) {
      if (FILE* f = fopen(getenv("SHM_GET_STAMPS"), "ab")) {
        fwrite(&n, 8, 1, f);
        fwrite(h.data(), 8, n, f);
        fclose(f);
      }
    }
    (void)hipFree(d);
  }
};

dev::WalkArgs walk_args(shm_tree* t) {
  dev::WalkArgs a{};
  a.arena = t->arena;
  a.arena_bytes = t->arena_bytes;
  a.node = t->cfg.node_id;
  a.root = t->root;
  a.err = t->d_err;
  return a;
}

// SHM_LEAF_HW=0: gets read whole leaves (A/B knob; the bound is kept anyway)
bool use_leaf_hw() {
  static const bool on = [] {
    const char* e = getenv("SHM_LEAF_HW");
    return !(e && strcmp(e, "0") == 0);
  }();
  return on;
}

// SHM_TILE_SCAN=0: segmentation and the new-page scan through rocPRIM
bool use_tile_scan() {
  static const bool on = [] {
    const char* e = getenv("SHM_TILE_SCAN");
    return !(e && strcmp(e, "0") == 0);
  }();
  return on;
}

// SHM_INT_DEV_COUNT=0: internal levels read their segment count back
bool int_dev_count() {
  static const bool on = [] {
    const char* e = getenv("SHM_INT_DEV_COUNT");
    return !(e && strcmp(e, "0") == 0);
  }();
  return on;
}

// SHM_FAST_INSERT=0 selects the page-at-a-time locate walk and the
// plan / update leaf kernels instead of the grouped locate + k_leaf_upsert
bool use_fast_insert() {
  static const bool on = [] {
    const char* e = getenv("SHM_FAST_INSERT");
    return !(e && strcmp(e, "0") == 0);
  }();
  return on;
}

// leaf directory on (SHM_FLAG_LEAF_DIR); SHM_LEAF_DIR=0 turns it off for
// A/B runs (gets then start at the prefix start table or the root)
bool use_leaf_dir(const shm_tree* t) {
  static const bool env_on = [] {
    const char* e = getenv("SHM_LEAF_DIR");
    return !(e && strcmp(e, "0") == 0);
  }();
  return env_on && (t->cfg.flags & SHM_FLAG_LEAF_DIR) != 0;
}

// (re)build the leaf directory when missing or the tree grew by > 1/32;
// 2^bits entries with bits = ceil(log2(pages)) (~1 entry per leaf)
bool dir_stale(const shm_tree* t) {
  return !(t->dir_valid && t->next_page <= t->dir_np + t->dir_np / 32);
}

int refresh_dir(shm_tree* t, hipStream_t s) {
  if (!dir_stale(t)) return SHM_OK;
  uint32_t bits = 10;
  while (bits < 24 && (1ull << bits) < t->next_page) ++bits;
  if (bits > t->cfg.key_bits) bits = t->cfg.key_bits;  // one entry per key at most
  if (!t->dir || bits != t->dir_bits) {
    if (t->dir) {
      HIP_OK(hipStreamSynchronize(s));
      HIP_OK(hipFree(t->dir));
      t->dir = nullptr;
    }
    if (dalloc(&t->dir, 4ull << bits)) return SHM_ENOMEM;  // 32 B per entry
    t->dir_bits = bits;
  }
  dev::launch_leaf_dir(t->arena, t->arena_bytes, t->cfg.node_id, t->root, t->cfg.key_lo,
                       t->cfg.key_bits - bits, 1ull << bits, t->dir, t->d_err, s);
  t->dir_np = t->next_page;
  t->dir_valid = true;
  return SHM_OK;
}

dev::SegArgs seg_args(shm_tree* t) {
  dev::SegArgs a{};
  a.arena = t->arena;
  a.arena_bytes = t->arena_bytes;
  a.node = t->cfg.node_id;
  a.seg_start = t->seg_start;
  a.seg_page = t->seg_page;
  a.seg_T = t->seg_T;
  a.seg_P = t->seg_P;
  a.seg_newpages = t->seg_np;
  a.seg_ver = t->seg_ver;
  a.seg_pbase = t->seg_pbase;
  a.locks = t->locks;
  a.num_locks = t->cfg.num_locks;
  a.tag_base = (t->batches + 1) << 32;
  a.err = t->d_err;
  a.leaf_hw = t->leaf_hw;
  return a;
}

// SHM_DEBUG=1: synchronise after every launch and name the failing step
bool debug_sync_enabled() {
  static const int on = [] {
    const char* e = getenv("SHM_DEBUG");
    return e && e[0] == '1' ? 1 : 0;
  }();
  return on != 0;
}
int dbg(hipStream_t s, const char* what) {
  if (!debug_sync_enabled()) return SHM_OK;
  hipError_t e = hipStreamSynchronize(s);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) {
    fprintf(stderr, "sherman_amd[debug]: %s failed: %s\n", what, hipGetErrorString(e));
    return SHM_EIO;
  }
  return SHM_OK;
}
#define DBG(s, what)                   \
  do {                                 \
    int _r = dbg((s), (what));         \
    if (_r) return _r;                 \
  } while (0)

constexpr uint32_t kFlagWord = 512;  // read-back sequence word: byte 2048 of h_pin
int readback_wait(shm_tree* t, hipStream_t s, uint32_t seq);

// SHM_ZC_READBACK=0: read-backs as a D2H copy + stream synchronisation
bool use_zc_readback() {
  static const bool on = [] {
    const char* e = getenv("SHM_ZC_READBACK");
    return !(e && strcmp(e, "0") == 0);
  }();
  return on;
}

// read `bytes` (<= 256) of device words into pinned host scratch and wait.
// Zero-copy: a one-wave kernel stores the words straight into the mapped,
// coherent host page, then a sequence number after a system-scope fence;
// the host spins on that word instead of a D2H copy (an SDMA/blit round
// trip) and a stream synchronisation.  While spinning it polls the stream,
// so a fault in an earlier kernel (which would keep the word from ever
// arriving) still returns SHM_EIO.
int readback(shm_tree* t, hipStream_t s, const void* src, size_t bytes) {
  if (!use_zc_readback()) {
    HIP_OK(hipMemcpyAsync(t->h_pin, src, bytes, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return SHM_OK;
  }
  const uint32_t seq = ++t->rb_seq;
  dev::launch_readback(t->h_pin_dev, static_cast<const uint32_t*>(src),
                       (uint32_t)((bytes + 3) / 4), t->h_pin_dev + kFlagWord, seq, s);  // <= 64
  return readback_wait(t, s, seq);
}

// the words *g.p[i] (scattered device u32s) into h_pin[0 ..] as u32s; with
// zero-copy read-backs one fused kernel, else a gather into `staging` + copy
int readback_gather(shm_tree* t, hipStream_t s, const dev::Gather8& g, uint32_t* staging) {
  if (!use_zc_readback()) {
    dev::launch_gather_u32(staging, g, s);
    return readback(t, s, staging, (size_t)g.n * sizeof(uint32_t));
  }
  const uint32_t seq = ++t->rb_seq;
  dev::launch_readback_gather(t->h_pin_dev, g, t->h_pin_dev + kFlagWord, seq, s);
  return readback_wait(t, s, seq);
}

// spin until the read-back kernel has published `seq`
int readback_wait(shm_tree* t, hipStream_t s, uint32_t seq) {
  HIP_OK(hipGetLastError());
  const uint32_t* flag = reinterpret_cast<const uint32_t*>(t->h_pin) + kFlagWord;
  for (uint32_t spin = 1;; ++spin) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return SHM_OK;
    if ((spin & 1023) == 0) {
      const hipError_t e = hipStreamQuery(s);
      if (e != hipSuccess && e != hipErrorNotReady) return SHM_EIO;
      if (e == hipSuccess && __atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) return SHM_EIO;
    }
    __builtin_ia32_pause();
  }
}

// superblock mirror (layout.h), written by a one-wave kernel: stream-ordered,
// no host synchronisation
int write_superblock(shm_tree* t, hipStream_t s) {
  Superblock sb{};
  sb.magic = kSuperMagic;
  sb.root_ptr = t->root;
  sb.root_level = t->root_level;
  sb.next_page = t->next_page;
  sb.capacity_pages = t->cap_pages;
  sb.node_id = t->cfg.node_id;
  sb.batches = t->batches;
  sb.splits = t->splits;
  dev::launch_write_superblock(t->arena, sb, s);
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

int check_err(shm_tree* t, hipStream_t s) {
  t->err_pending = false;
  int rc = readback(t, s, t->d_err, sizeof(uint32_t));
  if (rc) return rc;
  const uint32_t e = (uint32_t)t->h_pin[0];
  if (e) {
    t->sticky_err |= e;
    HIP_OK(hipMemsetAsync(t->d_err, 0, sizeof(uint32_t), s));
    fprintf(stderr, "sherman_amd: device error bits 0x%x\n", e);
    return SHM_EIO;
  }
  return SHM_OK;
}

// Segment a sorted op list by the page its walk ends on at `level`.
// Returns the segment count (or negative status); with sync == false the
// count is left in d_counts[8] and n_ops (an upper bound) is returned.
// SHM_LOCATE: 0 = header-only k_locate (default), 1 = the grouped k_get walk
// for leaves, 2 = the LDS page walk k_walk (A/B switches)
int locate_kernel() {
  static const int v = [] {
    const char* e = getenv("SHM_LOCATE");
    return e ? atoi(e) : 0;
  }();
  return v;
}

dev::SegLock seg_lock(shm_tree* t) {
  return dev::SegLock{t->locks, t->cfg.num_locks, (t->batches + 1) << 32, t->seg_lk, t->d_err};
}

// SHM_LOCK_AHEAD=0: k_leaf_upsert takes its lock words itself (A/B knob)
bool lock_ahead() {
  static const bool v = [] {
    const char* e = getenv("SHM_LOCK_AHEAD");
    return !(e && strcmp(e, "0") == 0);
  }();
  return v;
}

int64_t segment(shm_tree* t, hipStream_t s, const uint64_t* op_key,
                uint64_t n_ops, int level, bool sync = true,
                const uint64_t* n_dev = nullptr, bool lock = false) {
  dev::WalkArgs w = walk_args(t);
  w.keys = op_key;
  w.n = n_ops;
  w.n_dev = n_dev;
  w.out_page = t->pages;
  w.target_level = level;
  if (locate_kernel() != 2 && (level > 0 || use_fast_insert())) {
    // header-only descent, lane per op; leaves start at the leaf directory
    if (level == 0 && use_leaf_dir(t)) {
      const int rc = refresh_dir(t, s);
      if (rc) return rc;
      w.dir = t->dir;
      w.dir_lo = t->cfg.key_lo;
      w.dir_shift = t->cfg.key_bits - t->dir_bits;
      w.dir_n = 1ull << t->dir_bits;
    }
    if (locate_kernel() == 1 && level == 0)
      dev::launch_locate_leaf(w, n_ops, s);  // the grouped get walk (A/B)
    else
      dev::launch_locate(w, n_ops, s);
  } else {
    dev::launch_walk(w, n_ops, 4, true, s);
  }
  DBG(s, "walk(locate)");
  uint32_t* d_ns = reinterpret_cast<uint32_t*>(t->d_counts + 8);
  if (use_tile_scan()) {
    dev::launch_segment(t->pages, n_ops, n_dev, t->bsum, t->seg_start, t->seg_page, d_ns,
                        lock ? seg_lock(t) : dev::SegLock{}, s);
  } else {
    dev::launch_seg_heads(t->pages, n_ops, n_dev, t->heads, s);
    HIP_OK(dev::exclusive_scan_u32(t->temp, t->temp_bytes, t->heads, t->hpos, n_ops, s));
    if (lock)
      dev::launch_seg_fill_lock(t->pages, t->heads, t->hpos, n_ops, n_dev, t->seg_start,
                                t->seg_page, d_ns, seg_lock(t), s);
    else
      dev::launch_seg_fill(t->pages, t->heads, t->hpos, n_ops, n_dev, t->seg_start,
                           t->seg_page, d_ns, s);
  }
  DBG(s, "seg_fill");
  if (!sync) return (int64_t)n_ops;  // an upper bound; the count stays on the device
  int rc = readback(t, s, d_ns, sizeof(uint32_t));
  if (rc) return rc;
  return (int64_t)(uint32_t)t->h_pin[0];
}

// plan + scan + capacity check; returns new page count (or negative status)
int64_t new_page_total(shm_tree* t, hipStream_t s, dev::SegArgs& a, uint64_t reserve);

int64_t plan_level(shm_tree* t, hipStream_t s, dev::SegArgs& a, bool leaf,
                   uint64_t reserve) {
  if (leaf)
    dev::launch_leaf_plan(a, s);
  else
    dev::launch_int_plan(a, s);
  DBG(s, "plan");
  return new_page_total(t, s, a, reserve);
}

// scan seg_newpages into seg_pbase and read back the level's new-page total
int64_t new_page_total(shm_tree* t, hipStream_t s, dev::SegArgs& a, uint64_t reserve) {
  if (use_tile_scan())
    dev::launch_scan_u32(t->seg_np, t->seg_pbase, a.num_seg, t->bsum, s);
  else
    HIP_OK(dev::exclusive_scan_u32(t->temp, t->temp_bytes, t->seg_np, t->seg_pbase,
                                   a.num_seg, s));
  // total = pbase[last] + np[last]; with the error word, the device-side
  // segment count and the ordering's (upserts, deletes) in one read-back
  uint32_t* d_tot = reinterpret_cast<uint32_t*>(t->d_counts + 16);
  dev::Gather8 g{};
  g.p[0] = t->seg_pbase + (a.num_seg - 1);
  g.p[1] = t->seg_np + (a.num_seg - 1);
  g.p[2] = t->d_err;
  g.p[3] = reinterpret_cast<const uint32_t*>(t->d_counts + 8);
  g.p[4] = reinterpret_cast<const uint32_t*>(t->d_counts + 0);  // low words (n < 2^31)
  g.p[5] = reinterpret_cast<const uint32_t*>(t->d_counts + 1);
  g.n = 6;
  int rc = readback_gather(t, s, g, d_tot);
  if (rc) return rc;
  t->err_pending = false;
  const uint32_t* h = reinterpret_cast<const uint32_t*>(t->h_pin);
  const uint64_t total = (uint64_t)h[0] + h[1];
  t->rb_nup = h[4];
  t->rb_ndel = h[5];
  if (a.num_seg_dev) a.num_seg = h[3];  // the device-side segment count, now known
  if (h[2] & (dev::kErrKeyMax | dev::kErrSortOverflow)) {
    // the deferred ordering check (insert_chunk_impl): nothing was written
    HIP_OK(hipMemsetAsync(t->d_err, 0, 4, s));
    return (h[2] & dev::kErrKeyMax) ? SHM_EINVAL : kRedoOrder;
  }
  if (h[2]) return check_err(t, s);
  if (total > t->sep_cap) return SHM_ENOMEM;
  if (t->next_page + total + reserve > t->cap_pages) return SHM_ENOMEM;
  return (int64_t)total;
}

// Apply one level: ops sorted/unique; returns separators produced (written to
// sep[out]) or a negative status.
int64_t apply_level(shm_tree* t, hipStream_t s, const uint64_t* op_key,
                    const uint64_t* op_val, uint64_t n_ops, int level,
                    bool is_delete, int out, const uint64_t* n_dev = nullptr) {
  const bool fast_leaf = level == 0 && !is_delete && use_fast_insert();
  const bool ahead = fast_leaf && lock_ahead();
  // internal levels keep the segment count on the device too: the plan
  // kernel checks it and the new-page read-back returns it (one read-back
  // per level instead of two)
  const bool fast_int = level > 0 && use_fast_insert() && int_dev_count();
  const int64_t ns = segment(t, s, op_key, n_ops, level, !(fast_leaf || fast_int), n_dev, ahead);
  if (ns < 0) return ns;
  if (ns == 0) return 0;
  dev::SegArgs a = seg_args(t);
  a.op_key = op_key;
  a.op_val = op_val;
  a.n_ops = n_ops;
  a.num_seg = (uint32_t)ns;
  if (fast_leaf || fast_int) a.num_seg_dev = reinterpret_cast<const uint32_t*>(t->d_counts + 8);
  t->err_pending = true;
  a.level = level;
  a.is_delete = is_delete ? 1 : 0;
  a.sep_key = t->sep_key[out];
  a.sep_ptr = t->sep_ptr[out];
  if (is_delete) {
    dev::launch_leaf_delete(a, s);
    DBG(s, "leaf_delete");
    return 0;
  }
  const bool leaf = level == 0;
  // head-room for the parent levels a split of this level can trigger
  const uint64_t reserve = 2 * (uint64_t)kMaxLevelOfTree;
  int64_t total;
  if (leaf && use_fast_insert()) {
    // in-place segments are applied here; the rest go the k-way split path
    shm_tree::ProfRec* pi = t->prof_ins;
    if (pi && !pi->upsert_done) HIP_OK(hipEventRecord(pi->e[1], s));
    if (ahead) a.seg_lk = t->seg_lk;
    dev::launch_leaf_upsert(a, s);
    DBG(s, "leaf_upsert");
    if (ahead) {
      dev::launch_seg_unlock(t->seg_page, a.num_seg_dev, a.num_seg, seg_lock(t), s);
      DBG(s, "seg_unlock");
    }
    if (pi && !pi->upsert_done) {
      HIP_OK(hipEventRecord(pi->e[2], s));
      pi->upsert_done = true;
    }
    total = new_page_total(t, s, a, reserve);
    if (total <= 0) return total;
    a.split_only = 1;
  } else {
    total = plan_level(t, s, a, leaf, reserve);
  }
  if (total < 0) return total;
  a.first_new_page = t->next_page;
  if (leaf) {
    dev::launch_leaf_build(a, (uint32_t)total, s);
    DBG(s, "leaf_build");
    dev::launch_leaf_update(a, s);
    DBG(s, "leaf_update");
  } else {
    dev::launch_int_build(a, (uint32_t)total, s);
    DBG(s, "int_build");
    dev::launch_int_update(a, s);
    DBG(s, "int_update");
  }
  t->next_page += (uint64_t)total;
  t->splits += (uint64_t)total;
  return total;
}

// keys sorted with one op per key (the last writer) -> uk/uv (upserts) and
// dk (deletes); counts in t->h_pin[0..2] (upserts, deletes, error bits)
int order_and_dedup(shm_tree* t, hipStream_t s, const uint64_t* keys, const uint64_t* vals,
                    uint64_t n, bool fast) {
  const uint32_t* bins = nullptr;
  if (fast) {
    // per-tile de-dup, coarse bins, per-bin LDS sort (isort.hip)
    dev::launch_tile_dedup(keys, n, t->kb, t->ia, t->gcount, t->d_err, s);
    dev::launch_partition_coarse(t->kb, n, t->gcount, t->ia, t->cfg.key_lo, t->cfg.key_bits,
                                 t->part_hist, t->part_S, t->ka, t->ib, t->bins, s);
    if (bin_unique()) {
      // per-bin dedup + sort + emit: uk / uv / dk and the counts directly
      dev::launch_bin_unique(t->ka, t->ib, t->bins, t->cfg.key_lo, t->cfg.key_bits, vals,
                             t->ia, t->bins + 2 * dev::kCoarse, t->uk, t->uv, t->dk,
                             t->d_counts, t->part_S, t->d_err, s);
      DBG(s, "bin_unique");  // k_bin_emit also copies the error word to d_counts[2]
      t->err_pending = false;
      return readback(t, s, t->d_counts, 3 * sizeof(uint64_t));
    }
    dev::launch_bin_sort(t->ka, t->ib, t->bins, t->part_S, t->d_err, s);
    bins = t->bins;
    DBG(s, "sort(insert, fast)");
  } else {
    // stable sort (key, batch index)
    dev::launch_iota(t->ia, n, s);
    HIP_OK(dev::sort_pairs(t->temp, t->temp_bytes, keys, t->ka, t->ia, t->ib, n, s));
    DBG(s, "sort(insert)");
  }
  // keep the last writer of each key; split upserts / deletes
  dev::launch_mark_unique(t->ka, t->ib, vals, n, bins, t->flags, t->d_err, s);
  HIP_OK(dev::exclusive_scan_u64(t->temp, t->temp_bytes, t->flags, t->pos, n, s));
  dev::launch_compact_unique(t->ka, t->ib, vals, t->flags, t->pos, n, t->uk,
                             t->uv, t->dk, t->d_counts, s);
  DBG(s, "compact");
  HIP_OK(hipMemcpyAsync(t->d_counts + 2, t->d_err, 4, hipMemcpyDeviceToDevice, s));
  t->err_pending = false;
  return readback(t, s, t->d_counts, 3 * sizeof(uint64_t));
}

int insert_chunk_sync(shm_tree* t, hipStream_t s, const uint64_t* keys,
                      const uint64_t* vals, uint64_t n, bool fast);

// the split levels above the leaves, after the leaf level produced nsep
// separators into sep[cur]
int apply_upper_levels(shm_tree* t, hipStream_t s, int64_t nsep, int cur) {
  int level = 1;
  while (nsep > 0) {
    if (level > kMaxLevelOfTree) return SHM_EIO;
    if ((uint32_t)(level - 1) == t->root_level) {
      // the root split: new root above it (update_new_root, Tree.cpp:126-149)
      if (t->next_page + 1 > t->cap_pages) return SHM_ENOMEM;
      const uint64_t off = t->next_page * kPageSize;
      dev::launch_new_root(t->arena, off, t->root, (uint32_t)level, s);
      DBG(s, "new_root");
      t->next_page += 1;
      t->root = ga_make(t->cfg.node_id, off);
      t->root_level = (uint32_t)level;
    }
    const int nxt = 1 - cur;
    nsep = apply_level(t, s, t->sep_key[cur], t->sep_ptr[cur], (uint64_t)nsep,
                       level, false, nxt);
    cur = nxt;
    ++level;
  }
  return nsep < 0 ? (int)nsep : SHM_OK;
}

int insert_chunk_impl(shm_tree* t, hipStream_t s, const uint64_t* keys,
                      const uint64_t* vals, uint64_t n) {
  if (use_fast_insert() && bin_unique() && deferred_counts()) {
    // Ordering with its counts left on the device: the leaf level runs over
    // n (an upper bound) with the device-side upsert count, and the one
    // read-back after the in-place upserts returns the counts with the
    // split total.  An ordering error (kKeyMax, a bin too large) gates the
    // upsert kernel off, so nothing is written before the host sees it.
    dev::launch_tile_dedup(keys, n, t->kb, t->ia, t->gcount, t->d_err, s);
    dev::launch_partition_coarse(t->kb, n, t->gcount, t->ia, t->cfg.key_lo, t->cfg.key_bits,
                                 t->part_hist, t->part_S, t->ka, t->ib, t->bins, s);
    dev::launch_bin_unique(t->ka, t->ib, t->bins, t->cfg.key_lo, t->cfg.key_bits, vals, t->ia,
                           t->bins + 2 * dev::kCoarse, t->uk, t->uv, t->dk, t->d_counts,
                           t->part_S, t->d_err, s);
    DBG(s, "bin_unique (deferred counts)");
    const int64_t nsep = apply_level(t, s, t->uk, t->uv, n, 0, false, 0, t->d_counts);
    if (nsep == kRedoOrder) return insert_chunk_sync(t, s, keys, vals, n, false);
    if (nsep < 0) return (int)nsep;
    const uint64_t n_del = t->rb_ndel;
    int rc = apply_upper_levels(t, s, nsep, 0);
    if (rc) return rc;
    // deletes after the upserts: one op per key, so the order between them
    // does not change the contents
    if (n_del) {
      const int64_t r = apply_level(t, s, t->dk, nullptr, n_del, 0, true, 0);
      if (r < 0) return (int)r;
    }
    return SHM_OK;
  }
  return insert_chunk_sync(t, s, keys, vals, n, use_fast_insert());
}

// the ordering's counts read back before anything is applied
int insert_chunk_sync(shm_tree* t, hipStream_t s, const uint64_t* keys,
                      const uint64_t* vals, uint64_t n, bool fast) {
  // 1-2. order by key, one op per key (last writer in batch order)
  int rc = order_and_dedup(t, s, keys, vals, n, fast);
  if (rc) return rc;
  if ((uint32_t)t->h_pin[2] & dev::kErrSortOverflow) {
    // a coarse bin too large for the LDS sort (skewed keys): rocPRIM instead
    HIP_OK(hipMemsetAsync(t->d_err, 0, 4, s));
    rc = order_and_dedup(t, s, keys, vals, n, false);
    if (rc) return rc;
  }
  const uint64_t n_up = t->h_pin[0], n_del = t->h_pin[1];
  const uint32_t e = (uint32_t)t->h_pin[2];
  if (e & dev::kErrKeyMax) {  // kKeyMax in the batch: reject before mutating
    HIP_OK(hipMemsetAsync(t->d_err, 0, 4, s));
    return SHM_EINVAL;
  }
  if (e) return check_err(t, s);
  // 3. deletes (never split), then upserts
  if (n_del) {
    const int64_t r = apply_level(t, s, t->dk, nullptr, n_del, 0, true, 0);
    if (r < 0) return (int)r;
  }
  if (!n_up) return SHM_OK;
  const int64_t nsep = apply_level(t, s, t->uk, t->uv, n_up, 0, false, 0);
  if (nsep < 0) return (int)nsep;
  return apply_upper_levels(t, s, nsep, 0);
}

hipEvent_t take_event(shm_tree* t);
int prof_begin(shm_tree* t, hipStream_t s, int kind, uint64_t n, int ne, shm_tree::ProfRec& r);

// insert_chunk_impl, timed with events when profiling is on
int insert_chunk(shm_tree* t, hipStream_t s, const uint64_t* keys,
                 const uint64_t* vals, uint64_t n) {
  if (!t->prof_on) return insert_chunk_impl(t, s, keys, vals, n);
  shm_tree::ProfRec pr{};
  int rc = prof_begin(t, s, shm_tree::kProfInsert, n, 4, pr);
  if (rc) return rc;
  t->prof_ins = &pr;
  rc = insert_chunk_impl(t, s, keys, vals, n);
  t->prof_ins = nullptr;
  if (!pr.upsert_done) {  // no in-place pass ran: zero-length upsert interval
    HIP_OK(hipEventRecord(pr.e[1], s));
    HIP_OK(hipEventRecord(pr.e[2], s));
  }
  HIP_OK(hipEventRecord(pr.e[3], s));
  t->prof_pending.push_back(pr);
  return rc;
}

hipEvent_t take_event(shm_tree* t) {
  if (!t->event_pool.empty()) {
    hipEvent_t e = t->event_pool.back();
    t->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// fold finished event records into the accumulator
int drain_profile(shm_tree* t) {
  for (auto& r : t->prof_pending) {
    const int ne = r.kind == shm_tree::kProfInsert ? 4 : r.kind == shm_tree::kProfGet ? 3 : 2;
    HIP_OK(hipEventSynchronize(r.e[ne - 1]));
    float d[3] = {0.f, 0.f, 0.f};
    for (int i = 0; i + 1 < ne; ++i) HIP_OK(hipEventElapsedTime(&d[i], r.e[i], r.e[i + 1]));
    auto& a = t->prof_acc;
    if (r.kind == shm_tree::kProfGet) {
      a.calls += 1;
      a.queries += r.n;
      a.order_ms += d[0];
      a.walk_ms += d[1];
    } else if (r.kind == shm_tree::kProfInsert) {
      a.insert_calls += 1;
      a.insert_ops += r.n;
      a.insert_ms += d[0] + d[1] + d[2];
      a.upsert_ms += d[1];
    } else {
      a.range_calls += 1;
      a.range_queries += r.n;
      a.range_ms += d[0];
    }
    for (int i = 0; i < ne; ++i) t->event_pool.push_back(r.e[i]);
  }
  t->prof_pending.clear();
  return SHM_OK;
}

// start a ProfRec with `ne` events, e[0] recorded now on s
int prof_begin(shm_tree* t, hipStream_t s, int kind, uint64_t n, int ne,
               shm_tree::ProfRec& r) {
  r = shm_tree::ProfRec{{nullptr, nullptr, nullptr, nullptr}, n, kind, false};
  for (int i = 0; i < ne; ++i) {
    r.e[i] = take_event(t);
    if (!r.e[i]) return SHM_EIO;
  }
  HIP_OK(hipEventRecord(r.e[0], s));
  return SHM_OK;
}

void free_all(shm_tree* t) {
  auto F = [](void* p) {
    if (p) (void)hipFree(p);
  };
  F(t->arena); F(t->locks); F(t->d_err); F(t->d_counts); F(t->route_scratch);
  for (auto& r : t->route_ws)
    if (r.second != t->route_scratch) F(r.second);
  F(t->ka); F(t->kb); F(t->ia); F(t->ib); F(t->flags); F(t->pos);
  F(t->uk); F(t->uv); F(t->dk); F(t->pages); F(t->heads); F(t->hpos); F(t->bsum); F(t->bsum64);
  F(t->seg_start); F(t->seg_page); F(t->seg_T); F(t->seg_P); F(t->seg_np);
  F(t->seg_pbase); F(t->seg_ver); F(t->seg_lk); F(t->leaf_hw);
  for (int i = 0; i < 2; ++i) { F(t->sep_key[i]); F(t->sep_ptr[i]); }
  F(t->temp); F(t->part_hist); F(t->part_S); F(t->part_chunks); F(t->start); F(t->dir); F(t->gcount); F(t->bins);
  for (auto& r : t->prof_pending)
    for (hipEvent_t e : r.e)
      if (e) t->event_pool.push_back(e);
  for (hipEvent_t e : t->event_pool) (void)hipEventDestroy(e);
  if (t->rstage) (void)hipFree(t->rstage);
  {
    shm_tree::GetWs& w = t->gws[1];
    F(w.keys1); F(w.keys_out); F(w.pos1); F(w.src); F(w.M); F(w.S); F(w.chunks);
  }
  for (auto& r : t->shared_ev) (void)hipEventDestroy(r.ev);
  if (t->ex_ev) (void)hipEventDestroy(t->ex_ev);
  for (hipEvent_t e : t->gws_ev)
    if (e) (void)hipEventDestroy(e);
  if (t->h_pin) (void)hipHostFree(t->h_pin);
  if (t->stream) (void)hipStreamDestroy(t->stream);
}

// host-side structural check of an image (same invariants as SURVEY App. A)
int check_image(const uint8_t* img, uint64_t bytes, uint64_t root, uint16_t node,
                uint64_t* n_leaves, uint64_t* n_internal, uint64_t* n_keys) {
  auto rd64 = [&](uint64_t off) {
    uint64_t v;
    memcpy(&v, img + off, 8);
    return v;
  };
  auto page_off = [&](uint64_t ga) -> int64_t {
    if (ga == 0 || ga_node(ga) != node) return -1;
    const uint64_t o = ga_offset(ga);
    if (o < kPageSize || o + kPageSize > bytes || (o & (kPageSize - 1))) return -1;
    return (int64_t)o;
  };
  uint64_t leaves = 0, internals = 0, keys = 0;
  int64_t ro = page_off(root);
  if (ro < 0) return -1;
  int top = img[ro + kOffLevel];
  uint64_t head = root;
  for (int lvl = top; lvl >= 0; --lvl) {
    uint64_t p = head, expect_low = 0, next_head = 0;
    uint64_t guard = 0;
    while (p) {
      if (++guard > bytes / kPageSize + 1) return -20;
      const int64_t o = page_off(p);
      if (o < 0) return -2;
      const uint8_t* pg = img + o;
      const uint64_t leftmost = rd64(o + kOffLeftmost);
      const bool is_leaf = leftmost == 0;
      if (pg[kOffLevel] != lvl) return -3;
      if ((lvl == 0) != is_leaf) return -4;
      if (pg[kOffFrontVer] != pg[is_leaf ? kOffLeafRear : kOffInternalRear]) return -5;
      const uint64_t lo = rd64(o + kOffLowest), hi = rd64(o + kOffHighest);
      if (lo != expect_low || hi <= lo) return -6;
      if (is_leaf) {
        int c = 0;
        for (int i = 0; i < kLeafCardinality; ++i) {
          const uint64_t e = o + kOffRecords + (uint64_t)kLeafEntry * i;
          if (rd64(e + 9) == kValueNull) continue;
          const uint64_t k = rd64(e + 1);
          if (k < lo || k >= hi) return -7;
          ++c;
        }
        if (c > kLeafCardinality - 1) return -8;
        keys += (uint64_t)c;
        ++leaves;
      } else {
        int16_t li;
        memcpy(&li, pg + kOffLastIndex, 2);
        const int cnt = li + 1;
        if (cnt < 0 || cnt > kInternalCardinality - 1) return -9;
        if (!next_head) next_head = leftmost;
        int64_t co = page_off(leftmost);
        if (co < 0 || rd64(co + kOffLowest) != lo) return -10;
        uint64_t prev = lo;
        for (int j = 0; j < cnt; ++j) {
          const uint64_t k = rd64(o + kOffRecords + 16ull * j);
          const uint64_t c = rd64(o + kOffRecords + 16ull * j + 8);
          if (k <= prev || k >= hi) return -11;
          prev = k;
          co = page_off(c);
          if (co < 0 || rd64(co + kOffLowest) != k) return -12;
          if ((int)img[co + kOffLevel] != lvl - 1) return -13;
        }
        ++internals;
      }
      expect_low = hi;
      p = rd64(o + kOffSibling);
    }
    if (expect_low != kKeyMax) return -14;
    head = next_head;
  }
  if (n_leaves) *n_leaves = leaves;
  if (n_internal) *n_internal = internals;
  if (n_keys) *n_keys = keys;
  return 0;
}

}  // namespace

extern "C" {

int shm_abi_version(void) { return SHM_ABI_VERSION; }

const char* shm_strerror(int s) {
  switch (s) {
    case SHM_OK: return "ok";
    case SHM_EINVAL: return "invalid argument (key == kKeyMax or bad config)";
    case SHM_ENOMEM: return "page arena or workspace exhausted";
    case SHM_EIO: return "HIP failure or tree inconsistency";
    case SHM_EAGAIN: return "optimistic check failed";
    case SHM_E2BIG: return "batch larger than max_batch";
    case SHM_ENOSPC: return "output buffer too small";
    default: return "unknown status";
  }
}

int shm_config_init(shm_config* c) {
  if (!c) return SHM_EINVAL;
  memset(c, 0, sizeof(*c));
  c->struct_size = sizeof(shm_config);
  c->device = 0;
  c->node_id = 0;
  c->flags = SHM_FLAG_LEAF_DIR | SHM_FLAG_AUTO_SORT_GETS;
  c->arena_bytes = 1ull << 30;
  c->max_batch = 1ull << 20;
  c->num_locks = 1u << 22;  // 32 MB: rare false sharing between waves
  c->sort_bits = kDefaultSortBits;
  c->key_lo = 0;
  c->key_bits = 64;
  return SHM_OK;
}

int shm_tree_create(const shm_config* cfg, shm_tree** out) {
  if (!cfg || !out || cfg->struct_size != sizeof(shm_config)) return SHM_EINVAL;
  // arena < 4 TB: the leaf directory holds 32-bit page indices
  if (cfg->arena_bytes < 4 * kPageSize || cfg->arena_bytes > (1ull << 42) ||
      cfg->max_batch == 0 ||
      cfg->max_batch > (1ull << 31) || cfg->num_locks == 0 ||
      (cfg->sort_bits != 0 && cfg->sort_bits != kDefaultSortBits) || cfg->key_bits > 64)
    return SHM_EINVAL;
  shm_tree* t = new shm_tree();
  t->cfg = *cfg;
  if (!t->cfg.sort_bits || t->cfg.sort_bits > 64) t->cfg.sort_bits = kDefaultSortBits;
  if (t->cfg.key_bits == 0) t->cfg.key_bits = 64;
  if (t->cfg.key_bits == 64) t->cfg.key_lo = 0;
  auto fail = [&](int rc) {
    free_all(t);
    delete t;
    return rc;
  };
  if (hipSetDevice(cfg->device) != hipSuccess) return fail(SHM_EIO);
  if (hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) != hipSuccess)
    return fail(SHM_EIO);
  t->cap_pages = cfg->arena_bytes / kPageSize;
  t->arena_bytes = t->cap_pages * kPageSize;
  const uint64_t n = cfg->max_batch;
  t->nmax = n;
  t->sep_cap = 2 * n + 1024;
  const uint64_t segcap = t->sep_cap;
  int rc = SHM_OK;
  rc |= dalloc(&t->arena, t->arena_bytes);
  rc |= dalloc(&t->locks, cfg->num_locks);
  rc |= dalloc(&t->d_err, 4);
  rc |= dalloc(&t->d_counts, 32);
  rc |= dalloc(&t->route_scratch, dev::route_scratch_words(n));
  rc |= dalloc(&t->ka, n);
  rc |= dalloc(&t->kb, n);
  rc |= dalloc(&t->ia, n);
  rc |= dalloc(&t->ib, n);
  rc |= dalloc(&t->flags, n);
  rc |= dalloc(&t->pos, n);
  rc |= dalloc(&t->uk, n);
  rc |= dalloc(&t->uv, n);
  rc |= dalloc(&t->dk, n);
  rc |= dalloc(&t->pages, segcap);
  rc |= dalloc(&t->heads, segcap);
  rc |= dalloc(&t->hpos, segcap);
  rc |= dalloc(&t->bsum, dev::seg_tiles(segcap) + 1);
  rc |= dalloc(&t->bsum64, dev::seg_tiles(n) + 1);
  rc |= dalloc(&t->seg_start, segcap + 1);
  rc |= dalloc(&t->seg_page, segcap);
  rc |= dalloc(&t->seg_T, segcap);
  rc |= dalloc(&t->seg_P, segcap);
  rc |= dalloc(&t->seg_np, segcap);
  rc |= dalloc(&t->seg_pbase, segcap);
  rc |= dalloc(&t->seg_ver, segcap);
  rc |= dalloc(&t->seg_lk, segcap);
  rc |= dalloc(&t->leaf_hw, t->cap_pages);
  for (int i = 0; i < 2; ++i) {
    rc |= dalloc(&t->sep_key[i], t->sep_cap);
    rc |= dalloc(&t->sep_ptr[i], t->sep_cap);
  }
  rc |= dalloc(&t->part_hist, dev::kPartHistWords);
  rc |= dalloc(&t->part_S, dev::kPartGroupWords);
  rc |= dalloc(&t->part_chunks, 2 * (uint64_t)dev::partition_chunk_slots(n));
  rc |= dalloc(&t->start, 1ull << start_bits());
  rc |= dalloc(&t->gcount, n / dev::kIsortTile + 1);
  rc |= dalloc(&t->bins, 4 * dev::kCoarse);  // (start, count), then (upserts, deletes)
  // get workspaces: 0 shares the insert arrays, 1 is its own
  t->gws[0] = {t->kb, t->ka, t->ia, t->ib, t->part_hist, t->part_S, t->part_chunks};
  {
    shm_tree::GetWs& w = t->gws[1];
    rc |= dalloc(&w.keys1, n);
    rc |= dalloc(&w.keys_out, n);
    rc |= dalloc(&w.pos1, n);
    rc |= dalloc(&w.src, n);
    rc |= dalloc(&w.M, dev::kPartHistWords);
    rc |= dalloc(&w.S, dev::kPartGroupWords);
    rc |= dalloc(&w.chunks, 2 * (uint64_t)dev::partition_chunk_slots(n));
  }
  if (rc) return fail(SHM_ENOMEM);
  t->temp_bytes = std::max(dev::sort_pairs_temp_bytes(n),
                           dev::scan_temp_bytes_max(segcap));
  if (hipMalloc(&t->temp, t->temp_bytes) != hipSuccess) return fail(SHM_ENOMEM);
  if (hipHostMalloc((void**)&t->h_pin, 4096, hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void**)&t->h_pin_dev, t->h_pin, 0) != hipSuccess)
    return fail(SHM_ENOMEM);
  memset(t->h_pin, 0, 4096);
  hipStream_t s = t->stream;
  if (hipMemsetAsync(t->locks, 0, sizeof(uint64_t) * cfg->num_locks, s) ||
      hipMemsetAsync(t->d_err, 0, 16, s) ||
      hipMemsetAsync(t->part_S, 0, sizeof(uint32_t) * dev::kPartGroupWords, s) ||
      hipMemsetAsync(t->gws[1].S, 0, sizeof(uint32_t) * dev::kPartGroupWords, s) ||
      hipMemsetAsync(t->arena, 0, kPageSize, s) ||
      hipMemsetAsync(t->leaf_hw, kLeafHwFull, t->cap_pages, s))
    return fail(SHM_EIO);
  // Tree::Tree (Tree.cpp:44-60): empty leaf root
  t->next_page = 1;
  const uint64_t root_off = t->next_page * kPageSize;
  dev::launch_empty_leaf(t->arena, root_off, s);
  t->next_page += 1;
  t->root = ga_make(cfg->node_id, root_off);
  t->root_level = 0;
  if (write_superblock(t, s)) return fail(SHM_EIO);
  *out = t;
  return SHM_OK;
}

int shm_tree_destroy(shm_tree* t) {
  if (!t) return SHM_EINVAL;
  (void)hipSetDevice(t->cfg.device);
  (void)hipStreamSynchronize(t->stream);
  free_all(t);
  delete t;
  return SHM_OK;
}

int shm_search_batch(shm_tree* t, const uint64_t* keys, uint64_t n,
                     uint64_t* vals_out, uint8_t* found_out, void* stream) {
  if (!t || (n && (!keys || !vals_out))) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  hipStream_t s = pick(t, stream);
  // start pages: the leaf directory (any batch), else for ordered batches
  // the prefix start table, else the root
  // Ordering pays when queries share leaves: a batch of q uniform queries
  // over L leaves reads L(1 - e^(-q/L)) of them sorted, q unsorted (C2, q/L
  // 0.58: 24 % fewer page reads for ~35 us of partition + gather, +4 %; C3's
  // get half, q/L 0.29: 13 % fewer, -3 %).  Auto mode orders at q/L >= 0.4.
  const bool dense = (t->cfg.flags & SHM_FLAG_AUTO_SORT_GETS) && 5 * n >= 2 * t->next_page;
  const bool ordered = ((t->cfg.flags & SHM_FLAG_SORT_GETS) || dense) && n >= kSortMinGets;
  const bool dir = use_leaf_dir(t);
  Order ord(t, s, false);
  if (dir) {
    if (dir_stale(t)) ord.make_exclusive();  // the rebuild rewrites what searches read
    const int rc = ord.rc ? ord.rc : refresh_dir(t, s);
    if (rc) return rc;
  } else if (ordered && (t->start_np != t->next_page || t->start_root != t->root)) {
    ord.make_exclusive();
    dev::launch_start_table(t->arena, t->arena_bytes, t->cfg.node_id, t->root, start_bits(),
                            t->start, t->d_err, s);
    t->start_np = t->next_page;
    t->start_root = t->root;
  }
  for (uint64_t off = 0; off < n; off += t->nmax) {
    const uint64_t m = std::min(t->nmax, n - off);
    dev::WalkArgs a = walk_args(t);
    a.out_val = vals_out + off;
    a.out_found = found_out ? found_out + off : nullptr;
    a.n = m;
    bool gathered = false;
    shm_tree::ProfRec pr{};
    if (t->prof_on) {
      const int rc = prof_begin(t, s, shm_tree::kProfGet, m, 3, pr);
      if (rc) return rc;
    }
    if (ordered && m >= kSortMinGets) {
      // order the batch by its top key bits so queries that share pages are
      // walked by the same wave (one page read per group, not per query)
      // (keys1 = kb, pos1 = ia, walk order = ka, src = ib); the walk stores
      // result p at vals1[src[p]] (kb, inside p's chunk), unpartition gathers
      const bool direct = get_direct();
      const shm_tree::GetWs& w = t->gws[ord.ws >= 0 ? ord.ws : ord.take_ws()];
      if (ord.rc) return ord.rc;
      dev::launch_partition(keys + off, m, t->cfg.key_lo, t->cfg.key_bits, w.M, w.S, w.chunks,
                            w.keys1, w.pos1, w.keys_out, w.src, direct, s);
      a.keys = w.keys_out;
      a.perm = w.src;
      if (!direct) {  // else results go straight to input order (src = input index)
        a.out_val = w.keys1;
        a.out_found = nullptr;
      }
      a.xcd_remap = getenv("SHM_XCD_REMAP") ? atoi(getenv("SHM_XCD_REMAP")) : 1;
      if (dir) {
        a.dir = t->dir;
        a.dir_lo = t->cfg.key_lo;
        a.dir_shift = t->cfg.key_bits - t->dir_bits;
        a.dir_n = 1ull << t->dir_bits;
      } else {
        a.start = t->start;
        a.start_shift = 64 - start_bits();
      }
      gathered = !direct;
      DBG(s, "sort(get)");
    } else if (dir) {
      // unordered (default): every wave sorts its own 64 keys and starts at
      // the leaf directory; results land in input order (no unpartition pass).
      // With the directory a get reads one leaf, so the batch-wide key order
      // only buys page sharing between waves, which costs more to set up than
      // it saves (uniform and zipf 0.99 alike)
      a.keys = keys + off;
      a.perm = nullptr;
      a.xcd_remap = 0;
      a.dir = t->dir;
      a.dir_lo = t->cfg.key_lo;
      a.dir_shift = t->cfg.key_bits - t->dir_bits;
      a.dir_n = 1ull << t->dir_bits;
    } else {
      a.keys = keys + off;
      a.perm = nullptr;
    }
    a.nt = walk_nt(gathered || a.perm != nullptr);
    a.leaf_hw = use_leaf_hw() ? t->leaf_hw : nullptr;
    if (t->prof_on) HIP_OK(hipEventRecord(pr.e[1], s));
    if (get_kernel_v4()) {
      dev::launch_walk(a, m, kWalkDepth, false, s);
    } else {
      StampDump sd(a, m, s);
      dev::launch_get(a, m, s);
    }
    DBG(s, "walk(get)");
    if (t->prof_on) {
      HIP_OK(hipEventRecord(pr.e[2], s));
      t->prof_pending.push_back(pr);
    }
    if (gathered) {
      const shm_tree::GetWs& w = t->gws[ord.ws];
      dev::launch_unpartition(w.keys1, w.pos1, m, vals_out + off,
                              found_out ? found_out + off : nullptr, s);
      DBG(s, "gather");
    }
  }
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

int shm_insert_batch(shm_tree* t, const uint64_t* keys, const uint64_t* vals,
                     uint64_t n, void* stream) {
  if (!t || (n && (!keys || !vals))) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  Order ord(t, pick(t, stream), true);
  if (ord.rc) return ord.rc;
  hipStream_t s = pick(t, stream);
  int rc = SHM_OK;
  for (uint64_t off = 0; off < n && rc == SHM_OK; off += t->nmax) {
    const uint64_t m = std::min(t->nmax, n - off);
    rc = insert_chunk(t, s, keys + off, vals + off, m);
  }
  if (rc == SHM_OK) {
    t->batches += 1;
    rc = write_superblock(t, s);
    // kernels that ran after the last error read-back: check them now
    if (rc == SHM_OK && t->err_pending) rc = check_err(t, s);
  }
  return rc;
}

int shm_del_batch(shm_tree* t, const uint64_t* keys, uint64_t n, void* stream) {
  if (!t || (n && !keys)) return SHM_EINVAL;
  if (n == 0) return SHM_OK;
  // deletes are upserts of kValueNull (Tree.cpp:1040-1043)
  uint64_t* zeros = nullptr;
  const uint64_t m = std::min<uint64_t>(n, t->nmax);
  if (hipMalloc((void**)&zeros, m * sizeof(uint64_t)) != hipSuccess) return SHM_ENOMEM;
  hipStream_t s = pick(t, stream);
  int rc = SHM_OK;
  if (hipMemsetAsync(zeros, 0, m * sizeof(uint64_t), s) != hipSuccess) rc = SHM_EIO;
  for (uint64_t off = 0; off < n && rc == SHM_OK; off += m) {
    rc = shm_insert_batch(t, keys + off, zeros, std::min(m, n - off), stream);
  }
  (void)hipStreamSynchronize(s);
  (void)hipFree(zeros);
  return rc;
}

namespace {

dev::RangeArgs range_args(shm_tree* t, const uint64_t* from, const uint64_t* to, uint64_t n,
                          uint64_t* counts, const uint64_t* offsets, uint64_t* vals) {
  dev::RangeArgs a{};
  a.arena = t->arena;
  a.arena_bytes = t->arena_bytes;
  a.node = t->cfg.node_id;
  a.root = t->root;
  a.from = from;
  a.to = to;
  a.n = n;
  a.counts = counts;
  a.offsets = offsets;
  a.vals = vals;
  a.err = t->d_err;
  a.vals_cap = ~0ull;
  if (use_leaf_dir(t)) {
    a.dir = t->dir;
    a.dir_lo = t->cfg.key_lo;
    a.dir_shift = t->cfg.key_bits - t->dir_bits;
    a.dir_n = 1ull << t->dir_bits;
  }
  return a;
}

// one timed k_range launch
int range_launch(shm_tree* t, hipStream_t s, const dev::RangeArgs& a) {
  shm_tree::ProfRec pr{};
  if (t->prof_on) {
    const int rc = prof_begin(t, s, shm_tree::kProfRange, a.n, 2, pr);
    if (rc) return rc;
  }
  dev::launch_range(a, s);
  HIP_OK(hipGetLastError());
  if (t->prof_on) {
    HIP_OK(hipEventRecord(pr.e[1], s));
    t->prof_pending.push_back(pr);
  }
  return SHM_OK;
}

// one-chunk batches whose staging fits kRangeStageBytes keep up to
// kRangeStage values per scan from the count pass for the fill pass
int range_stage(shm_tree* t, hipStream_t s, uint64_t n, bool* staged) {
  *staged = n <= t->nmax && n * kRangeStage * 8 <= kRangeStageBytes;
  if (*staged && t->rstage_words < n * kRangeStage) {
    if (t->rstage) {
      HIP_OK(hipStreamSynchronize(s));
      HIP_OK(hipFree(t->rstage));
      t->rstage = nullptr;
      t->rstage_words = 0;
    }
    const uint64_t words = std::max<uint64_t>(n, 1u << 14) * kRangeStage;
    if (dalloc(&t->rstage, words)) return SHM_ENOMEM;
    t->rstage_words = words;
  }
  return SHM_OK;
}

}  // namespace

int shm_range_query(shm_tree* t, const uint64_t* from, const uint64_t* to,
                    uint64_t n, uint64_t* counts_out, const uint64_t* offsets,
                    uint64_t* vals_out, void* stream) {
  if (!t || (n && (!from || !to || !counts_out))) return SHM_EINVAL;
  if (offsets && !vals_out) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  hipStream_t s = pick(t, stream);
  Order ord(t, s, true);  // range workspace (scan temp, staging)
  if (ord.rc) return ord.rc;
  if (use_leaf_dir(t)) {
    const int rc = refresh_dir(t, s);
    if (rc) return rc;
  }
  t->err_pending = true;
  return range_launch(t, s, range_args(t, from, to, n, counts_out, offsets, vals_out));
}

int shm_range_query_batch(shm_tree* t, const uint64_t* from, const uint64_t* to, uint64_t n,
                          uint64_t* counts_out, uint64_t* offsets_out, uint64_t* vals_out,
                          uint64_t vals_cap, uint64_t* total_out, void* stream) {
  if (!t || !total_out || (n && (!from || !to || !counts_out || !offsets_out))) return SHM_EINVAL;
  if (vals_cap && !vals_out) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  hipStream_t s = pick(t, stream);
  Order ord(t, s, true);  // range workspace (scan temp, staging)
  if (ord.rc) return ord.rc;
  *total_out = 0;
  if (n == 0) return SHM_OK;
  if (use_leaf_dir(t)) {
    const int rc = refresh_dir(t, s);
    if (rc) return rc;
  }
  // pass 1 per chunk (the scan workspace holds nmax): counts, exclusive scan,
  // chunk total and error word back in one read.  A single chunk whose
  // staging fits kRangeStageBytes keeps its values for pass 2.
  uint64_t total = 0;
  std::vector<uint64_t> base;
  bool staged = false;
  if (const int rc = range_stage(t, s, n, &staged)) return rc;
  auto rargs = [&](uint64_t off, uint64_t m, const uint64_t* offs, uint64_t* vals) {
    dev::RangeArgs a = range_args(t, from + off, to + off, m, counts_out + off, offs, vals);
    if (staged) {
      a.stage = t->rstage;
      a.stage_cap = kRangeStage;
    }
    return a;
  };
  for (uint64_t off = 0; off < n; off += t->nmax) {
    const uint64_t m = std::min(t->nmax, n - off);
    int rc = range_launch(t, s, rargs(off, m, nullptr, nullptr));
    if (rc) return rc;
    if (use_tile_scan()) {
      dev::launch_scan_u64_total(counts_out + off, offsets_out + off, m, t->bsum64, t->d_err,
                                 t->d_counts + 12, s);
    } else {
      HIP_OK(dev::exclusive_scan_u64(t->temp, t->temp_bytes, counts_out + off,
                                     offsets_out + off, m, s));
      dev::launch_range_total(offsets_out + off, counts_out + off, m, t->d_err,
                              t->d_counts + 12, s);
    }
    rc = readback(t, s, t->d_counts + 12, 2 * sizeof(uint64_t));
    if (rc) return rc;
    if (t->h_pin[1]) return check_err(t, s);
    base.push_back(total);
    total += t->h_pin[0];
  }
  t->err_pending = false;
  *total_out = total;
  // offsets are chunk-relative until shifted by the totals before them
  for (size_t c = 1; c < base.size(); ++c) {
    const uint64_t off = c * t->nmax;
    dev::launch_add_u64(offsets_out + off, std::min(t->nmax, n - off), base[c], s);
  }
  if (total > vals_cap) return SHM_ENOSPC;  // counts / offsets stay valid
  // pass 2: values
  for (uint64_t off = 0, c = 0; off < n; off += t->nmax, ++c) {
    const uint64_t m = std::min(t->nmax, n - off);
    const int rc = range_launch(t, s, rargs(off, m, offsets_out + off, vals_out));
    if (rc) return rc;
  }
  t->err_pending = true;
  return SHM_OK;
}

int shm_range_query_batch_async(shm_tree* t, const uint64_t* from, const uint64_t* to,
                                uint64_t n, uint64_t* counts_out, uint64_t* offsets_out,
                                uint64_t* vals_out, uint64_t vals_cap, uint64_t* total_dev,
                                void* stream) {
  if (!t || !total_dev || (n && (!from || !to || !counts_out || !offsets_out)))
    return SHM_EINVAL;
  if (vals_cap && !vals_out) return SHM_EINVAL;
  if (n > t->nmax) return SHM_EINVAL;  // one chunk: offsets need no host-side base
  std::lock_guard<std::mutex> g(t->mu);
  hipStream_t s = pick(t, stream);
  Order ord(t, s, true);
  if (ord.rc) return ord.rc;
  if (n == 0) {
    HIP_OK(hipMemsetAsync(total_dev, 0, 2 * sizeof(uint64_t), s));
    return SHM_OK;
  }
  if (use_leaf_dir(t)) {
    const int rc = refresh_dir(t, s);
    if (rc) return rc;
  }
  bool staged = false;
  if (const int rc = range_stage(t, s, n, &staged)) return rc;
  dev::RangeArgs a = range_args(t, from, to, n, counts_out, nullptr, nullptr);
  if (staged) {
    a.stage = t->rstage;
    a.stage_cap = kRangeStage;
  }
  t->err_pending = true;
  int rc = range_launch(t, s, a);
  if (rc) return rc;
  // count pass -> offsets and (total, error word) into total_dev, then the
  // fill pass bounded by vals_cap; no host synchronisation
  if (use_tile_scan()) {
    dev::launch_scan_u64_total(counts_out, offsets_out, n, t->bsum64, t->d_err, total_dev, s);
  } else {
    HIP_OK(dev::exclusive_scan_u64(t->temp, t->temp_bytes, counts_out, offsets_out, n, s));
    dev::launch_range_total(offsets_out, counts_out, n, t->d_err, total_dev, s);
  }
  if (!vals_cap) return SHM_OK;
  a.offsets = offsets_out;
  a.vals = vals_out;
  a.vals_cap = vals_cap;
  return range_launch(t, s, a);
}

int shm_stats(shm_tree* t, shm_stats_t* o) {
  if (!t || !o) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  memset(o, 0, sizeof(*o));
  o->root_ptr = t->root;
  o->root_level = t->root_level;
  o->height = t->root_level + 1;
  o->pages_used = t->next_page - 1;
  o->pages_capacity = t->cap_pages - 1;
  o->arena_bytes = t->arena_bytes;
  o->batches = t->batches;
  o->splits = t->splits;
  o->last_error = t->sticky_err;
  return SHM_OK;
}

int shm_read_words(shm_tree* t, const void* src, uint64_t bytes, void* host_out,
                   void* stream) {
  if (!t || !src || !host_out || bytes == 0 || bytes > 256 || (bytes & 3)) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  const int rc = readback(t, pick(t, stream), src, bytes);
  if (rc) return rc;
  memcpy(host_out, t->h_pin, bytes);
  return SHM_OK;
}

int shm_synchronize(shm_tree* t) {
  if (!t) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  HIP_OK(hipDeviceSynchronize());
  return check_err(t, t->stream);
}

int shm_dump_image(shm_tree* t, void* host_buf, uint64_t cap,
                   uint64_t* bytes_used, uint64_t* root_ptr) {
  if (!t) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  const uint64_t used = t->next_page * kPageSize;
  if (bytes_used) *bytes_used = used;
  if (root_ptr) *root_ptr = t->root;
  if (!host_buf) return SHM_OK;
  if (cap < used) return SHM_EINVAL;
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(host_buf, t->arena, used, hipMemcpyDeviceToHost));
  return SHM_OK;
}

int shm_load_image(shm_tree* t, const void* host_buf, uint64_t bytes,
                   uint64_t root_ptr) {
  if (!t || !host_buf || bytes < 2 * kPageSize) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  const uint64_t pages = (bytes + kPageSize - 1) / kPageSize;
  if (pages > t->cap_pages || ga_node(root_ptr) != t->cfg.node_id) return SHM_EINVAL;
  const uint64_t ro = ga_offset(root_ptr);
  if (ro < kPageSize || ro + kPageSize > bytes) return SHM_EINVAL;
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(t->arena, host_buf, bytes, hipMemcpyHostToDevice));
  // occupancy unknown for the loaded pages: whole-page reads until rewritten
  HIP_OK(hipMemset(t->leaf_hw, kLeafHwFull, t->cap_pages));
  t->root = root_ptr;
  t->root_level = reinterpret_cast<const uint8_t*>(host_buf)[ro + kOffLevel];
  t->next_page = pages;
  t->start_np = ~0ull;  // contents changed: rebuild the get start table
  t->dir_valid = false;  // and the leaf directory
  Order ord(t, t->stream, true);
  return write_superblock(t, t->stream);
}

int shm_check(shm_tree* t, uint64_t* n_leaves, uint64_t* n_internal,
              uint64_t* n_keys) {
  if (!t) return SHM_EINVAL;
  uint64_t used = 0, root = 0;
  int rc = shm_dump_image(t, nullptr, 0, &used, &root);
  if (rc) return rc;
  std::vector<uint8_t> img(used);
  rc = shm_dump_image(t, img.data(), used, &used, &root);
  if (rc) return rc;
  rc = check_image(img.data(), used, root, t->cfg.node_id, n_leaves, n_internal, n_keys);
  if (rc) {
    fprintf(stderr, "sherman_amd: structural check failed (%d)\n", rc);
    return SHM_EIO;
  }
  return SHM_OK;
}

int shm_profile_enable(shm_tree* t, int on) {
  if (!t) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  t->prof_on = on != 0;
  return SHM_OK;
}

int shm_profile_read(shm_tree* t, shm_profile_t* out, int reset) {
  if (!t || !out) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  int rc = drain_profile(t);
  if (rc) return rc;
  *out = t->prof_acc;
  if (reset) t->prof_acc = shm_profile_t{};
  return SHM_OK;
}

int shm_route_bucket(shm_tree* t, const uint64_t* keys, uint64_t n,
                     uint32_t num_shards, uint64_t* counts_out,
                     uint64_t* keys_out, uint32_t* perm_out, void* stream) {
  if (!t || num_shards == 0 || num_shards > 64 || !counts_out) return SHM_EINVAL;
  if (n && (!keys || !keys_out || !perm_out)) return SHM_EINVAL;
  if (n > t->nmax) return SHM_E2BIG;
  std::lock_guard<std::mutex> g(t->mu);
  hipStream_t s = pick(t, stream);
  Order ord(t, s, false);  // reads only the caller's keys; scratch per stream
  if (ord.rc) return ord.rc;
  uint32_t* scratch = nullptr;
  for (auto& r : t->route_ws)
    if (r.first == s) scratch = r.second;
  if (!scratch) {
    if (t->route_ws.empty()) {
      scratch = t->route_scratch;
    } else if (dalloc(&scratch, dev::route_scratch_words(t->nmax))) {
      return SHM_ENOMEM;
    }
    t->route_ws.push_back({s, scratch});
  }
  dev::launch_route_bucket(keys, n, num_shards, counts_out, keys_out, perm_out, scratch, s);
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

int shm_route_permute(shm_tree* t, const uint64_t* in, const uint32_t* perm,
                      uint64_t n, uint64_t* out, void* stream) {
  if (!t || (n && (!in || !perm || !out))) return SHM_EINVAL;
  dev::launch_permute(in, perm, n, out, pick(t, stream));
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

int shm_route_unpermute(shm_tree* t, const uint64_t* in, const uint32_t* perm,
                        uint64_t n, uint64_t* out, void* stream) {
  if (!t || (n && (!in || !perm || !out))) return SHM_EINVAL;
  dev::launch_unpermute(in, perm, n, out, nullptr, pick(t, stream));
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

int shm_route_unpermute_found(shm_tree* t, const uint64_t* in, const uint32_t* perm,
                              uint64_t n, uint64_t* out, uint8_t* found_out, void* stream) {
  if (!t || (n && (!in || !perm || !out || !found_out))) return SHM_EINVAL;
  dev::launch_unpermute(in, perm, n, out, found_out, pick(t, stream));
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

int shm_gen_keys(shm_tree* t, uint64_t first, uint64_t n, uint64_t keyspace,
                 uint64_t* keys_out, void* stream) {
  if (!t || (n && !keys_out)) return SHM_EINVAL;
  dev::launch_gen_keys(first, n, keyspace, keys_out, pick(t, stream));
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

int shm_hash_keys(shm_tree* t, const uint64_t* ids, uint64_t n, uint64_t keyspace,
                  uint64_t* keys_out, void* stream) {
  if (!t || (n && (!ids || !keys_out))) return SHM_EINVAL;
  dev::launch_hash_ids(ids, n, keyspace, keys_out, pick(t, stream));
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

}  // extern "C"

// ---- internal test hooks (not part of include/sherman_amd.h) ----------------
extern "C" int shm__debug_sort(shm_tree* t, const uint64_t* keys, uint64_t n,
                               uint64_t* keys_out, uint32_t* perm_out,
                               unsigned begin_bit, void* stream) {
  if (!t || n > t->nmax) return SHM_EINVAL;
  hipStream_t s = pick(t, stream);
  (void)begin_bit;
  dev::launch_iota(t->ia, n, s);
  HIP_OK(dev::sort_pairs(t->temp, t->temp_bytes, keys, keys_out, t->ia, perm_out,
                         n, s));
  HIP_OK(hipStreamSynchronize(s));
  return SHM_OK;
}

extern "C" int shm__debug_walk(shm_tree* t, const uint64_t* keys,
                               const uint32_t* perm, uint64_t n, uint64_t* vals,
                               uint8_t* found, int depth, void* stream) {
  if (!t) return SHM_EINVAL;
  hipStream_t s = pick(t, stream);
  dev::WalkArgs a = walk_args(t);
  a.keys = keys;
  a.perm = perm;
  a.n = n;
  a.out_val = vals;
  a.out_found = found;
  dev::launch_walk(a, n, depth, false, s);
  HIP_OK(hipStreamSynchronize(s));
  return SHM_OK;
}
