// tree.cpp — host runtime behind the C-ABI (include/sherman_amd.h).
//
// Owns one shard's HBM page arena, lock table and batch workspace, and issues
// the kernels of get.hip / isort.hip / upsert.hip / insert.hip / range.hip /
// util.hip.  The roles of the reference's DSM (include/DSM.h:33-176: remote
// read/write/CAS, alloc), the Directory's root publication
// (src/Directory.cpp:72-83) and the Local/GlobalAllocator
// (include/LocalAllocator.h, GlobalAllocator.h) are taken by: plain HBM
// pointers, a device bump allocator (the superblock's next_page in page 0,
// advanced by k_upper) and a root page that never moves.  An insert batch is
// issued without any host wait: the host keeps a lagging mirror of the
// superblock (published by k_upper into mapped host memory) for heuristics
// only (directory staleness, get ordering) and reads exact values at
// synchronising calls.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <optional>
#include <thread>
#include <vector>

#include "../../include/sherman_amd.h"
#include "kernels.h"
#include "layout.h"

using namespace shm;

namespace {

constexpr uint64_t kSortMinGets = 8192;   // below this, walk in input order
constexpr uint32_t kDefaultSortBits = 16; // top key bits that order gets (8 + 8)
constexpr uint32_t kRangeStage = 160;      // staged values per range scan
constexpr uint64_t kRangeStageBytes = 256ull << 20;  // staging budget
constexpr uint32_t kFlagWord = 512;        // read-back sequence word: byte 2048 of h_pin
constexpr uint32_t kPubWord = 768;         // superblock mirror: u64 words 384.. of h_pin
constexpr int kAppWaitMs = 5;              // insert_order's host wait before an event fallback
// polls of an earlier segmentation tile's word before a tile counts that
// tile's staged heads itself (seg_tile.h; ~1 ms, far past a placed tile's
// few microseconds)
constexpr uint32_t kSegSelfAfter = 1024;

}  // namespace

struct shm_tree {
  shm_config cfg{};
  hipStream_t stream = nullptr;
  uint8_t* arena = nullptr;
  uint64_t arena_bytes = 0;
  uint64_t cap_pages = 0;
  uint64_t* locks = nullptr;
  uint64_t* stamps = nullptr;  // k_upper phase clock (shm__upper_stamps), off when null
  uint32_t* d_err = nullptr;
  uint64_t* d_counts = nullptr;  // 16 words of device scratch
  uint32_t* route_scratch = nullptr;
  // route_bucket scratch per stream (route_scratch serves the first one), so
  // routed batches on distinct streams bucket concurrently
  std::vector<std::pair<hipStream_t, uint32_t*>> route_ws;
  uint64_t* h_pin = nullptr;     // 4 KB pinned host scratch (coherent, mapped)
  uint32_t* h_pin_dev = nullptr; // its device address (zero-copy read-backs)
  uint32_t rb_seq = 0;           // last zero-copy read-back sequence number
  uint64_t* rstage = nullptr;    // range-scan value staging (RangeArgs.stage)
  uint64_t rstage_words = 0;
  // root page (fixed; a root split relocates the left half, insert.hip) and
  // the host mirror of the device superblock (lagging between syncs)
  uint64_t root = 0;
  uint32_t root_level = 0;
  uint64_t next_page = 0;
  uint64_t splits = 0;
  uint64_t batches = 0;   // mutating API calls
  uint32_t chunks = 0;    // insert chunks issued (the device-side tag)
  uint32_t sticky_err = 0;
  // workspace (sized for cfg.max_batch)
  uint64_t nmax = 0, sep_cap = 0;
  uint64_t *ka = nullptr, *kb = nullptr;
  uint32_t *ia = nullptr, *ib = nullptr, *ic = nullptr;
  uint64_t* kc = nullptr;  // tile-mode ordering scratch (insert_order)
  uint32_t* id = nullptr;
  uint64_t *uk = nullptr, *uv = nullptr, *dk = nullptr;
  uint64_t* pages = nullptr;
  uint64_t* seg_lb = nullptr;  // tagged per-tile staged-head counts (launch_segment)
  uint64_t* bsum64 = nullptr;  // tagged tile words of launch_scan_u64_total
  uint32_t scan_seq = 0;
  uint32_t* seg_start = nullptr;
  uint32_t* seg_end = nullptr;
  uint64_t* seg_page = nullptr;
  uint32_t *seg_T = nullptr, *seg_P = nullptr, *seg_np = nullptr, *seg_ver = nullptr;
  uint8_t* leaf_hw = nullptr;   // per-page occupancy bound (layout.h kLeafHwFull)
  uint8_t* sum = nullptr;       // leaf summaries, kSumBytes per page (layout.h)
  // upsert staging verdicts: per op the slot it overwrites (k_locate), per
  // page the last chunk tag that brought it a new key
  uint32_t* oslot = nullptr;
  uint8_t* pnew = nullptr;  // per page: dev::new_mark(tag) of the last chunk that gave it a new key
  // k_upper state (insert.hip)
  dev::UpperCtl* ctl = nullptr;
  uint64_t* leaf_rd = nullptr;
  // shm__upper_force: bit 0 = the next chunk's k_upper gives up at its first
  // hand-off, bit 1 = it propagates through the level lists (no direct path),
  // bit 2 = its upsert kernel leaves every split to k_upper (any bit does)
  uint32_t force_flags = 0;
  // shm_last_error: the last synchronising call that saw device error bits
  shm_error_t last_error{};
  uint64_t *sep_key[2] = {nullptr, nullptr}, *sep_ptr[2] = {nullptr, nullptr};
  uint64_t* ipage[2] = {nullptr, nullptr};
  uint32_t *h_end = nullptr, *h_T = nullptr, *h_P = nullptr, *h_ver = nullptr, *h_lk = nullptr;
  uint32_t *d_head = nullptr, *d_base = nullptr;
  uint64_t* int_rd = nullptr;
  uint32_t* part_hist = nullptr;  // [kMaxTiles][kCoarse] coarse tile counts
  uint32_t* part_S = nullptr;     // coarse group sums (zero between batches)
  uint32_t* part_mx = nullptr;    // [kCoarse][kMaxTiles] tile mode: each bin's run offset in a tile
  uint32_t* part_mt = nullptr;    // [kCoarse][kMaxTiles] tile mode: each bin's run length in a tile
  uint32_t* part_chunks = nullptr;  // fine-pass chunk table
  uint32_t* gcount = nullptr;       // insert ordering: survivors per 4096-op tile
  uint32_t* bins = nullptr;         // insert ordering: (start, count) per coarse bin
  // leaf directory (leafdir.hip): 2^dir_bits entries of 64 B over the shard's
  // key range, rebuilt before a search once the tree grew by 1/32 since the
  // last build (stale entries only cost B-link right moves)
  bool err_pending = false;  // kernels ran since d_err was last read back
  uint32_t reads_since_write = 0;  // search calls since the last insert chunk (dir_stale)
  uint64_t pub_batch = 0;          // the chunk tag the mirror last showed (mirror)
  uint64_t pub_seen = 0;           // the tag at the last quiet-rule look (insert_apply)
  uint64_t np_seen = 0;            // the page count then
  uint32_t quiet_chunks = 0;       // published chunks in a row that left it unchanged
  uint64_t* dir = nullptr;
  uint32_t dir_bits = 0;
  uint32_t* dir_hint = nullptr;  // per prefix: the level-1 / level-2 page on its path
  uint64_t dir_np = 0;
  bool dir_valid = false;
  bool dir_pairs = false;  // the directory is in pair form (a read phase's build)
  bool hint_ok = false;  // dir_hint holds the last build's pages of this tree
  // the allocation: 2^dir_cap_bits entries (a build may use fewer); never
  // shrunk, so a change of form or phase reallocates nothing
  uint32_t dir_cap_bits = 0;
  uint32_t dir_bits_limit = 64;  // an allocation this large failed: not asked again
  uint64_t dir_mem_limit = 0;    // shm__dir_mem_limit (test hook): bytes, 0 = none
  // rebuild cost: timing events around each build, read once they completed
  hipEvent_t dir_ev[2] = {nullptr, nullptr};
  bool dir_ev_pending = false;
  uint64_t dir_builds = 0;
  double dir_last_ms = -1.0, dir_total_ms = 0.0;
  bool dir_maint = false;    // the writers keep the entries current (dir_maint_enabled)
  // the insert chunks' repair lists (dir_upkeep.h, k_dir_repair): prefix
  // indices, and a count per chunk parity
  uint32_t* dir_fix = nullptr;
  uint32_t* dir_fix_n = nullptr;
  uint32_t dir_fix_cap = 0;
  uint64_t dir_lost_at_build = 0;  // the host word kPubDirLost at the last build
  uint64_t dir_work_seen = 0;      // the host words kPubDirWork / kPubDirUpkeeps at the last look
  uint64_t dir_upk_seen = 0;
  uint32_t dir_idle_upkeeps = 0;   // finished upkeeps in a row that found nothing to do
  bool dir_off = false;      // no directory could be allocated: walks from the root
  bool dir_exact = false;    // built with upkeep on, and upkeep on ever since (WalkArgs.dir_exact)
  bool dir_maint_always = false;  // shm__dir_config maint 2: every chunk keeps it (tests)
  bool dir_last_upkept = false;   // the previous chunk kept the directory
  double dir_debt_ps = 0.0;  // gets' estimated extra cost on shared prefixes since the build
  // LDS replica of the top of the tree (SHM_FLAG_TOP_LDS without the
  // directory; launch_top), rebuilt with the same staleness rule
  uint64_t* top_keys = nullptr;
  uint32_t* top_pages = nullptr;
  uint64_t* top_scratch = nullptr;
  uint32_t top_n = 0;
  uint64_t top_np = 0;
  bool top_valid = false;
  // index statistics of the get walk (shm_index_stats), when prof_stats
  uint64_t* idx_stats = nullptr;
  // per-chunk insert counts while profiling (UpperArgs.prof): unique
  // upserts, deletes, staged segments
  uint64_t* prof_ins = nullptr;
  bool prof_stats = false;
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
    int clk = -1;         // a get walk's clock slot in prof_clk (k_get_sum), or -1
    uint64_t blocks = 0;  // its grid
  };
  // the summary walk's device clock words while profiling (WalkArgs.clk):
  // kClkSlots launches of (blocks + 4 blocks) words, reused round robin
  static constexpr int kClkSlots = 16;
  uint64_t* prof_clk = nullptr;
  uint64_t clk_words = 0;  // per slot
  int clk_next = 0, clk_live = 0;
  double clk_khz = 0.0;
  std::vector<ProfRec> prof_pending;
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
  // A call's completion point on its stream, recorded lazily (Order): the
  // event is recorded at the stream's tail only when a call on another
  // stream first has to follow it -- an event record between two kernels
  // leaves the device idle ≈ 4.6 µs (tools/event_gap.hip), so none is placed
  // where nobody waits.  The tail then holds everything issued there so far:
  // the first waiter may wait for a little more than it needs, never less.
  struct Mark {
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;
    bool valid = false;     // a call to follow exists
    bool recorded = false;  // ev marks it (recorded at the first wait)
  };
  std::vector<Mark> shared_ev;  // last shared calls per stream, since the last exclusive one
  Mark ex;                      // last exclusive call
  // insert ordering pipeline.  The ordering of chunk `tag` writes the op
  // buffers of parity tag & 1 (uk / uv / dk / counts, op_keys() below),
  // which the apply of chunk tag - 2 read last (app_tag / app_m); every ordering
  // reuses the ordering scratch (ka .. bins), so it follows the previous
  // ordering (ord_ev).  A later chunk's ordering may therefore run on
  // another stream beside this chunk's apply.
  // (app: the apply's chunk tag, which its k_upper publishes in the host
  // mirror once it is done with the op buffers, and a lazily recorded mark
  // of its stream; ord: a lazily recorded mark)
  uint64_t app_tag[2] = {0, 0};
  bool app_valid[2] = {false, false};
  Mark app_m[2];
  Mark ord;
  // chunks ordered by shm_insert_order and not yet applied, oldest first
  struct Pending {
    uint32_t tag;
    uint64_t n;
    ProfRec pr;
    hipEvent_t ev;  // the ordering done (on s)
    hipStream_t s;
  };
  Pending pend[2];
  int n_pend = 0;
  Mark gws_m[2];  // last user of each get workspace
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
hipStream_t pick(void* s) { return (hipStream_t)s; }

// Cross-stream ordering events of one device: recording one needs no
// system-scope release and waiting on one no system-scope acquire (the
// streams share the device's memory; the host reads device results through
// copies or the read-back kernel's own system-scope fence, never through
// these events).  Default HIP events fence at system scope: a write-back of
// the L2s at every record, measured as 12-22 us gaps around each C5 step's
// cross-stream wait (round 4 A/B, tools/ab_events.sh: C2 +0.7 %, C3 +4.7 %,
// C5 +3.1 % with device scope; the system-fence switch is gone).
unsigned event_flags() { return (unsigned)(hipEventDisableTiming | hipEventDisableSystemFence); }

// INVARIANT: events from new_event() order streams of this device and
// nothing else.  They are only ever passed to hipEventRecord and
// hipStreamWaitEvent; never host-queried (hipEventSynchronize /
// hipEventQuery) and never relied on to make device writes visible to the
// host or to another device: with hipEventDisableSystemFence their record
// does not write back the L2s.  Host-facing completion goes through
// take_event() (HIP's default events: the profiler's timing) or the
// read-back kernel's system-scope release (readback below).
hipEvent_t new_event() {
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, event_flags()) != hipSuccess) return nullptr;
  return e;
}

// stream s follows the call mark m notes (its stream's tail, recorded at the
// first wait: shm_tree::Mark)
int follow(shm_tree::Mark& m, hipStream_t s) {
  if (!m.valid || m.s == s) return SHM_OK;
  if (!m.recorded) {
    if (!m.ev) m.ev = new_event();
    if (!m.ev || hipEventRecord(m.ev, m.s) != hipSuccess) return SHM_EIO;
    m.recorded = true;
  }
  return hipStreamWaitEvent(s, m.ev, 0) == hipSuccess ? SHM_OK : SHM_EIO;
}
void note(shm_tree::Mark& m, hipStream_t s) {
  m.s = s;
  m.valid = true;
  m.recorded = false;
}

// Cross-stream ordering of one API call (shm_tree: shared / exclusive calls).
// Constructed under t->mu before the call's first launch; the destructor
// notes the call's stream (no event: shm_tree::Mark).  Waits are skipped for
// marks of the same stream (stream order already covers them).
struct Order {
  shm_tree* t;
  hipStream_t s;
  bool ex;
  int ws = -1;  // get workspace used by a shared call (-1: none)
  int rc = SHM_OK;
  Order(shm_tree* tt, hipStream_t ss, bool exclusive) : t(tt), s(ss), ex(exclusive) {
    wait(t->ex);
    if (ex) {
      for (auto& m : t->shared_ev) wait(m);
      for (int j = 0; j < 2; ++j) wait(t->gws_m[j]);
    }
  }
  // a shared call that turns exclusive (a directory rebuild)
  void make_exclusive() {
    if (ex) return;
    ex = true;
    for (auto& m : t->shared_ev) wait(m);
    for (int j = 0; j < 2; ++j) wait(t->gws_m[j]);
  }
  // take the next get workspace; returns its index
  int take_ws() {
    ws = t->next_gws;
    t->next_gws ^= 1;
    if (!ex) wait(t->gws_m[ws]);
    return ws;
  }
  void wait(shm_tree::Mark& m) {
    if (follow(m, s) != SHM_OK) rc = SHM_EIO;
  }
  ~Order() {
    if (ex) {
      // the waits above ordered this call after every earlier one
      note(t->ex, s);
      for (auto& m : t->shared_ev) m.valid = false;
      t->gws_m[0].valid = t->gws_m[1].valid = false;
      return;
    }
    shm_tree::Mark* r = nullptr;
    for (auto& m : t->shared_ev)
      if (m.s == s) r = &m;
    if (!r) {
      for (auto& m : t->shared_ev)
        if (!m.valid) r = &m;  // a slot of a stream no call waits for any more
      if (!r) {
        t->shared_ev.push_back(shm_tree::Mark{});
        r = &t->shared_ev.back();
      }
    }
    note(*r, s);
    if (ws >= 0) note(t->gws_m[ws], s);
  }
};

dev::WalkArgs walk_args(shm_tree* t) {
  dev::WalkArgs a{};
  a.arena = t->arena;
  a.arena_bytes = t->arena_bytes;
  a.node = t->cfg.node_id;
  a.root = t->root;
  a.err = t->d_err;
  a.leaf_hw = t->leaf_hw;
  a.sum = t->sum;
  return a;
}

bool use_leaf_dir(const shm_tree* t) { return (t->cfg.flags & SHM_FLAG_LEAF_DIR) != 0; }
bool use_top(const shm_tree* t) {
  return !use_leaf_dir(t) && (t->cfg.flags & SHM_FLAG_TOP_LDS) != 0;
}

// the superblock mirror k_upper publishes into h_pin (kPubWord): {chunk tag,
// next_page, root_level, splits}; exact once the device is idle
void mirror(shm_tree* t) {
  const volatile uint64_t* p = reinterpret_cast<const volatile uint64_t*>(t->h_pin) + kPubWord / 2;
  t->pub_batch = p[0];  // first: the words below are at least this chunk's
  t->next_page = p[1];
  t->root_level = (uint32_t)p[2];
  t->splits = p[3];
}

void publish_host(shm_tree* t) {
  volatile uint64_t* p = reinterpret_cast<volatile uint64_t*>(t->h_pin) + kPubWord / 2;
  p[1] = t->next_page;
  p[2] = t->root_level;
  p[3] = t->splits;
  p[0] = t->chunks;
}

// (re)build the leaf directory when missing or the tree grew by > 1/32;
// 2^bits entries with bits = ceil(log2(pages)) (~1 entry per leaf)
// ... and in a read phase (kReadPhase searches since the last insert chunk)
// once the tree changed at all since the last build: a read-only workload
// (C2) then runs on an exact directory, with no B-link right moves left
// from the pages the last 1/32 of growth split (0.039 per get at C2 before
// this rule: each one a header and a summary read)
constexpr uint32_t kReadPhase = 4;
// ... and likewise once the tree has gone quiet: the mirror showed
// kQuietChunks newer chunk tags in a row with the same page count (updates
// only, C3's mix after the load; while the directory is behind, every chunk
// publishes its tag, UpperArgs.pub_always), so a write-heavy workload that no
// longer splits also gets one rebuild instead of running on the directory of
// up to 1/32 growth ago (C3 lost 7 % to 0.01 right moves per get when the
// load's last rebuild fell early).  A mirror that merely lags (the host ahead
// of the device) shows no newer tag, so it never looks quiet
constexpr uint32_t kQuietChunks = 2;
// finished directory upkeeps in a row with no new key and no split page after
// which the chunks stop keeping the directory (insert_apply)
constexpr uint32_t kIdleUpkeeps = 2;

// Directory entries per tree page, as a power of two (SHM_DIR_EXTRA_BITS
// overrides both): eight 64 B entries per page while the tree is written
// (late round 5, with the shared candidate rounds and a quiet phase's pair
// form: same box C3 15671 / 15171 -> 15994 / 16078 Mops/s against four, C5
// unchanged; sixteen no better), and sixteen in a
// read phase, in pair form (every C2 get answered from its entry, 2 GB at
// C2's 2^26 keys): same box, C2 18200 / 18217 at four, 18941 / 18964 at
// eight, 19651 / 19685 Mops/s at sixteen (DESIGN §3 "The pair form")
uint32_t dir_extra_bits(bool read_phase) {
  static const int env = [] {
    const char* e = getenv("SHM_DIR_EXTRA_BITS");
    return e ? atoi(e) : -1;
  }();
  const int v = env >= 0 ? env : read_phase ? 4 : 3;
  return (uint32_t)(v > 4 ? 4 : v);
}
bool read_phase(const shm_tree* t) { return t->reads_since_write >= kReadPhase; }
uint32_t dir_bits_for(const shm_tree* t, bool rp) {
  uint32_t bits = 10;
  while (bits < 24 && (1ull << bits) < t->next_page) ++bits;
  bits += dir_extra_bits(rp);
  if (bits > 25) bits = 25;  // 2 GB of entries at most
  if (bits > t->cfg.key_bits) bits = t->cfg.key_bits;  // one entry per key at most
  if (bits > t->dir_bits_limit) bits = t->dir_bits_limit;  // a larger allocation failed
  return bits;
}
// The form of the next build: pairs while no page is added (a read phase,
// or a write phase whose chunks leave the page count as it is: C3's
// updates), fingerprints while the tree grows (C5: a pair build reads every
// leaf).  The form only changes at a rebuild the staleness rules call for
// anyway (and once when a read phase starts), so sporadic splits cause no
// rebuilds of their own.
bool want_pairs(const shm_tree* t) {
  return read_phase(t) || t->quiet_chunks >= kQuietChunks;
}

// Directory upkeep by the writers (SHM_DIR_MAINT, default on, VERDICT r5
// #3): an insert chunk keeps the entries it affects current -- a new key in
// an empty slot adds its pair (pair form) or its fingerprint (fingerprint
// form) to its prefix's entry, and every page a split writes rewrites the
// entries of the prefixes that lie wholly inside its fences (one leaf, its
// keys' slots) and leaves the one or two prefixes it shares with a
// neighbour to the summary walk (kDirPairsBad / kDirFp cleared).  The
// directory then goes stale only by those shared prefixes, about two per
// page a split adds, and by density (the tree doubling); a rebuild is
// bought when the gets' estimated extra cost on the shared prefixes has
// reached the measured cost of one build (ski rental: at most twice the
// best offline choice).  SHM_DIR_MAINT=0: the writers leave the directory
// alone and round 5's rules rebuild it (growth by 1/32, every read phase
// after a change).
bool dir_maint_enabled() {
  static const bool on = [] {
    const char* e = getenv("SHM_DIR_MAINT");
    return !(e && e[0] == '0');
  }();
  return on;
}
// a get that starts at a stale entry reads the leaf's summary line (and may
// turn right): about one 128 B request more than an exact entry's (2.18
// requests per get at C2, 51 ps per get at 19.5 G gets/s: DESIGN §3)
constexpr double kSharedPrefixGetPs = 25.0;
// the cost of a build before one was measured: 100 ps per entry (k_leaf_dir
// + k_dir_pairs at 2^25 entries: 3.1-3.4 ms, profiles/r05)
constexpr double kBuildPsPerEntry = 100.0;

double dir_build_ps(const shm_tree* t) {
  return t->dir_last_ms > 0 ? t->dir_last_ms * 1e9 : kBuildPsPerEntry * (double)(1ull << t->dir_bits);
}
// the host word the repair kernel adds its lost repairs to (cumulative)
uint64_t dir_lost(const shm_tree* t) {
  return reinterpret_cast<const volatile uint64_t*>(t->h_pin)[kPubWord / 2 + dev::kPubDirLost];
}
// the fraction of entries left stale since the last build: the repairs the
// chunks could not list (k_dir_repair's count past its list)
double dir_shared_frac(const shm_tree* t) {
  if (!t->dir_valid) return 0.0;
  const uint64_t l = dir_lost(t);
  if (l <= t->dir_lost_at_build) return 0.0;
  const double f = (double)(l - t->dir_lost_at_build) / (double)(1ull << t->dir_bits);
  return f < 1.0 ? f : 1.0;
}

bool dir_stale(const shm_tree* t) {
  if (t->dir_off) return false;
  if (!t->dir_valid) return true;
  const bool rp = read_phase(t);
  if (t->dir_maint && t->dir_exact) {
    if (want_pairs(t) && !t->dir_pairs) return true;   // the form a read / quiet phase wants
    if (dir_bits_for(t, rp) > t->dir_bits) return true;  // a read phase's density, or the tree doubled
    return dir_lost(t) != t->dir_lost_at_build && t->dir_debt_ps >= dir_build_ps(t);
  }
  if (t->next_page > t->dir_np + t->dir_np / 32) return true;
  // a read phase also wants its denser directory, once
  if (rp && (t->dir_bits < dir_bits_for(t, true) || !t->dir_pairs)) return true;
  return t->next_page != t->dir_np && (rp || t->quiet_chunks >= kQuietChunks);
}

// a search of n keys: its estimated extra cost on the shared prefixes
void dir_note_gets(shm_tree* t, uint64_t n) {
  if (t->dir_maint && t->dir_exact) t->dir_debt_ps += (double)n * dir_shared_frac(t) * kSharedPrefixGetPs;
}

// the last build's device time once its end event completed (wait: block
// for it)
int dir_poll(shm_tree* t, bool wait) {
  if (!t->dir_ev_pending) return SHM_OK;
  const hipError_t q = wait ? hipEventSynchronize(t->dir_ev[1]) : hipEventQuery(t->dir_ev[1]);
  if (q == hipErrorNotReady) return SHM_OK;
  HIP_OK(q);
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, t->dir_ev[0], t->dir_ev[1]));
  t->dir_last_ms = ms;
  t->dir_total_ms += ms;
  t->dir_ev_pending = false;
  return SHM_OK;
}


// The look-back kernels' block-index counters (lookback_index): the
// ordering's bin prefix (k_bin_unique: 256 blocks, one per CU; two ranks on
// one GPU spun on each other with blockIdx, kErrBinSpin) and the scans take a
// ticket, which costs nothing measurable there.  k_seg_fill keeps blockIdx:
// its 1024 blocks per C5 chunk serialised on a counter (C5 5.19-5.23 K
// against 5.33-5.38 K Mops/s, round-4 A/B), and it needs none for forward
// progress: a tile that waits too long for an earlier tile counts that
// tile's staged heads itself (seg_tile.h).
uint32_t* lb_ctr(shm_tree* t, int which) {
  return which == dev::kLbSeg ? nullptr : t->ctl->lb_ids[which];
}

// The directory's allocation holds 2^bits entries (+ the level hints);
// never shrunk.  A larger one is allocated before the old one is freed, and
// when it cannot be had the tree keeps the directory it has, at its size
// (ADVICE r5): dir_bits_limit then caps every later build, so the failed
// allocation is not tried again.  No directory at all: progressively smaller
// ones, and at the last the gets walk from the root.
int dir_alloc(shm_tree* t, uint32_t bits, hipStream_t s) {
  if (t->dir && bits <= t->dir_cap_bits) return SHM_OK;
  for (;;) {
    const uint64_t ent = 1ull << bits;
    const uint64_t bytes = ent * (8 * kDirWords) + ent * 8;  // entries + 2 u32 hints
    uint64_t* nd = nullptr;
    uint32_t* nh = nullptr;
    bool ok = !(t->dir_mem_limit && bytes > t->dir_mem_limit);
    if (ok && dalloc(&nd, kDirWords * ent)) ok = false;
    if (ok && dalloc(&nh, 2 * ent)) {
      (void)hipFree(nd);
      ok = false;
    }
    if (ok) {
      if (t->dir) {  // the old directory's last readers are ordered before s
        HIP_OK(hipStreamSynchronize(s));
        HIP_OK(hipFree(t->dir));
        HIP_OK(hipFree(t->dir_hint));
      }
      t->dir = nd;
      t->dir_hint = nh;
      t->dir_cap_bits = bits;
      t->hint_ok = false;
      return SHM_OK;
    }
    (void)hipGetLastError();  // clear the failed allocation's sticky status
    if (t->dir) {
      t->dir_bits_limit = t->dir_cap_bits;
      return SHM_OK;  // keep what we have
    }
    if (bits <= 10) {
      t->dir_off = true;  // no directory: the walks start at the root
      return SHM_OK;
    }
    t->dir_bits_limit = --bits;
  }
}

int refresh_dir(shm_tree* t, hipStream_t s) {
  if (const int rc = dir_poll(t, false)) return rc;
  if (!dir_stale(t)) return SHM_OK;
  static const bool trace = [] {
    const char* e = getenv("SHM_TRACE_DIR");
    return e && e[0] == '1';
  }();
  if (trace)
    fprintf(stderr, "sherman_amd: leaf directory rebuild: pages %llu (last build %llu), %u reads "
            "since the last insert, debt %.1f us\n", (unsigned long long)t->next_page,
            (unsigned long long)t->dir_np, t->reads_since_write, t->dir_debt_ps * 1e-6);
  uint32_t bits = dir_bits_for(t, read_phase(t));
  if (const int rc = dir_alloc(t, bits, s)) return rc;
  if (t->dir_off) {
    t->dir_valid = false;
    return SHM_OK;
  }
  if (bits > t->dir_cap_bits) bits = t->dir_cap_bits;
  if (bits != t->dir_bits) t->hint_ok = false;  // the hints are laid out by entry count
  t->dir_bits = bits;
  // the previous build's time first (its events are reused)
  if (const int rc = dir_poll(t, true)) return rc;
  for (hipEvent_t& e : t->dir_ev)
    if (!e) HIP_OK(hipEventCreate(&e));  // timing events (a rebuild is rare)
  HIP_OK(hipEventRecord(t->dir_ev[0], s));
  // a read phase builds the pair form (layout.h kDirPairs): each prefix's
  // own keys, a get reads fewer false candidates and prefixes that span
  // several leaves are answered from the entry as well
  const bool pairs = want_pairs(t);
  dev::launch_leaf_dir(t->arena, t->arena_bytes, t->cfg.node_id, t->root, t->cfg.key_lo,
                       t->cfg.key_bits - bits, 1ull << bits, t->dir, t->dir_hint,
                       t->hint_ok ? 1 : 0, t->sum, t->d_err, s, pairs ? 1 : 0);
  if (pairs)
    dev::launch_dir_pairs(t->arena, t->next_page, t->cfg.node_id, t->cfg.key_lo,
                          t->cfg.key_bits - bits, 1ull << bits, t->dir, s);
  HIP_OK(hipEventRecord(t->dir_ev[1], s));
  t->dir_ev_pending = true;
  ++t->dir_builds;
  t->dir_pairs = pairs;
  t->dir_np = t->next_page;
  t->dir_valid = true;
  t->hint_ok = true;
  t->dir_debt_ps = 0.0;
  t->dir_lost_at_build = dir_lost(t);
  t->dir_idle_upkeeps = 0;
  t->dir_exact = t->dir_maint;
  return SHM_OK;
}

int readback(shm_tree* t, hipStream_t s, const void* src, size_t bytes, int clear = 0);

// the LDS replica's table (rebuilt like the directory, once the tree grew
// by 1/32); one read-back of its size per rebuild
int refresh_top(shm_tree* t, hipStream_t s) {
  if (!use_top(t) || (t->top_valid && t->next_page <= t->top_np + t->top_np / 32)) return SHM_OK;
  if (!t->top_keys) {
    if (dalloc(&t->top_keys, dev::kTopMax) || dalloc(&t->top_pages, dev::kTopMax) ||
        dalloc(&t->top_scratch, 4ull * dev::kTopMax))
      return SHM_ENOMEM;
  }
  dev::launch_top(t->arena, t->arena_bytes, t->cfg.node_id, t->root, dev::kTopMax, t->top_keys,
                  t->top_pages, t->top_scratch, reinterpret_cast<uint32_t*>(t->d_counts + 14),
                  t->d_err, s);
  HIP_OK(hipGetLastError());
  const int rc = readback(t, s, t->d_counts + 14, sizeof(uint32_t));
  if (rc) return rc;
  t->top_n = (uint32_t)t->h_pin[0];
  t->top_np = t->next_page;
  t->top_valid = t->top_n > 0;
  return SHM_OK;
}

void set_dir(shm_tree* t, const uint64_t** dir, uint64_t* lo, uint32_t* shift, uint64_t* n) {
  if (!use_leaf_dir(t) || !t->dir_valid) return;
  *dir = t->dir;
  *lo = t->cfg.key_lo;
  *shift = t->cfg.key_bits - t->dir_bits;
  *n = 1ull << t->dir_bits;
}

// SHM_DEBUG=1: synchronise after every launch and name the failing step
// (diagnostics only; the launch sequence is the same)
bool debug_sync_enabled() {
  static const int on = [] {
    const char* e = getenv("SHM_DEBUG");
    return e && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0;
  }();
  return on != 0;
}
// SHM_DEBUG=2: also name every step as it completes (a hang's last line)
bool debug_trace_enabled() {
  static const bool on = [] {
    const char* e = getenv("SHM_DEBUG");
    return e && e[0] == '2';
  }();
  return on;
}
int dbg(hipStream_t s, const char* what) {
  if (!debug_sync_enabled()) return SHM_OK;
  hipError_t e = hipStreamSynchronize(s);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) {
    fprintf(stderr, "sherman_amd[debug]: %s failed: %s\n", what, hipGetErrorString(e));
    return SHM_EIO;
  }
  if (debug_trace_enabled()) fprintf(stderr, "sherman_amd[debug]: %s done\n", what);
  return SHM_OK;
}
#define DBG(s, what)                   \
  do {                                 \
    int _r = dbg((s), (what));         \
    if (_r) return _r;                 \
  } while (0)

// Read `bytes` (<= 256) of device words into pinned host scratch and wait.
// A one-wave kernel stores the words straight into the mapped, coherent host
// page, then a sequence number after a system-scope fence; the host spins on
// that word instead of a D2H copy (an SDMA/blit round trip) and a stream
// synchronisation.  While spinning it polls the stream, so a fault in an
// earlier kernel (which would keep the word from ever arriving) still returns
// SHM_EIO.
int readback(shm_tree* t, hipStream_t s, const void* src, size_t bytes, int clear) {
  const uint32_t seq = ++t->rb_seq;
  dev::launch_readback(t->h_pin_dev, static_cast<const uint32_t*>(src),
                       (uint32_t)((bytes + 3) / 4), t->h_pin_dev + kFlagWord, seq, clear, s);
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

// the host's superblock written by a one-wave kernel (create / load_image);
// afterwards k_upper owns next_page, root_level, splits and batches
int write_superblock(shm_tree* t, hipStream_t s) {
  Superblock sb{};
  sb.magic = kSuperMagic;
  sb.root_ptr = t->root;
  sb.root_level = t->root_level;
  sb.next_page = t->next_page;
  sb.capacity_pages = t->cap_pages;
  sb.node_id = t->cfg.node_id;
  sb.batches = t->chunks;
  sb.splits = t->splits;
  dev::launch_write_superblock(t->arena, sb, s);
  HIP_OK(hipGetLastError());
  publish_host(t);
  return SHM_OK;
}

// device error block -> status.  Word 0 holds the bits (kErrKeyMax: a chunk
// with kKeyMax was rejected whole; kErrNoMem: the arena ran out, splits left
// unapplied; kErrHandoff: a chunk's k_upper gave up at a hand-off and its
// last block completed the chunk alone -- word 2 counts those chunks; the
// rest: a tree inconsistency or a kernel bound, SHM_EIO), word 1 the first
// insert chunk that saw a bit (0: none did).  The words are taken by atomic
// exchange (readback clear), so a bit set by another stream after the read
// stays for the next call.  shm_last_error reports what was read.
int check_err(shm_tree* t, hipStream_t s) {
  t->err_pending = false;
  int rc = readback(t, s, t->d_err, 3 * sizeof(uint32_t), 1);
  if (rc) return rc;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(t->h_pin);
  const uint32_t e = w[0], chunk = w[1], resumed = w[2];
  mirror(t);  // the stream is idle up to here: the mirror is exact
  t->last_error.resumed += resumed;
  if (!e) return SHM_OK;
  t->sticky_err |= e;
  const uint32_t other = e & ~(dev::kErrKeyMax | kErrNoMem | kErrHandoff);
  rc = other ? SHM_EIO : (e & kErrNoMem) ? SHM_ENOMEM : (e & dev::kErrKeyMax) ? SHM_EINVAL : SHM_OK;
  t->last_error.bits = e;
  t->last_error.chunk = chunk;
  t->last_error.status = rc;
  if (other) fprintf(stderr, "sherman_amd: device error bits 0x%x (first seen by chunk %u)\n", e, chunk);
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

// start a ProfRec with `ne` events, e[0] recorded now on s
int prof_begin(shm_tree* t, hipStream_t s, int kind, uint64_t n, int ne,
               shm_tree::ProfRec& r) {
  r = shm_tree::ProfRec{{nullptr, nullptr, nullptr, nullptr}, n, kind, -1, 0};
  for (int i = 0; i < ne; ++i) {
    r.e[i] = take_event(t);
    if (!r.e[i]) return SHM_EIO;
  }
  HIP_OK(hipEventRecord(r.e[0], s));
  return SHM_OK;
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
      if (r.clk >= 0) {
        // the walk's own span on the device clock: first block start to last
        // wave end (what a kernel trace reports, without the launch gap the
        // events include)
        std::vector<uint64_t> c(r.blocks * 5);
        HIP_OK(hipMemcpy(c.data(), t->prof_clk + (uint64_t)r.clk * t->clk_words,
                         c.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
        const uint64_t t0 = *std::min_element(c.begin(), c.begin() + r.blocks);
        const uint64_t t1 = *std::max_element(c.begin() + r.blocks, c.end());
        a.walk_kernel_ms += t1 > t0 ? (double)(t1 - t0) / t->clk_khz : 0.0;
        --t->clk_live;
      }
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

// the op buffers of chunk tag's parity (the ordering's outputs)
uint64_t* op_keys(shm_tree* t, uint32_t tag) { return t->uk + (uint64_t)(tag & 1u) * t->nmax; }
uint64_t* op_vals(shm_tree* t, uint32_t tag) { return t->uv + (uint64_t)(tag & 1u) * t->nmax; }
uint64_t* op_dels(shm_tree* t, uint32_t tag) { return t->dk + (uint64_t)(tag & 1u) * t->nmax; }
// {upserts, deletes} of the chunk (k_bin_unique)
uint64_t* op_counts(shm_tree* t, uint32_t tag) { return t->d_counts + 16 * (tag & 1u); }

// One insert chunk (n <= nmax ops), issued without a host wait:
//   1. ordering: k_tile_dedup, coarse partition, k_bin_unique
//      -> uk / uv (upserts, key order, last writer) and dk (deletes); counts
//      stay on the device (d_counts[0..1]);
//   2. k_locate: each upsert's leaf from the leaf directory (summary or
//      header walk); an op whose key its leaf holds is applied right there
//      (lock word, one entry write);
//   3. segmentation (k_seg_count, k_seg_fill_scan): only the runs of ops
//      on a page that gets a new key are listed (the upsert stages them);
//   4. k_leaf_upsert_pipe: lock words with the page DMAs, in-place upserts,
//      splits flagged and counted;
//   5. k_upper: leaf splits, parent levels, root growth, unlocks, the
//      chunk's deletes, superblock.
// step 1: it reads only the batch and writes the insert workspace
int insert_order(shm_tree* t, hipStream_t s, const uint64_t* keys, const uint64_t* vals,
                 uint64_t n, uint32_t tag, bool skip_pad) {
  // the scratch's last user (the previous ordering) and the op buffers'
  // (the apply of tag - 2), when they ran on another stream
  if (const int rc = follow(t->ord, s)) return rc;
  const uint32_t p = tag & 1u;
  // The apply of tag - 2 (another stream) last read these op buffers.  Flow
  // control on the host: its k_upper publishes its tag in the host mirror
  // once it is done with them, and this call waits for that (in a pipeline
  // the host then runs at most about two chunks ahead of the device).  The
  // apply's stream gets no event record (≈ 4.6 µs of idle device between
  // kernels, tools/event_gap.hip), and the device no polling wait (a
  // wait-value kernel: a profiler that serialises kernels deadlocks on it).
  // A wait past kAppWaitMs (5 ms: the apply's stream held up by the caller,
  // or the card shared) falls back to an event at that stream's tail, so a
  // stalled apply costs this call (which holds the tree's mutex) at most
  // that long on the host.
  if (t->app_valid[p] && t->app_m[p].s != s) {
    const volatile uint64_t* ap =
        reinterpret_cast<const volatile uint64_t*>(t->h_pin) + kPubWord / 2 + dev::kPubApplied;
    if (*ap < t->app_tag[p]) {
      const auto t0 = std::chrono::steady_clock::now();
      while (*ap < t->app_tag[p] &&
             std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(kAppWaitMs))
        std::this_thread::yield();
      if (*ap < t->app_tag[p])
        if (const int rc = follow(t->app_m[p], s)) return rc;
    }
  }
  // Tile mode (chunks of <= kMaxTiles tiles, i.e. <= 1 Mi ops): the tiles
  // write their survivors sorted by coarse bin and k_bin_unique gathers its
  // bin's runs from every tile, so there is no coarse scatter pass (round 4:
  // C3 9612 -> 10231, C5 4425 -> 4703 Mops/s); a larger chunk takes the
  // coarse pass.  The tiles' output
  // (kb / ia) stays live through k_bin_unique, so a bin over kUniqCap ops
  // sorts in ka / ib with kc / id as scratch and ic for its ranks.
  const uint64_t tiles = (n + dev::kIsortTile - 1) / dev::kIsortTile;
  const bool tile_mode = tiles <= (uint64_t)dev::kMaxTiles;
  // tile mode: M and Mx bin-major in part_mt / part_mx (part_hist keeps the
  // coarse pass's tile-major layout for the other path and ordered gets)
  dev::launch_tile_dedup(keys, n, t->kb, t->ia, t->gcount, t->d_err, &t->ctl->gate, tag,
                         t->cfg.key_lo, t->cfg.key_bits, tile_mode ? t->part_mt : t->part_hist,
                         t->part_S, tile_mode ? t->part_mx : nullptr, skip_pad ? 1 : 0, s);
  dev::TileRuns tr{t->kb, t->ia, t->part_mt, t->part_mx, tile_mode ? (uint32_t)tiles : 0u};
  if (!tile_mode)
    dev::launch_partition_coarse(t->kb, n, t->gcount, t->ia, t->cfg.key_lo, t->cfg.key_bits,
                                 t->part_hist, t->part_S, t->ka, t->ib, t->bins, s);
  dev::launch_bin_unique(t->ka, t->ib, t->bins, t->cfg.key_lo, t->cfg.key_bits, vals,
                         tile_mode ? t->ic : t->ia,
                         reinterpret_cast<uint64_t*>(t->bins + 2 * dev::kCoarse),
                         tile_mode ? t->kc : t->kb, tile_mode ? t->id : t->ic,
                         op_keys(t, tag), op_vals(t, tag), op_dels(t, tag), op_counts(t, tag),
                         t->d_err, t->part_S, &t->ctl->gate,
                         tag, t->stamps ? t->stamps + dev::kUpperStamps : nullptr, tr,
                         lb_ctr(t, dev::kLbBin), s);
  DBG(s, "ordering");
  note(t->ord, s);
  return SHM_OK;
}

// steps 2-5 on the ordered chunk of tag (the leaf directory is current)
int insert_apply(shm_tree* t, hipStream_t s, uint64_t n, uint32_t tag,
                 shm_tree::ProfRec& pr) {
  const uint64_t lock_tag = (uint64_t)tag << 32;
  const bool searched = t->reads_since_write > 0;
  t->reads_since_write = 0;
  if (t->pub_batch != t->pub_seen) {  // a newer chunk published since the last look
    if (t->next_page == t->np_seen) {
      if (t->quiet_chunks < kQuietChunks) ++t->quiet_chunks;
    } else {
      t->quiet_chunks = 0;
      t->np_seen = t->next_page;
    }
    t->pub_seen = t->pub_batch;
  }
  // the chunk keeps the directory exact (dir_upkeep.h: two launches after
  // its k_upper) only where gets read it between chunks and the chunks
  // still add keys: a write-only stream (C5) or one whose upkeeps found
  // nothing to do kIdleUpkeeps times in a row (C3's updates) runs round 5's
  // rules instead -- its directory stops being exact until the next build --
  // rather than pay the launches for nothing
  {  // the upkeeps finished since the last look: did any find work?
    const volatile uint64_t* p =
        reinterpret_cast<const volatile uint64_t*>(t->h_pin) + kPubWord / 2;
    const uint64_t done = p[dev::kPubDirUpkeeps];  // first: the work word is at least this new
    const uint64_t work = p[dev::kPubDirWork];
    if (done != t->dir_upk_seen) {
      t->dir_idle_upkeeps = work == t->dir_work_seen ? t->dir_idle_upkeeps + (uint32_t)(done - t->dir_upk_seen) : 0;
      t->dir_upk_seen = done;
      t->dir_work_seen = work;
    }
  }
  const bool upkeep = t->dir_maint && t->dir_exact && t->dir_valid &&
                      ((searched && t->dir_idle_upkeeps < kIdleUpkeeps) || t->dir_maint_always);
  if (!upkeep) t->dir_exact = false;
  // the byte marks repeat every 255 chunks: clear them when they wrap, so
  // no page still carries this chunk's mark from 255 chunks ago
  if (dev::new_mark(tag) == 1)
    HIP_OK(hipMemsetAsync(t->pnew, 0, t->cap_pages, s));
  dev::WalkArgs w = walk_args(t);
  uint64_t* const cnt = op_counts(t, tag);
  w.keys = op_keys(t, tag);
  w.n = n;
  w.n_dev = cnt + 0;
  w.out_page = t->pages;
  w.target_level = 0;
  w.out_slot = t->oslot;
  w.out_new = t->pnew;  // the page marks the segmentation reads
  w.out_new_tag = tag;
  w.any_new = reinterpret_cast<uint32_t*>(t->d_counts + 10);
  w.vals = op_vals(t, tag);
  w.locks = t->locks;
  w.num_locks = t->cfg.num_locks;
  w.lock_tag = lock_tag;
  set_dir(t, &w.dir, &w.dir_lo, &w.dir_shift, &w.dir_n);
  w.dir_pairs = w.dir && t->dir_pairs ? 1 : 0;
  w.dir_exact = w.dir && t->dir_exact ? 1 : 0;
  dev::launch_locate(w, n, s);
  DBG(s, "locate");
  uint32_t* d_ns = reinterpret_cast<uint32_t*>(t->d_counts + 8);
  dev::UpperArgs u{};
  u.arena = t->arena;
  u.arena_bytes = t->arena_bytes;
  u.node = t->cfg.node_id;
  u.root = t->root;
  u.leaf_hw = t->leaf_hw;
  u.sum = t->sum;
  u.locks = t->locks;
  u.num_locks = t->cfg.num_locks;
  u.tag = lock_tag;
  u.batch = tag;
  u.par = tag & 1u;
  u.err = t->d_err;
  u.ctl = t->ctl;
  u.op_key = op_keys(t, tag);
  u.op_val = op_vals(t, tag);
  u.seg_start = t->seg_start;
  u.seg_end = t->seg_end;
  u.seg_page = t->seg_page;
  u.seg_T = t->seg_T;
  u.seg_P = t->seg_P;
  u.seg_np = t->seg_np;
  u.seg_ver = t->seg_ver;
  u.ns_dev = d_ns;
  u.leaf_rd = t->leaf_rd;
  u.sep_cap = t->sep_cap;
  for (int i = 0; i < 2; ++i) {
    u.sep_key[i] = t->sep_key[i];
    u.sep_ptr[i] = t->sep_ptr[i];
    u.ipage[i] = t->ipage[i];
  }
  u.h_end = t->h_end;
  u.h_T = t->h_T;
  u.h_P = t->h_P;
  u.h_ver = t->h_ver;
  u.h_lk = t->h_lk;
  u.d_head = t->d_head;
  u.d_base = t->d_base;
  u.int_rd = t->int_rd;
  u.pub = reinterpret_cast<uint64_t*>(t->h_pin_dev) + kPubWord / 2;
  u.dk = op_dels(t, tag);
  u.n_del = cnt + 1;
  set_dir(t, &u.dir, &u.dir_lo, &u.dir_shift, &u.dir_n);
  if (u.dir) u.dir_hint = t->dir_hint;
  if (u.dir && upkeep) {  // the chunk's directory upkeep after its k_upper (dir_upkeep.h)
    // the first kept chunk after chunks that were not: its parity's list
    // count may still hold the count of the last kept chunk of that parity
    // (each repair zeroes only the other parity's, for the chunk after it)
    if (!t->dir_last_upkept) HIP_OK(hipMemsetAsync(t->dir_fix_n + u.par, 0, sizeof(uint32_t), s));
    u.dir_w = t->dir;
    u.dir_form = t->dir_pairs ? dev::kDirFormPairs : dev::kDirFormFp;
    u.dir_fix = t->dir_fix;
    u.dir_fix_n = t->dir_fix_n;
    u.dir_fix_cap = t->dir_fix_cap;
  }
  u.stamps = t->stamps;
  u.force_abort = (t->force_flags & 1u) ? 1u : 0u;
  u.no_direct = (t->force_flags & 2u) ? 1u : 0u;
  u.prof = t->prof_on ? t->prof_ins : nullptr;
  u.pub_always = t->next_page != t->dir_np ? 1u : 0u;
  // small splits built by the upsert kernel itself; the forced k_upper paths
  // (force flags 1, 2, 4) leave them all to k_upper
  dev::UpperArgs ue = u;
  ue.early = (t->force_flags & 7u) ? 0u : 1u;
  // a chunk with no new key and no delete is completed by the segmentation
  // kernel's block 0 (u: k_upper's quick path; k_upper then returns at once).
  const bool quick_ok = !u.force_abort;
  // force flag bit 3: every tile counts its predecessors itself (the
  // look-back's fallback, exercised by a test)
  dev::launch_segment(t->pages, n, cnt + 0, t->seg_lb, t->seg_start, t->seg_end,
                      t->seg_page, d_ns, t->pnew, tag, w.any_new, t->d_err, s,
                      quick_ok ? &u : nullptr, lb_ctr(t, dev::kLbSeg),
                      (t->force_flags & 8u) ? 0u : kSegSelfAfter, cnt + 1,
                      &t->ctl->ndel[tag & 1u][0]);
  DBG(s, "segment");
  if (t->prof_on) HIP_OK(hipEventRecord(pr.e[1], s));
  dev::SegArgs a{};
  a.arena = t->arena;
  a.arena_bytes = t->arena_bytes;
  a.node = t->cfg.node_id;
  a.op_key = op_keys(t, tag);
  a.op_val = op_vals(t, tag);
  a.seg_start = t->seg_start;
  a.seg_end = t->seg_end;
  a.seg_page = t->seg_page;
  a.num_seg = (uint32_t)n;
  a.num_seg_dev = d_ns;
  a.seg_T = t->seg_T;
  a.seg_P = t->seg_P;
  a.seg_newpages = t->seg_np;
  a.seg_ver = t->seg_ver;
  a.oslot = t->oslot;
  a.placed = u.dir_w ? t->oslot : nullptr;  // new keys' slots for k_dir_upkeep
  a.locks = t->locks;
  a.num_locks = t->cfg.num_locks;
  a.tag = lock_tag;
  a.err = t->d_err;
  a.leaf_hw = t->leaf_hw;
  a.sum = t->sum;
  a.ctl = t->ctl;
  a.par = tag & 1u;
  a.up_nb = dev::upper_blocks();
  dev::launch_leaf_upsert(a, ue, s);
  DBG(s, "leaf_upsert");
  if (t->prof_on) HIP_OK(hipEventRecord(pr.e[2], s));
  t->force_flags = 0;
  dev::launch_upper(u, s);
  DBG(s, "upper");
  t->dir_last_upkept = u.dir_w != nullptr;
  if (u.dir_w) {
    // the chunk's directory upkeep (new keys' pairs / fingerprints, split
    // pages' prefixes), then the entries it listed rebuilt from the tree
    dev::launch_dir_upkeep(u, t->oslot, t->pages, cnt + 0, n, s);
    DBG(s, "dir_upkeep");
    dev::launch_dir_repair(t->arena, t->arena_bytes, t->cfg.node_id, t->root, u.dir_lo,
                           u.dir_shift, u.dir_n, t->dir, t->dir_hint, (int)u.dir_form, t->dir_fix,
                           t->dir_fix_n, u.par, t->dir_fix_cap, u.pub + dev::kPubDirLost,
                           t->d_err, s);
    DBG(s, "dir_repair");
  }
  HIP_OK(hipGetLastError());
  t->err_pending = true;
  if (t->prof_on) {
    HIP_OK(hipEventRecord(pr.e[3], s));
    t->prof_pending.push_back(pr);
  }
  return SHM_OK;
}

// the chunk's ordering (step 1): its tag, profile record started
int insert_begin(shm_tree* t, hipStream_t s, const uint64_t* keys, const uint64_t* vals,
                 uint64_t n, bool skip_pad, uint32_t* tag, shm_tree::ProfRec& pr) {
  *tag = ++t->chunks;
  if (t->prof_on) {
    const int rc = prof_begin(t, s, shm_tree::kProfInsert, n, 4, pr);
    if (rc) return rc;
  }
  return insert_order(t, s, keys, vals, n, *tag, skip_pad);
}

// steps 2-5 once the device state may change (the leaf directory current)
int insert_finish(shm_tree* t, hipStream_t s, uint64_t n, uint32_t tag, shm_tree::ProfRec& pr) {
  if (use_leaf_dir(t)) {
    const int rc = refresh_dir(t, s);
    if (rc) return rc;
  }
  const int rc = insert_apply(t, s, n, tag, pr);
  if (rc != SHM_OK) return rc;
  // k_upper was queued: it publishes the tag once done with the op buffers
  const uint32_t p = tag & 1u;
  t->app_tag[p] = tag;
  t->app_valid[p] = true;
  note(t->app_m[p], s);
  return SHM_OK;
}

int insert_chunk(shm_tree* t, hipStream_t s, const uint64_t* keys, const uint64_t* vals,
                 uint64_t n, bool skip_pad = false) {
  uint32_t tag = 0;
  shm_tree::ProfRec pr{};
  if (const int rc = insert_begin(t, s, keys, vals, n, skip_pad, &tag, pr)) return rc;
  return insert_finish(t, s, n, tag, pr);
}

// every chunk of one insert call, in order.  A chunk holding kKeyMax is
// rejected whole on the device (SHM_EINVAL at the next synchronising call);
// the call's other chunks, before and after it, are applied (the host does
// not wait between chunks).  skip_pad: kKeyMax keys are a routed insert's
// slot padding and are skipped (shm__insert_batch_padded).
int insert_all(shm_tree* t, const uint64_t* keys, const uint64_t* vals, uint64_t n, void* stream,
               bool sync, bool skip_pad = false) {
  if (!t || (n && (!keys || !vals))) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  if (t->n_pend) return SHM_EINVAL;  // chunks ordered by shm_insert_order come first
  hipStream_t s = pick(stream);
  // The first chunk's ordering reads only the batch and writes the insert
  // workspace, so it is queued before this call's cross-stream wait: it
  // waits for the workspace's last users (insert_order) but not for, e.g.,
  // the range scans just issued on another stream, and runs beside them.
  // (An ordered search's workspace aliases the insert workspace: not with
  // SHM_FLAG_SORT_GETS.)
  const bool early = n > 0 && !(t->cfg.flags & SHM_FLAG_SORT_GETS);
  uint32_t tag0 = 0;
  shm_tree::ProfRec pr0{};
  const uint64_t m0 = std::min(t->nmax, n);
  if (early) {
    if (const int rc = insert_begin(t, s, keys, vals, m0, skip_pad, &tag0, pr0)) return rc;
  }
  Order ord(t, s, true);
  if (ord.rc) return ord.rc;
  mirror(t);
  int rc = SHM_OK;
  for (uint64_t off = 0; off < n && rc == SHM_OK; off += t->nmax) {
    const uint64_t m = std::min(t->nmax, n - off);
    rc = off == 0 && early ? insert_finish(t, s, m0, tag0, pr0)
                           : insert_chunk(t, s, keys + off, vals + off, m, skip_pad);
  }
  if (rc == SHM_OK) {
    t->batches += 1;
    if (sync) rc = check_err(t, s);
  }
  return rc;
}

void free_all(shm_tree* t) {
  auto F = [](void* p) {
    if (p) (void)hipFree(p);
  };
  F(t->arena); F(t->locks); F(t->stamps); F(t->d_err); F(t->d_counts); F(t->route_scratch);
  for (auto& r : t->route_ws)
    if (r.second != t->route_scratch) F(r.second);
  F(t->ka); F(t->kb); F(t->ia); F(t->ib); F(t->ic); F(t->kc); F(t->id); F(t->part_mx); F(t->part_mt);
  F(t->uk); F(t->uv); F(t->dk); F(t->pages); F(t->seg_lb); F(t->bsum64);
  F(t->seg_start); F(t->seg_end); F(t->seg_page); F(t->seg_T); F(t->seg_P); F(t->seg_np);
  F(t->seg_ver); F(t->leaf_hw); F(t->sum); F(t->oslot); F(t->pnew);
  F(t->ctl); F(t->leaf_rd); F(t->dir_fix); F(t->dir_fix_n);
  for (int i = 0; i < 2; ++i) { F(t->sep_key[i]); F(t->sep_ptr[i]); F(t->ipage[i]); }
  F(t->h_end); F(t->h_T); F(t->h_P); F(t->h_ver); F(t->h_lk);
  F(t->d_head); F(t->d_base); F(t->int_rd);
  F(t->part_hist); F(t->part_S); F(t->part_chunks); F(t->dir); F(t->dir_hint); F(t->gcount); F(t->bins);
  F(t->top_keys); F(t->top_pages); F(t->top_scratch); F(t->idx_stats); F(t->prof_ins); F(t->prof_clk);
  for (auto& r : t->prof_pending)
    for (hipEvent_t e : r.e)
      if (e) t->event_pool.push_back(e);
  for (hipEvent_t e : t->event_pool) (void)hipEventDestroy(e);
  if (t->rstage) (void)hipFree(t->rstage);
  {
    shm_tree::GetWs& w = t->gws[1];
    F(w.keys1); F(w.keys_out); F(w.pos1); F(w.src); F(w.M); F(w.S); F(w.chunks);
  }
  for (auto& r : t->shared_ev)
    if (r.ev) (void)hipEventDestroy(r.ev);
  if (t->ex.ev) (void)hipEventDestroy(t->ex.ev);
  if (t->ord.ev) (void)hipEventDestroy(t->ord.ev);
  for (auto& m : t->app_m)
    if (m.ev) (void)hipEventDestroy(m.ev);
  for (auto& pd : t->pend)
    if (pd.ev) (void)hipEventDestroy(pd.ev);
  for (auto& m : t->gws_m)
    if (m.ev) (void)hipEventDestroy(m.ev);
  for (hipEvent_t e : t->dir_ev)
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
  a.leaf_hw = t->leaf_hw;
  set_dir(t, &a.dir, &a.dir_lo, &a.dir_shift, &a.dir_n);
  return a;
}

// a fresh tag for launch_scan_u64_total's tile words (16 bits: the words
// are zeroed again when the tag wraps, so no stale word can match)
uint32_t scan_tag(shm_tree* t, hipStream_t s) {
  uint32_t tag = ++t->scan_seq & 0xFFFFu;
  if (tag == 0) {
    (void)hipMemsetAsync(t->bsum64, 0, sizeof(uint64_t) * (dev::seg_tiles(t->nmax) + 1), s);
    tag = ++t->scan_seq & 0xFFFFu;
  }
  return tag;
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
    // headroom: batches of similar size must not each reallocate (a
    // reallocation waits for the stream)
    const uint64_t words = std::max<uint64_t>(n + n / 4, 1u << 14) * kRangeStage;
    if (dalloc(&t->rstage, words)) return SHM_ENOMEM;
    t->rstage_words = words;
  }
  return SHM_OK;
}

// range scans read what the directory points at: refresh it first
int range_prepare(shm_tree* t, hipStream_t s) {
  mirror(t);
  if (use_leaf_dir(t)) return refresh_dir(t, s);
  return SHM_OK;
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
  // the reference's kNumOfLock (Common.h:87-93): 128 KB of lock words stay
  // cached at the memory side, where the atomics run (C5 locate 76 -> 69 us
  // against 4 Mi words; 2^17 measured the same as 2^14)
  c->num_locks = 16384;
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
      cfg->max_batch >= (1ull << 24) || cfg->num_locks == 0 ||
      (cfg->sort_bits != 0 && cfg->sort_bits != kDefaultSortBits) || cfg->key_bits > 64)
    return SHM_EINVAL;
  shm_tree* t = new shm_tree();
  t->cfg = *cfg;
  if (!t->cfg.sort_bits || t->cfg.sort_bits > 64) t->cfg.sort_bits = kDefaultSortBits;
  if (t->cfg.key_bits == 0) t->cfg.key_bits = 64;
  if (t->cfg.key_bits == 64) t->cfg.key_lo = 0;
  t->dir_maint = dir_maint_enabled();
  auto fail = [&](int rc) {
    free_all(t);
    delete t;
    return rc;
  };
  if (hipSetDevice(cfg->device) != hipSuccess) return fail(SHM_EIO);
  // k_upper's grid barriers need one resident 512-thread block per CU
  if (!dev::upper_resident()) {
    fprintf(stderr, "sherman_amd: k_upper blocks do not fit a CU\n");
    return fail(SHM_EIO);
  }
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
  rc |= dalloc(&t->ic, n);
  rc |= dalloc(&t->kc, n);
  rc |= dalloc(&t->id, n);
  rc |= dalloc(&t->uk, 2 * n);  // two parities (op_keys)
  rc |= dalloc(&t->uv, 2 * n);
  rc |= dalloc(&t->dk, 2 * n);
  rc |= dalloc(&t->pages, segcap);
  rc |= dalloc(&t->seg_lb, dev::seg_tiles(segcap) + 1);
  rc |= dalloc(&t->bsum64, dev::seg_tiles(n) + 1);
  rc |= dalloc(&t->seg_start, segcap + 1);
  rc |= dalloc(&t->seg_end, segcap);
  rc |= dalloc(&t->seg_page, segcap);
  rc |= dalloc(&t->seg_T, segcap);
  rc |= dalloc(&t->seg_P, segcap);
  rc |= dalloc(&t->seg_np, segcap);
  rc |= dalloc(&t->seg_ver, segcap);
  rc |= dalloc(&t->leaf_hw, t->cap_pages);
  rc |= dalloc(&t->sum, t->cap_pages * kSumBytes);
  rc |= dalloc(&t->oslot, n);
  rc |= dalloc(&t->pnew, t->cap_pages);
  rc |= dalloc(&t->ctl, 1);
  t->dir_fix_cap = (uint32_t)std::max<uint64_t>(n, 1u << 16);
  rc |= dalloc(&t->dir_fix, t->dir_fix_cap);
  rc |= dalloc(&t->dir_fix_n, 32);
  rc |= dalloc(&t->leaf_rd, segcap);
  for (int i = 0; i < 2; ++i) {
    rc |= dalloc(&t->sep_key[i], t->sep_cap);
    rc |= dalloc(&t->sep_ptr[i], t->sep_cap);
    rc |= dalloc(&t->ipage[i], t->sep_cap);
  }
  rc |= dalloc(&t->h_end, t->sep_cap);
  rc |= dalloc(&t->h_T, t->sep_cap);
  rc |= dalloc(&t->h_P, t->sep_cap);
  rc |= dalloc(&t->h_ver, t->sep_cap);
  rc |= dalloc(&t->h_lk, t->sep_cap);
  rc |= dalloc(&t->d_head, t->sep_cap);
  rc |= dalloc(&t->d_base, t->sep_cap);
  rc |= dalloc(&t->int_rd, t->sep_cap);
  rc |= dalloc(&t->part_hist, dev::kPartHistWords);
  rc |= dalloc(&t->part_S, dev::kPartGroupWords);
  rc |= dalloc(&t->part_mx, dev::kPartHistWords);
  rc |= dalloc(&t->part_mt, dev::kPartHistWords);
  rc |= dalloc(&t->part_chunks, 2 * (uint64_t)dev::partition_chunk_slots(n));
  rc |= dalloc(&t->gcount, n / dev::kIsortTile + 1);
  rc |= dalloc(&t->bins, 4 * dev::kCoarse);  // (start, count) per bin, then the bins' tagged counts
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
  if (hipHostMalloc((void**)&t->h_pin, 4096, hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void**)&t->h_pin_dev, t->h_pin, 0) != hipSuccess)
    return fail(SHM_ENOMEM);
  memset(t->h_pin, 0, 4096);
  hipStream_t s = t->stream;
  if (hipMemsetAsync(t->locks, 0, sizeof(uint64_t) * cfg->num_locks, s) ||
      hipMemsetAsync(t->d_err, 0, 16, s) ||
      hipMemsetAsync(t->seg_lb, 0, sizeof(uint64_t) * (dev::seg_tiles(segcap) + 1), s) ||
      hipMemsetAsync(t->bsum64, 0, sizeof(uint64_t) * (dev::seg_tiles(n) + 1), s) ||
      hipMemsetAsync(t->ctl, 0, sizeof(dev::UpperCtl), s) ||
      hipMemsetAsync(t->dir_fix_n, 0, sizeof(uint32_t) * 32, s) ||
      hipMemsetAsync(t->bins, 0, sizeof(uint32_t) * 4 * dev::kCoarse, s) ||
      hipMemsetAsync(t->leaf_rd, 0, sizeof(uint64_t) * segcap, s) ||
      hipMemsetAsync(t->int_rd, 0, sizeof(uint64_t) * t->sep_cap, s) ||
      hipMemsetAsync(t->part_S, 0, sizeof(uint32_t) * dev::kPartGroupWords, s) ||
      hipMemsetAsync(t->gws[1].S, 0, sizeof(uint32_t) * dev::kPartGroupWords, s) ||
      hipMemsetAsync(t->arena, 0, kPageSize, s) ||
      hipMemsetAsync(t->leaf_hw, kLeafHwFull, t->cap_pages, s) ||
      hipMemsetAsync(t->sum, 0, t->cap_pages * kSumBytes, s) ||
      hipMemsetAsync(t->pnew, 0, t->cap_pages, s))
    return fail(SHM_EIO);
  // Tree::Tree (Tree.cpp:44-60): empty leaf root
  t->next_page = 1;
  const uint64_t root_off = t->next_page * kPageSize;
  dev::launch_empty_leaf(t->arena, root_off, t->sum, s);
  t->next_page += 1;
  t->root = ga_make(cfg->node_id, root_off);
  t->root_level = 0;
  if (write_superblock(t, s)) return fail(SHM_EIO);
  if (hipStreamSynchronize(s) != hipSuccess) return fail(SHM_EIO);
  *out = t;
  return SHM_OK;
}

uint64_t shm_tree_max_batch(const shm_tree* t) { return t ? t->nmax : 0; }

int shm_tree_destroy(shm_tree* t) {
  if (!t) return SHM_EINVAL;
  (void)hipSetDevice(t->cfg.device);
  (void)hipDeviceSynchronize();
  free_all(t);
  delete t;
  return SHM_OK;
}

// The batched get on s under ord (the leaf directory is current).
static int search_impl(shm_tree* t, hipStream_t s, Order& ord, const uint64_t* keys,
                       uint64_t n, uint64_t* vals_out, uint8_t* found_out);

int shm_search_batch(shm_tree* t, const uint64_t* keys, uint64_t n,
                     uint64_t* vals_out, uint8_t* found_out, void* stream) {
  if (!t || (n && (!keys || !vals_out))) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  hipStream_t s = pick(stream);
  mirror(t);
  Order ord(t, s, false);
  if (t->reads_since_write < kReadPhase) ++t->reads_since_write;
  if (use_leaf_dir(t)) {
    dir_note_gets(t, n);
    if (dir_stale(t)) ord.make_exclusive();  // the rebuild rewrites what searches read
    const int rc = ord.rc ? ord.rc : refresh_dir(t, s);
    if (rc) return rc;
  } else if (use_top(t)) {
    if (!(t->top_valid && t->next_page <= t->top_np + t->top_np / 32)) ord.make_exclusive();
    const int rc = ord.rc ? ord.rc : refresh_top(t, s);
    if (rc) return rc;
  }
  return search_impl(t, s, ord, keys, n, vals_out, found_out);
}

static int search_impl(shm_tree* t, hipStream_t s, Order& ord, const uint64_t* keys,
                       uint64_t n, uint64_t* vals_out, uint8_t* found_out) {
  // Unordered batches take the summary walk (k_get_sum: directory entry,
  // summary line, matching entry: ~3 random lines per get).  Ordering the
  // batch by key first (SHM_FLAG_SORT_GETS) feeds the page walk (k_get),
  // which shares a leaf's 1 KB read among the queries that need it; at C2
  // that is 6.3 G gets/s against 15.4 for the summary walk, so the auto mode
  // no longer orders.
  const bool ordered = (t->cfg.flags & SHM_FLAG_SORT_GETS) && n >= kSortMinGets;
  for (uint64_t off = 0; off < n; off += t->nmax) {
    const uint64_t m = std::min(t->nmax, n - off);
    dev::WalkArgs a = walk_args(t);
    a.out_val = vals_out + off;
    a.out_found = found_out ? found_out + off : nullptr;
    a.n = m;
    set_dir(t, &a.dir, &a.dir_lo, &a.dir_shift, &a.dir_n);
    a.dir_exact = a.dir && t->dir_exact ? 1 : 0;
    a.page_check = (t->cfg.flags & SHM_FLAG_PAGE_CHECK) ? 1 : 0;
    if (use_top(t) && t->top_valid) {
      a.top_keys = t->top_keys;
      a.top_pages = t->top_pages;
      a.top_n = t->top_n;
    }
    a.stats = t->prof_stats ? t->idx_stats : nullptr;
    bool gathered = false;
    shm_tree::ProfRec pr{};
    if (t->prof_on) {
      if (t->clk_live >= shm_tree::kClkSlots) {  // every clock slot holds a record
        const int rc = drain_profile(t);
        if (rc) return rc;
      }
      const int rc = prof_begin(t, s, shm_tree::kProfGet, m, 3, pr);
      if (rc) return rc;
    }
    if (ordered && m >= kSortMinGets) {
      // order the batch by its top key bits so queries that share pages are
      // walked by the same wave (one page read per group, not per query)
      // (keys1, pos1, walk order keys_out, src); the walk stores result p at
      // vals1[src[p]] (= keys1, inside p's chunk), unpartition gathers
      const shm_tree::GetWs& w = t->gws[ord.ws >= 0 ? ord.ws : ord.take_ws()];
      if (ord.rc) return ord.rc;
      dev::launch_partition(keys + off, m, t->cfg.key_lo, t->cfg.key_bits, w.M, w.S, w.chunks,
                            w.keys1, w.pos1, w.keys_out, w.src, s);
      a.keys = w.keys_out;
      a.perm = w.src;
      a.out_val = w.keys1;
      a.out_found = nullptr;
      a.xcd_remap = 1;
      gathered = true;
      DBG(s, "sort(get)");
    } else {
      // unordered: every wave sorts its own 64 keys and starts at the leaf
      // directory; results land in input order (no unpartition pass)
      a.keys = keys + off;
      a.perm = nullptr;
      a.xcd_remap = 0;
    }
    // leaf DMA policy: an ordered walk reads each leaf once per batch, so
    // non-temporal loads keep the directory in L2 (C2 +5 %)
    a.nt = gathered ? 1 : 0;
    // the walk's profile events: around the page walk's launch; the summary
    // walk's own dispatch carries them (hipExtLaunchKernel: its start and
    // end, the span a kernel trace reports, with no marker packets between)
    if (t->prof_on && gathered) HIP_OK(hipEventRecord(pr.e[1], s));
    // ordered: the page walk (k_get); unordered: the summary walk (k_get_sum,
    // three lines per get)
    if (t->prof_on && !gathered && t->prof_clk) {
      pr.clk = t->clk_next;
      pr.blocks = dev::get_sum_blocks(m);
      t->clk_next = (t->clk_next + 1) % shm_tree::kClkSlots;
      ++t->clk_live;
      a.clk = t->prof_clk + (uint64_t)pr.clk * t->clk_words;
    }
    if (gathered)
      dev::launch_get(a, m, s);
    else
      dev::launch_get_sum(a, m, s, t->prof_on ? pr.e[1] : nullptr, t->prof_on ? pr.e[2] : nullptr);
    DBG(s, "walk(get)");
    if (t->prof_on) {
      if (gathered) HIP_OK(hipEventRecord(pr.e[2], s));
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

int shm_mixed_batch(shm_tree* t, const uint64_t* get_keys, uint64_t n_get, uint64_t* vals_out,
                    uint8_t* found_out, const uint64_t* ins_keys, const uint64_t* ins_vals,
                    uint64_t n_ins, void* stream) {
  if (!t || (n_get && (!get_keys || !vals_out)) || (n_ins && (!ins_keys || !ins_vals)))
    return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  if (t->n_pend && n_ins) return SHM_EINVAL;  // apply the ordered chunks first
  hipStream_t s = pick(stream);
  mirror(t);
  Order ord(t, s, true);
  if (ord.rc) return ord.rc;
  if (use_leaf_dir(t)) {
    dir_note_gets(t, n_get);
    const int rc = refresh_dir(t, s);
    if (rc) return rc;
  }
  // the gets, then the inserts, on s.  (Running the inserts' ordering on a
  // second stream beside the walk was measured: the walk's blocks hold every
  // CU, the ordering kernels ran in its tail anyway and the join cost
  // ~10 us; C3 4125 vs 4160-4188 Mops/s.)
  int rc = search_impl(t, s, ord, get_keys, n_get, vals_out, found_out);
  for (uint64_t off = 0; off < n_ins && rc == SHM_OK; off += t->nmax)
    rc = insert_chunk(t, s, ins_keys + off, ins_vals + off, std::min(t->nmax, n_ins - off));
  if (rc == SHM_OK && n_ins) t->batches += 1;
  return rc;
}

int shm_insert_batch(shm_tree* t, const uint64_t* keys, const uint64_t* vals,
                     uint64_t n, void* stream) {
  return insert_all(t, keys, vals, n, stream, true);
}

int shm_insert_batch_async(shm_tree* t, const uint64_t* keys, const uint64_t* vals,
                           uint64_t n, void* stream) {
  return insert_all(t, keys, vals, n, stream, false);
}

// Split insert (one chunk): the ordering on one stream, the tree phase
// later on another, so a caller can order chunk i + 1 while chunk i applies.
int shm_insert_order(shm_tree* t, const uint64_t* keys, const uint64_t* vals, uint64_t n,
                     void* stream, uint32_t* ticket) {
  if (!t || !ticket || (n && (!keys || !vals))) return SHM_EINVAL;
  if (n > t->nmax) return SHM_E2BIG;
  std::lock_guard<std::mutex> g(t->mu);
  if (t->n_pend >= 2) return SHM_EAGAIN;  // two op-buffer parities
  hipStream_t s = pick(stream);
  // The ordering reads only the batch and writes the insert workspace, whose
  // users it waits for itself (insert_order: ord_ev, app_ev), so it takes no
  // part in the tree's call ordering: it neither waits for the calls before
  // it nor makes the next tree change wait for it (the apply waits for its
  // own ticket only) -- chunk i + 1 is ordered beside chunk i's tree phase.
  // With SHM_FLAG_SORT_GETS an ordered search shares the ordering scratch:
  // the ordering is then ordered like an exclusive call.
  const bool sorted = (t->cfg.flags & SHM_FLAG_SORT_GETS) != 0;
  std::optional<Order> ord;
  if (sorted) {
    ord.emplace(t, s, true);
    if (ord->rc) return ord->rc;
  }
  shm_tree::Pending& pd = t->pend[t->n_pend];
  pd.pr = shm_tree::ProfRec{};
  if (const int rc = insert_begin(t, s, keys, vals, n, false, &pd.tag, pd.pr)) return rc;
  pd.n = n;
  pd.s = s;
  if (!pd.ev) pd.ev = new_event();
  if (!pd.ev) return SHM_EIO;
  HIP_OK(hipEventRecord(pd.ev, s));
  ++t->n_pend;
  *ticket = pd.tag;
  return SHM_OK;
}

int shm_insert_apply(shm_tree* t, uint32_t ticket, void* stream) {
  if (!t) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  if (!t->n_pend || t->pend[0].tag != ticket) return SHM_EINVAL;  // oldest first
  const shm_tree::Pending pd = t->pend[0];
  hipStream_t s = pick(stream);
  Order ord(t, s, true);
  if (ord.rc) return ord.rc;
  if (pd.s != s) HIP_OK(hipStreamWaitEvent(s, pd.ev, 0));
  // the slot is free once its apply is queued (the buffers' reuse waits on
  // the host for this chunk's kPubApplied tag in the mirror, with an event
  // at the apply stream's tail as the fallback: insert_order)
  std::swap(t->pend[0], t->pend[1]);
  --t->n_pend;
  mirror(t);
  shm_tree::ProfRec pr = pd.pr;
  if (t->prof_on) {
    // the profile times the apply alone (the ordering ran earlier, elsewhere)
    if (!pr.e[0]) {
      if (const int rc = prof_begin(t, s, shm_tree::kProfInsert, pd.n, 4, pr)) return rc;
    } else {
      HIP_OK(hipEventRecord(pr.e[0], s));
    }
  }
  const int rc = insert_finish(t, s, pd.n, pd.tag, pr);
  if (rc == SHM_OK) t->batches += 1;
  return rc;
}

int shm_del_batch(shm_tree* t, const uint64_t* keys, uint64_t n, void* stream) {
  if (!t || (n && !keys)) return SHM_EINVAL;
  if (n == 0) return SHM_OK;
  // deletes are upserts of kValueNull (Tree.cpp:1040-1043)
  uint64_t* zeros = nullptr;
  const uint64_t m = std::min<uint64_t>(n, t->nmax);
  if (hipMalloc((void**)&zeros, m * sizeof(uint64_t)) != hipSuccess) return SHM_ENOMEM;
  hipStream_t s = pick(stream);
  int rc = SHM_OK;
  if (hipMemsetAsync(zeros, 0, m * sizeof(uint64_t), s) != hipSuccess) rc = SHM_EIO;
  for (uint64_t off = 0; off < n && rc == SHM_OK; off += m) {
    rc = shm_insert_batch(t, keys + off, zeros, std::min(m, n - off), stream);
  }
  (void)hipStreamSynchronize(s);
  (void)hipFree(zeros);
  return rc;
}

int shm_range_query(shm_tree* t, const uint64_t* from, const uint64_t* to,
                    uint64_t n, uint64_t* counts_out, const uint64_t* offsets,
                    uint64_t* vals_out, void* stream) {
  if (!t || (n && (!from || !to || !counts_out))) return SHM_EINVAL;
  if (offsets && !vals_out) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  hipStream_t s = pick(stream);
  Order ord(t, s, true);  // range workspace (scan temp, staging)
  if (ord.rc) return ord.rc;
  if (const int rc = range_prepare(t, s)) return rc;
  t->err_pending = true;
  return range_launch(t, s, range_args(t, from, to, n, counts_out, offsets, vals_out));
}

int shm_range_query_batch(shm_tree* t, const uint64_t* from, const uint64_t* to, uint64_t n,
                          uint64_t* counts_out, uint64_t* offsets_out, uint64_t* vals_out,
                          uint64_t vals_cap, uint64_t* total_out, void* stream) {
  if (!t || !total_out || (n && (!from || !to || !counts_out || !offsets_out))) return SHM_EINVAL;
  if (vals_cap && !vals_out) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  hipStream_t s = pick(stream);
  Order ord(t, s, true);  // range workspace (scan temp, staging)
  if (ord.rc) return ord.rc;
  *total_out = 0;
  if (n == 0) return SHM_OK;
  if (const int rc = range_prepare(t, s)) return rc;
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
    dev::launch_scan_u64_total(counts_out + off, offsets_out + off, m, t->bsum64,
                               scan_tag(t, s), t->d_err, t->d_counts + 12, t->d_err,
                               lb_ctr(t, dev::kLbScan), s);
    rc = readback(t, s, t->d_counts + 12, 2 * sizeof(uint64_t));
    if (rc) return rc;
    if (t->h_pin[1]) return check_err(t, s);
    base.push_back(total);
    total += t->h_pin[0];
  }
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
  hipStream_t s = pick(stream);
  Order ord(t, s, true);
  if (ord.rc) return ord.rc;
  if (n == 0) {
    HIP_OK(hipMemsetAsync(total_dev, 0, 2 * sizeof(uint64_t), s));
    return SHM_OK;
  }
  if (const int rc = range_prepare(t, s)) return rc;
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
  dev::launch_scan_u64_total(counts_out, offsets_out, n, t->bsum64, scan_tag(t, s), t->d_err,
                             total_dev, t->d_err, lb_ctr(t, dev::kLbScan), s);
  if (!vals_cap) return SHM_OK;
  a.offsets = offsets_out;
  a.vals = vals_out;
  a.vals_cap = vals_cap;
  return range_launch(t, s, a);
}

// one pass: the count walk with the caller's per-scan buffers as its staging
int shm_range_query_slots(shm_tree* t, const uint64_t* from, const uint64_t* to, uint64_t n,
                          uint64_t slot_cap, uint64_t* counts_out, uint64_t* vals_out,
                          uint64_t* status_dev, void* stream) {
  if (!t || (n && (!from || !to || !counts_out)) || slot_cap >= (1ull << 32))
    return SHM_EINVAL;
  if (slot_cap && n && !vals_out) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  hipStream_t s = pick(stream);
  Order ord(t, s, true);  // the directory refresh
  if (ord.rc) return ord.rc;
  if (n == 0) return SHM_OK;
  if (const int rc = range_prepare(t, s)) return rc;
  dev::RangeArgs a = range_args(t, from, to, n, counts_out, nullptr, nullptr);
  a.stage = slot_cap ? vals_out : nullptr;
  a.stage_cap = (uint32_t)slot_cap;
  a.status = status_dev;
  t->err_pending = true;
  return range_launch(t, s, a);
}

// Library-internal, not part of include/sherman_amd.h (shard.cpp): a routed
// insert's received slots, kKeyMax padding skipped, queued as
// shm_insert_batch_async (n <= max_batch: one chunk)
int shm__insert_batch_padded(shm_tree* t, const uint64_t* keys, const uint64_t* vals, uint64_t n,
                             void* stream) {
  if (t && n > t->nmax) return SHM_E2BIG;
  return insert_all(t, keys, vals, n, stream, false, true);
}

// Library-internal (shard.cpp): exclusive scan of n <= max_batch u64 words
// on `stream`; tot_dev (device, 2 words) = {total, the tree's error word}
int shm__scan_u64(shm_tree* t, const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* tot_dev,
                  void* stream) {
  if (!t || !tot_dev || (n && (!in || !out))) return SHM_EINVAL;
  if (n > t->nmax) return SHM_E2BIG;
  std::lock_guard<std::mutex> g(t->mu);
  hipStream_t s = pick(stream);
  // the tile words and the look-back counter are the tree's: no other scan
  // of the tree (shm_range_query_*) may run beside this one
  Order ord(t, s, true);
  if (ord.rc) return ord.rc;
  if (n == 0) {
    HIP_OK(hipMemsetAsync(tot_dev, 0, 2 * sizeof(uint64_t), s));
    return SHM_OK;
  }
  dev::launch_scan_u64_total(in, out, n, t->bsum64, scan_tag(t, s), t->d_err, tot_dev, t->d_err,
                             lb_ctr(t, dev::kLbScan), s);
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

// Library-internal, not part of include/sherman_amd.h: the tree's sticky
// device error word (shard.cpp's kernels report into it, so the next
// synchronising call on the tree returns their errors)
uint32_t* shm__error_word(shm_tree* t) { return t ? t->d_err : nullptr; }

// Diagnostics, not part of include/sherman_amd.h: flags for the next insert
// chunk's k_upper.  Bit 0: every block gives up at its first phase hand-off
// (as a timed-out wait would; the launch's last block then completes the
// chunk alone); bit 1: the chunk propagates its splits through the level
// lists instead of the direct path; bit 2 (or any bit): the chunk's upsert
// kernel leaves every split to k_upper (no early splits).
int shm__upper_force(shm_tree* t, uint32_t flags) {
  if (!t) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  t->force_flags = flags;
  return SHM_OK;
}
int shm__upper_force_abort(shm_tree* t) { return shm__upper_force(t, 1u); }

// Diagnostics: the pages the last insert chunk's early splits took (its
// upsert kernel's, upsert.hip), after synchronising the tree
int shm__early_pages(shm_tree* t, uint64_t* out) {
  if (!t || !out) return SHM_EINVAL;
  const int rc = shm_synchronize(t);
  if (rc) return rc;
  std::lock_guard<std::mutex> g(t->mu);
  HIP_OK(hipMemcpy(out, &t->ctl->ualloc[t->chunks & 1u][0], sizeof(uint64_t),
                   hipMemcpyDeviceToHost));
  return SHM_OK;
}

// Diagnostics, not part of include/sherman_amd.h: `blocks` blocks that each
// hold a whole CU (all of its LDS) for `ticks` of the 100 MHz wall clock, on
// `stream`: other streams' kernels meanwhile get the remaining CUs only
int shm__hog(uint32_t blocks, uint64_t ticks, void* stream) {
  if (blocks > 4096 || ticks > 1000000000ull) return SHM_EINVAL;  // <= 10 s
  dev::launch_hog(blocks, ticks, pick(stream));
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

// Diagnostics, not part of include/sherman_amd.h: an empty kernel on
// `stream` whose dispatch marks the edge of a profiling window (bench.py
// Region, tools/fold_roofline.py)
int shm__mark(uint32_t tag, void* stream) {
  dev::launch_mark(tag, pick(stream));
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

// Diagnostics, not part of include/sherman_amd.h: enable = 1 turns k_upper's
// phase clock on, 0 off; out (nullable, kUpperStamps words) receives the last
// chunk's stamps (out[0] = count, then 100 MHz wall-clock values).
int shm__upper_stamps(shm_tree* t, int enable, uint64_t* out) {
  if (!t) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  if (enable == 1 && !t->stamps) {
    if (hipMalloc(&t->stamps, sizeof(uint64_t) * dev::kStampWords) != hipSuccess)
      return SHM_ENOMEM;
    HIP_OK(hipMemset(t->stamps, 0, sizeof(uint64_t) * dev::kStampWords));
  }
  if (out && t->stamps) {
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(out, t->stamps, sizeof(uint64_t) * dev::kStampWords,
                     hipMemcpyDeviceToHost));
  }
  if (enable == 0 && t->stamps) {
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipFree(t->stamps));
    t->stamps = nullptr;
  }
  return SHM_OK;
}

int shm_stats(shm_tree* t, shm_stats_t* o) {
  if (!t || !o) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  HIP_OK(hipDeviceSynchronize());
  mirror(t);  // exact: the device is idle
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
  if (!t || !src || !host_out || bytes == 0 || bytes > 1024 || (bytes & 3)) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  const int rc = readback(t, pick(stream), src, bytes);
  if (rc) return rc;
  memcpy(host_out, t->h_pin, bytes);
  return SHM_OK;
}

int shm_last_error(shm_tree* t, shm_error_t* out, int reset) {
  if (!t || !out) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  *out = t->last_error;
  if (reset) {
    const uint32_t resumed = t->last_error.resumed;
    t->last_error = shm_error_t{};
    t->last_error.resumed = resumed;
  }
  return SHM_OK;
}

uint32_t shm_last_chunk(shm_tree* t) {
  if (!t) return 0;
  std::lock_guard<std::mutex> g(t->mu);
  return t->chunks;
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
  HIP_OK(hipDeviceSynchronize());
  mirror(t);
  const uint64_t used = t->next_page * kPageSize;
  if (bytes_used) *bytes_used = used;
  if (root_ptr) *root_ptr = t->root;
  if (!host_buf) return SHM_OK;
  if (cap < used) return SHM_EINVAL;
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
  // leaf summaries from the loaded pages
  HIP_OK(hipMemset(t->sum, 0, t->cap_pages * kSumBytes));
  dev::launch_sum_rebuild(t->arena, pages, t->sum, nullptr);
  HIP_OK(hipDeviceSynchronize());
  t->root = root_ptr;
  t->root_level = reinterpret_cast<const uint8_t*>(host_buf)[ro + kOffLevel];
  t->next_page = pages;
  t->dir_valid = false;  // contents changed: rebuild the leaf directory
  t->hint_ok = false;    // ... from the root
  t->top_valid = false;
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
  t->prof_on = (on & 1) != 0;
  if (t->prof_on && !t->prof_ins) {
    if (dalloc(&t->prof_ins, 4)) return SHM_ENOMEM;
    HIP_OK(hipMemset(t->prof_ins, 0, sizeof(uint64_t) * 4));
  }
  if (t->prof_on && !t->prof_clk) {
    t->clk_words = dev::get_sum_blocks(t->nmax) * 5;
    if (dalloc(&t->prof_clk, t->clk_words * shm_tree::kClkSlots)) return SHM_ENOMEM;
    int khz = 0, dev_id = 0;
    HIP_OK(hipGetDevice(&dev_id));
    HIP_OK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_id));
    t->clk_khz = khz > 0 ? (double)khz : 1e5;  // 100 MHz on gfx950
  }
  const bool st = (on & 2) != 0;
  if (st && !t->idx_stats) {
    if (dalloc(&t->idx_stats, dev::kIdxStats)) return SHM_ENOMEM;
    HIP_OK(hipMemset(t->idx_stats, 0, sizeof(uint64_t) * dev::kIdxStats));
  }
  t->prof_stats = st;
  return SHM_OK;
}

int shm_index_stats(shm_tree* t, shm_index_stats_t* out, int reset) {
  if (!t || !out) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  memset(out, 0, sizeof(*out));
  if (!t->idx_stats) return SHM_OK;
  HIP_OK(hipDeviceSynchronize());
  uint64_t v[dev::kIdxStats];
  HIP_OK(hipMemcpy(v, t->idx_stats, sizeof(v), hipMemcpyDeviceToHost));
  out->gets = v[dev::kIdxGets];
  out->start_internal = v[dev::kIdxStartInternal];
  out->right_moves = v[dev::kIdxRightMoves];
  out->page_hops = v[dev::kIdxPageHops];
  out->entry_reads = v[dev::kIdxEntryReads];
  out->hits = v[dev::kIdxHits];
  out->dir_fp_hits = v[dev::kIdxDirFp];
  if (reset) HIP_OK(hipMemset(t->idx_stats, 0, sizeof(v)));
  return SHM_OK;
}

int shm_dir_stats(shm_tree* t, shm_dir_stats_t* out) {
  if (!t || !out) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  memset(out, 0, sizeof(*out));
  if (const int rc = dir_poll(t, true)) return rc;
  mirror(t);
  out->form = !t->dir_valid ? 0u : t->dir_pairs ? 2u : 1u;
  out->bits = t->dir_valid ? t->dir_bits : 0u;
  out->entries = t->dir_valid ? 1ull << t->dir_bits : 0ull;
  out->bytes = t->dir ? (1ull << t->dir_cap_bits) * (8 * kDirWords + 8) : 0ull;
  out->builds = t->dir_builds;
  out->pages_at_build = t->dir_np;
  out->pages_since_build = t->next_page > t->dir_np ? t->next_page - t->dir_np : 0ull;
  out->last_build_ms = t->dir_last_ms;
  out->total_build_ms = t->dir_total_ms;
  out->maintained = t->dir_maint ? 1u : 0u;
  out->exact = t->dir_valid && t->dir_exact ? 1u : 0u;
  return SHM_OK;
}

// test hook: directory upkeep on / off for this tree (maint < 0: as is; 2:
// on for every chunk, also those with no search before them) and
// a cap on the bytes a directory allocation may take (0: none), as a device
// short of memory would impose
int shm__dir_config(shm_tree* t, int maint, uint64_t mem_limit) {
  if (!t) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  if (maint >= 0) t->dir_maint = maint != 0;
  if (maint >= 0) t->dir_maint_always = maint == 2;
  if (!t->dir_maint) t->dir_exact = false;  // until the next build
  t->dir_mem_limit = mem_limit;
  return SHM_OK;
}

// diagnostics: every entry the walks trust against the tree as it is now
// (k_dir_verify): out[0] checked, out[1..3] bad leaf lists / pair sets /
// fingerprint copies, out[4..7] first bad prefixes + 1
int shm__dir_verify(shm_tree* t, uint64_t* out) {
  if (!t || !out) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  memset(out, 0, 8 * sizeof(uint64_t));
  HIP_OK(hipDeviceSynchronize());
  if (!t->dir_valid) return SHM_OK;
  unsigned long long* d = nullptr;
  if (dalloc(&d, 8)) return SHM_ENOMEM;
  int rc = SHM_OK;
  if (hipMemset(d, 0, 64) != hipSuccess) rc = SHM_EIO;
  if (!rc) {
    dev::launch_dir_verify(t->arena, t->arena_bytes, t->cfg.node_id, t->root, t->cfg.key_lo,
                           t->cfg.key_bits - t->dir_bits, 1ull << t->dir_bits, t->dir, t->dir_hint,
                           d, t->stream);
    if (hipStreamSynchronize(t->stream) != hipSuccess ||
        hipMemcpy(out, d, 64, hipMemcpyDeviceToHost) != hipSuccess)
      rc = SHM_EIO;
  }
  (void)hipFree(d);
  return rc;
}

int shm_profile_read(shm_tree* t, shm_profile_t* out, int reset) {
  if (!t || !out) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  int rc = drain_profile(t);
  if (rc) return rc;
  if (t->prof_ins) {
    HIP_OK(hipDeviceSynchronize());
    uint64_t c[4];
    HIP_OK(hipMemcpy(c, t->prof_ins, sizeof(c), hipMemcpyDeviceToHost));
    t->prof_acc.insert_unique = c[0];
    t->prof_acc.insert_dels = c[1];
    t->prof_acc.insert_staged = c[2];
    if (reset) HIP_OK(hipMemset(t->prof_ins, 0, sizeof(c)));
  }
  *out = t->prof_acc;
  if (reset) t->prof_acc = shm_profile_t{};
  return SHM_OK;
}

namespace {
int route_bucket(shm_tree* t, const uint64_t* keys, uint64_t n, uint32_t num_shards,
                 uint64_t* counts_out, uint64_t* keys_out, uint32_t* perm_out, void* stream,
                 bool reject_keymax);
}

int shm_route_bucket(shm_tree* t, const uint64_t* keys, uint64_t n,
                     uint32_t num_shards, uint64_t* counts_out,
                     uint64_t* keys_out, uint32_t* perm_out, void* stream) {
  return route_bucket(t, keys, n, num_shards, counts_out, keys_out, perm_out, stream, false);
}

// Library-internal (shard.cpp shm_shard_insert): the bucketing of a routed
// insert; a batch holding kKeyMax is rejected whole on the sending rank
// (nothing routed, SHM_EINVAL at the next synchronising call), as a local
// insert rejects its chunk (the receivers skip kKeyMax as slot
// padding, so it must be caught before packing)
int shm__route_bucket_insert(shm_tree* t, const uint64_t* keys, uint64_t n, uint32_t num_shards,
                             uint64_t* counts_out, uint64_t* keys_out, uint32_t* perm_out,
                             void* stream) {
  return route_bucket(t, keys, n, num_shards, counts_out, keys_out, perm_out, stream, true);
}

}  // extern "C"

namespace {
int route_bucket(shm_tree* t, const uint64_t* keys, uint64_t n, uint32_t num_shards,
                 uint64_t* counts_out, uint64_t* keys_out, uint32_t* perm_out, void* stream,
                 bool reject_keymax) {
  if (!t || num_shards == 0 || num_shards > 64 || !counts_out) return SHM_EINVAL;
  if (n && (!keys || !keys_out || !perm_out)) return SHM_EINVAL;
  if (n > t->nmax) return SHM_E2BIG;
  std::lock_guard<std::mutex> g(t->mu);
  hipStream_t s = pick(stream);
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
  // d_err[3]: the kKeyMax flag of a routed insert (zero between calls)
  dev::launch_route_bucket(keys, n, num_shards, counts_out, keys_out, perm_out, scratch,
                           reject_keymax ? t->d_err + 3 : nullptr, t->d_err, s);
  HIP_OK(hipGetLastError());
  return SHM_OK;
}
}  // namespace

extern "C" {

int shm_route_permute(shm_tree* t, const uint64_t* in, const uint32_t* perm,
                      uint64_t n, uint64_t* out, void* stream) {
  if (!t || (n && (!in || !perm || !out))) return SHM_EINVAL;
  dev::launch_permute(in, perm, n, out, pick(stream));
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

int shm_route_unpermute(shm_tree* t, const uint64_t* in, const uint32_t* perm,
                        uint64_t n, uint64_t* out, void* stream) {
  if (!t || (n && (!in || !perm || !out))) return SHM_EINVAL;
  dev::launch_unpermute(in, perm, n, out, nullptr, pick(stream));
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

int shm_route_unpermute_found(shm_tree* t, const uint64_t* in, const uint32_t* perm,
                              uint64_t n, uint64_t* out, uint8_t* found_out, void* stream) {
  if (!t || (n && (!in || !perm || !out || !found_out))) return SHM_EINVAL;
  dev::launch_unpermute(in, perm, n, out, found_out, pick(stream));
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

int shm_lock_bench(shm_tree* t, const uint64_t* keys, uint64_t n, void* stream) {
  if (!t || (n && !keys)) return SHM_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  hipStream_t s = pick(stream);
  Order ord(t, s, true);  // the lock words: no chunk may hold them meanwhile
  if (ord.rc) return ord.rc;
  // the tag of the last chunk issued: every word is free for it once that
  // chunk has retired (stream order)
  dev::launch_lock_bench(keys, n, t->locks, t->cfg.num_locks, (uint64_t)t->chunks << 32, t->d_err,
                         s);
  HIP_OK(hipGetLastError());
  t->err_pending = true;
  return SHM_OK;
}

int shm_gen_keys(shm_tree* t, uint64_t first, uint64_t n, uint64_t keyspace,
                 uint64_t* keys_out, void* stream) {
  if (!t || (n && !keys_out)) return SHM_EINVAL;
  dev::launch_gen_keys(first, n, keyspace, keys_out, pick(stream));
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

int shm_hash_keys(shm_tree* t, const uint64_t* ids, uint64_t n, uint64_t keyspace,
                  uint64_t* keys_out, void* stream) {
  if (!t || (n && (!ids || !keys_out))) return SHM_EINVAL;
  dev::launch_hash_ids(ids, n, keyspace, keys_out, pick(stream));
  HIP_OK(hipGetLastError());
  return SHM_OK;
}

}  // extern "C"
