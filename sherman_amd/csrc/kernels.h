// kernels.h — launch interface between the host runtime (tree.cpp) and the
// HIP kernels (walk.hip, insert.hip, util.hip).  Host-only types; no torch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.h"

namespace shm {
namespace dev {

struct WalkArgs {
  const uint8_t* arena;
  uint64_t arena_bytes;
  uint16_t node;
  uint64_t root;
  const uint64_t* keys;
  const uint32_t* perm;   // output position of walk query i (nullable)
  const uint64_t* n_dev;  // device count (nullable -> use n)
  uint64_t n;
  uint64_t* out_val;      // GET
  uint8_t* out_found;     // GET (nullable)
  uint64_t* out_page;     // LOCATE
  int target_level;       // LOCATE
  uint32_t* err;
  // GET: per-key-prefix start pages (nullable -> every query starts at root)
  const uint64_t* start;
  uint32_t start_shift;   // prefix = key >> start_shift
  // GET: leaf directory (leafdir.hip; nullable): 8 u64 per entry, entry p
  // covers keys [dir_lo + (p << dir_shift), ... + 2^dir_shift)
  const uint64_t* dir;
  uint64_t dir_lo;
  uint64_t dir_n;
  uint32_t dir_shift;
  // GET: map blocks to chunks XCD-contiguously (see get.hip)
  int xcd_remap;
  // GET: page DMAs with the non-temporal policy (nt; streamed once per batch)
  int nt;
  // diagnostics (nullable): per wave {start, end} s_memrealtime stamps
  uint64_t* stamps;
  // GET: per-page occupancy bound (nullable -> whole pages are read).  For a
  // leaf, every slot >= leaf_hw[page] is empty (value 0), so its page DMA
  // stops after that slot; kLeafHwFull (internal pages, pages of a loaded
  // image) reads the whole page
  const uint8_t* leaf_hw;
};

void launch_walk(const WalkArgs& a, uint64_t n_upper, int depth, bool locate,
                 hipStream_t s);
// batched get walk with grouped page resolution (get.hip)
void launch_get(const WalkArgs& a, uint64_t n, hipStream_t s);
// the same walk as a leaf locate (insert path): out_page[i] = leaf of keys[i]
void launch_locate_leaf(const WalkArgs& a, uint64_t n, hipStream_t s);
// header-only descent, lane = op (locate.hip): out_page[i] = the page of
// a.target_level holding keys[i]; starts at the leaf directory for level 0
void launch_locate(const WalkArgs& a, uint64_t n_upper, hipStream_t s);
// start[p] = the deepest page whose fences cover every key with prefix p
// (key >> (64 - bits) == p), found by walking from root.  A page's lowest
// fence never changes (a split keeps the left half in place), so a start page
// stays a valid B-link entry point for its prefix after later splits: keys
// past its highest fence move right (Tree.cpp:626-629).
void launch_start_table(const uint8_t* arena, uint64_t arena_bytes, uint16_t node,
                        uint64_t root, uint32_t bits, uint64_t* table, uint32_t* err,
                        hipStream_t s);
// leaf directory (leafdir.hip): n_ent entries of 8 u64 from dir_lo, 2^shift
// keys each
void launch_leaf_dir(const uint8_t* arena, uint64_t arena_bytes, uint16_t node, uint64_t root,
                     uint64_t dir_lo, uint32_t shift, uint64_t n_ent, uint64_t* dir,
                     uint32_t* err, hipStream_t s);

// ---- insert pipeline -------------------------------------------------------
struct SegArgs {
  uint8_t* arena;
  uint64_t arena_bytes;
  uint16_t node;
  // sorted unique operation keys / values of this level (values: leaf values
  // or child GlobalAddresses for internal levels)
  const uint64_t* op_key;
  const uint64_t* op_val;
  uint64_t n_ops;
  // segments (runs of ops targeting one page)
  const uint32_t* seg_start;  // [num_seg + 1]
  const uint64_t* seg_page;   // [num_seg]
  uint32_t num_seg;           // (an upper bound when num_seg_dev is set)
  const uint32_t* num_seg_dev;  // device-side segment count (nullable)
  uint32_t* seg_T;            // entries after applying
  uint32_t* seg_P;            // pages after applying (1 = in place)
  uint32_t* seg_newpages;     // P - 1
  uint32_t* seg_ver;          // front_version observed by plan
  const uint32_t* seg_pbase;  // exclusive scan of seg_newpages
  uint64_t first_new_page;    // arena page index of the first new page
  uint64_t* sep_key;          // separators for the parent level
  uint64_t* sep_ptr;
  uint64_t* locks;
  uint32_t num_locks;
  uint64_t tag_base;
  // per segment: 1 = its page's lock word was taken ahead by k_seg_fill
  // (nullable: k_leaf_upsert takes the words itself)
  const uint32_t* seg_lk;
  int level;
  int is_delete;
  int split_only;             // k_leaf_update: skip segments with P == 1
  uint32_t* err;
  // per-page occupancy bound kept by every leaf writer (see WalkArgs)
  uint8_t* leaf_hw;
};

void launch_leaf_plan(const SegArgs& a, hipStream_t s);
void launch_leaf_build(const SegArgs& a, uint32_t total_new, hipStream_t s);
void launch_leaf_update(const SegArgs& a, hipStream_t s);
// in-place upserts, 4 segments per wave (upsert.hip); flags P > 1 segments
void launch_leaf_upsert(const SegArgs& a, hipStream_t s);
void launch_leaf_delete(const SegArgs& a, hipStream_t s);
void launch_int_plan(const SegArgs& a, hipStream_t s);
void launch_int_build(const SegArgs& a, uint32_t total_new, hipStream_t s);
void launch_int_update(const SegArgs& a, hipStream_t s);
void launch_new_root(uint8_t* arena, uint64_t page_off, uint64_t old_root,
                     uint32_t level, hipStream_t s);
void launch_empty_leaf(uint8_t* arena, uint64_t page_off, hipStream_t s);
void launch_write_superblock(uint8_t* arena, const Superblock& sb, hipStream_t s);

// ---- utilities (util.hip) -----------------------------------------------------
void launch_iota(uint32_t* idx, uint64_t n, hipStream_t s);
// order a get batch by its top 16 key bits (partition.hip): keys_out is the
// walk order, src[p] = keys1 slot of walk slot p, pos1[i] = keys1 slot of
// input i.  M = [kMaxTiles][kCoarse] tile counts, S = group sums (all zero
// between calls; zero it once at creation), chunks = 2 x
// partition_chunk_slots(n) words.
constexpr int kCoarse = 256;
constexpr int kFine = 256;
constexpr int kMaxTiles = 256;
constexpr int kFineCap = 8192;
constexpr int kPartHistWords = kMaxTiles * kCoarse;
constexpr int kPartGroupWords = 16 * kCoarse;
uint32_t partition_chunk_slots(uint64_t n);
// get ordering by the top 16 bits of the key's offset in the shard's range
// [key_lo, key_lo + 2^key_bits) (keys outside clamp to the first/last bucket)
void launch_partition(const uint64_t* keys, uint64_t n, uint64_t key_lo, uint32_t key_bits,
                      uint32_t* M, uint32_t* S, uint32_t* chunks, uint64_t* keys1,
                      uint32_t* pos1, uint64_t* keys_out, uint32_t* src, bool direct, hipStream_t s);
// insert ordering, step 2: the coarse pass alone over per-group
// de-duplicated runs (group gi = keys [gi * 4096, ...) holds gcount[gi]
// keys), carrying a u32 payload; bins = 2 x 256 words of (start, count)
void launch_partition_coarse(const uint64_t* keys, uint64_t n, const uint32_t* gcount,
                             const uint32_t* pay_in, uint64_t key_lo, uint32_t key_bits,
                             uint32_t* M, uint32_t* S, uint64_t* keys1, uint32_t* pay1,
                             uint32_t* bins, hipStream_t s);
// insert ordering (isort.hip).  Step 1: every 4096-op tile reduced to its
// last writer per key (LDS hash table, atomic max of the op index).  Step 3:
// every coarse bin (<= 8192 keys) fully sorted by (key, op index) in place;
// a larger bin sets kErrSortOverflow (the host then re-sorts with rocPRIM).
constexpr int kIsortTile = 4096;
constexpr uint32_t kErrSortOverflow = 1u << 30;
constexpr uint32_t kErrKeyMax = 1u << 31;
void launch_tile_dedup(const uint64_t* keys, uint64_t n, uint64_t* keys_out, uint32_t* idx_out,
                       uint32_t* gcount, uint32_t* err, hipStream_t s);
void launch_bin_sort(uint64_t* keys1, uint32_t* pay1, const uint32_t* bins, uint32_t* S,
                     uint32_t* err, hipStream_t s);
// steps 3-4 in two launches: per-bin last-writer dedup + sort (<= 6144 ops
// per bin, else kErrSortOverflow), then uk / uv / dk at the bins' prefixes
// and (upserts, deletes, error word) in counts[0..2]; bcnt = 2 x 256 words, lrank = one
// u32 per op
void launch_bin_unique(uint64_t* keys1, uint32_t* pay1, const uint32_t* bins, uint64_t key_lo,
                       uint32_t key_bits, const uint64_t* vals, uint32_t* lrank, uint32_t* bcnt,
                       uint64_t* uk, uint64_t* uv, uint64_t* dk, uint64_t* counts, uint32_t* S,
                       uint32_t* err, hipStream_t s);
// out[i] = vals1[pos1[i]], found[i] = out[i] != 0
void launch_unpartition(const uint64_t* vals1, const uint32_t* pos1, uint64_t n,
                        uint64_t* out, uint8_t* found, hipStream_t s);
// out[i] = (uint32_t)(keys[i] >> 32), idx[i] = i
void launch_top32(const uint64_t* keys, uint64_t n, uint32_t* out,
                  uint32_t* idx, hipStream_t s);
// flags[i] = (last of equal-key run) * (v != 0 ? 1 : 1 << 32), key checks
void launch_mark_unique(const uint64_t* sk, const uint32_t* sidx,
                        const uint64_t* vals, uint64_t n, const uint32_t* bins,
                        uint64_t* flags, uint32_t* err, hipStream_t s);
void launch_compact_unique(const uint64_t* sk, const uint32_t* sidx,
                           const uint64_t* vals, const uint64_t* flags,
                           const uint64_t* pos, uint64_t n, uint64_t* uk,
                           uint64_t* uv, uint64_t* dk, uint64_t* counts,
                           hipStream_t s);
// segments of a located op list (n_dev: device-side op count <= n, nullable)
void launch_seg_heads(const uint64_t* page, uint64_t n, const uint64_t* n_dev, uint32_t* heads,
                      hipStream_t s);
void launch_seg_fill(const uint64_t* page, const uint32_t* heads,
                     const uint32_t* pos, uint64_t n, const uint64_t* n_dev, uint32_t* seg_start,
                     uint64_t* seg_page, uint32_t* num_seg, hipStream_t s);
// the same, also taking each segment's lock word (lane per segment,
// atomicCAS(0 -> tag) on lock[CityHash64(page) % num_locks], bounded spin):
// seg_lk[s] = 1 when held.  launch_seg_unlock releases them.
struct SegLock {
  uint64_t* locks;
  uint32_t num_locks;
  uint64_t tag;
  uint32_t* seg_lk;
  uint32_t* err;
};
void launch_seg_fill_lock(const uint64_t* page, const uint32_t* heads, const uint32_t* pos,
                          uint64_t n, const uint64_t* n_dev, uint32_t* seg_start,
                          uint64_t* seg_page, uint32_t* num_seg, const SegLock& lk,
                          hipStream_t s);
void launch_seg_unlock(const uint64_t* seg_page, const uint32_t* num_seg_dev, uint64_t n_max,
                       const SegLock& lk, hipStream_t s);
// Segmentation in two launches instead of heads + library scan + fill: per
// 1024-op tile a head count (bsum), then each tile sums the counts before it
// and fills its segments (lock words as launch_seg_fill_lock when lk.locks).
// bsum holds seg_tiles(n) words.
constexpr uint32_t kSegTile = 1024;
inline uint64_t seg_tiles(uint64_t n) { return (n + kSegTile - 1) / kSegTile; }
void launch_segment(const uint64_t* page, uint64_t n, const uint64_t* n_dev, uint32_t* bsum,
                    uint32_t* seg_start, uint64_t* seg_page, uint32_t* num_seg,
                    const SegLock& lk, hipStream_t s);
// out = exclusive scan of in[0, n) in the same two-launch form
void launch_scan_u32(const uint32_t* in, uint32_t* out, uint64_t n, uint32_t* bsum,
                     hipStream_t s);
// the same over u64 (bsum: seg_tiles(n) words); tot = {total, *err} for the
// range scan's one read-back
void launch_scan_u64_total(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* bsum,
                           const uint32_t* err, uint64_t* tot, hipStream_t s);
void launch_gen_keys(uint64_t first, uint64_t n, uint64_t keyspace,
                     uint64_t* out, hipStream_t s);
void launch_hash_ids(const uint64_t* ids, uint64_t n, uint64_t keyspace, uint64_t* out,
                     hipStream_t s);
// stable bucketing by owning shard; cm = route_scratch_words(n) words
uint64_t route_scratch_words(uint64_t n_max);
void launch_route_bucket(const uint64_t* keys, uint64_t n, uint32_t shards,
                         uint64_t* counts, uint64_t* keys_out, uint32_t* perm,
                         uint32_t* cm, hipStream_t s);
// out[i] = in[perm[i]]
void launch_permute(const uint64_t* in, const uint32_t* perm, uint64_t n, uint64_t* out,
                    hipStream_t s);
void launch_unpermute(const uint64_t* in, const uint32_t* perm, uint64_t n,
                      uint64_t* out, uint8_t* found, hipStream_t s);
// batched range scans (range.hip)
struct RangeArgs {
  const uint8_t* arena;
  uint64_t arena_bytes;
  uint16_t node;
  uint64_t root;
  const uint64_t* from;
  const uint64_t* to;
  uint64_t n;
  uint64_t* counts;
  const uint64_t* offsets;  // nullptr -> count only
  uint64_t* vals;
  uint32_t* err;
  // leaf directory (nullable), as in WalkArgs
  const uint64_t* dir;
  uint64_t dir_lo;
  uint64_t dir_n;
  uint32_t dir_shift;
  // staging (nullable): the count pass also keeps up to stage_cap values of
  // scan q at stage[q * stage_cap]; the fill pass copies those scans from
  // there instead of walking their leaves again
  uint64_t* stage;
  uint32_t stage_cap;
  // fill pass: values at output index >= vals_cap are dropped (the async
  // batch call writes before the host knows the total; it reports the total)
  uint64_t vals_cap;
};
void launch_range(const RangeArgs& a, hipStream_t s);
// out[0] = offsets[n-1] + counts[n-1], out[1] = *err  (n >= 1)
void launch_range_total(const uint64_t* offsets, const uint64_t* counts, uint64_t n,
                        const uint32_t* err, uint64_t* out, hipStream_t s);
// dst[i] = *s_i (one launch instead of four device-to-device copies)
void launch_gather4_u32(uint32_t* dst, const uint32_t* s0, const uint32_t* s1,
                        const uint32_t* s2, const uint32_t* s3, hipStream_t s);
struct Gather8 {
  const uint32_t* p[8];
  int n;
};
// dst[i] = *g.p[i], i < g.n
void launch_gather_u32(uint32_t* dst, const Gather8& g, hipStream_t s);
// dst[i] = src[i] for i < nw (<= 64, dst in mapped host memory), then a
// system-scope release store of seq to *flag
void launch_readback(uint32_t* dst, const uint32_t* src, uint32_t nw, uint32_t* flag,
                     uint32_t seq, hipStream_t s);
void launch_readback_gather(uint32_t* dst, const Gather8& g, uint32_t* flag, uint32_t seq,
                            hipStream_t s);
// x[i] += c for i < n
void launch_add_u64(uint64_t* x, uint64_t n, uint64_t c, hipStream_t s);

}  // namespace dev
}  // namespace shm
