/*
 * sherman_amd.h — C-ABI of the MI355X-native Sherman B+tree hot path.
 *
 * Plain C: opaque handle, plain pointers and sizes, int status codes. No HIP,
 * torch or C++ types appear in the signatures (streams are passed as void*,
 * i.e. a hipStream_t cast; NULL = the HIP null/default stream).
 *
 * Every batch entry point takes DEVICE pointers (HBM of the tree's GPU). The
 * host C++ facade (sherman_amd/csrc/Tree.hpp) provides the reference's
 * single-op, host-pointer Tree API on top of these.
 *
 * Reference interface each entry point replaces (paths relative to the
 * Sherman source tree, cmemory/Sherman):
 *   shm_tree_create     Tree::Tree(DSM*, uint16_t)        include/Tree.h:45,  src/Tree.cpp:27-61
 *                       + DSM::getInstance / alloc        include/DSM.h:33-40, 198-224
 *   shm_tree_destroy    (process teardown; DSM is a singleton, src/DSM.cpp:23-35)
 *   shm_search_batch    Tree::search(const Key&, Value&)  include/Tree.h:49-50, src/Tree.cpp:405-459
 *   shm_insert_batch    Tree::insert(const Key&, const Value&)
 *   shm_insert_batch_async                                include/Tree.h:47-48, src/Tree.cpp:353-403
 *   shm_mixed_batch     Tree::search + Tree::insert of one mixed op stream
 *                       (test/benchmark.cpp:165-188)
 *   shm_del_batch       Tree::del(const Key&)             include/Tree.h:51,   src/Tree.cpp:542-591
 *   shm_range_query     Tree::range_query(from, to, Value*)
 *                                                         include/Tree.h:53-54, src/Tree.cpp:461-540
 *   shm_stats           Tree::print_and_check_tree / index_cache_statistics
 *                                                         include/Tree.h:56, 62; src/Tree.cpp:151-203
 *   shm_dump_image / shm_load_image
 *                       the MN arena + root pointer (src/DSM.cpp:37-53, src/Tree.cpp:90-114)
 *   shm_route_*         (no reference counterpart: the multi-GPU key routing
 *                        that replaces DSM chunk round-robin, include/DSM.h:198-224)
 *   shm_shard_*         a Tree spread over memory nodes: DSM::alloc's chunk
 *                       round-robin over nodes (include/DSM.h:198-224) and the
 *                       remote page reads of Tree::search / Tree::insert
 *                       (src/Tree.cpp:353-459), here range shards over RCCL
 */
#ifndef SHERMAN_AMD_H
#define SHERMAN_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHM_ABI_VERSION 11

/* status codes (negative errno style) */
#define SHM_OK 0
#define SHM_EINVAL (-22)   /* bad argument, key == UINT64_MAX (kKeyMax) */
#define SHM_ENOMEM (-12)   /* page arena or workspace exhausted */
#define SHM_EIO (-5)       /* HIP failure or tree inconsistency detected */
#define SHM_EAGAIN (-11)   /* optimistic version/lock check failed */
#define SHM_E2BIG (-7)     /* batch larger than cfg.max_batch */
#define SHM_ENOSPC (-28)   /* output buffer too small (size reported) */

/* flags for shm_config.flags */
#define SHM_FLAG_SORT_GETS 0x1u  /* reorder gets by key and walk whole pages
                                    (k_get) instead of the leaf summaries */
#define SHM_FLAG_LEAF_DIR 0x2u   /* start gets / leaf locates at the leaf
                                    directory (default on) */
#define SHM_FLAG_AUTO_SORT_GETS 0x4u /* accepted; since ABI 5 no batch is
                                    reordered unless SHM_FLAG_SORT_GETS: the
                                    leaf-summary walk reads ~3 lines per get
                                    and ordering never pays */
#define SHM_FLAG_PAGE_CHECK 0x10u /* the batched get also checks the page-level
                                    version (front == rear, Tree.h:241-261) of
                                    every page it takes a value from, and
                                    reports a torn page as SHM_EIO; off by
                                    default: gets never overlap writers
                                    (exclusive calls), and it costs two lines
                                    per get */
#define SHM_FLAG_TOP_LDS 0x8u    /* without SHM_FLAG_LEAF_DIR: gets start from
                                    an LDS replica of the top of the tree (the
                                    pages of the deepest upper level that fits
                                    4096 entries) instead of the root */

typedef struct shm_tree shm_tree;

typedef struct shm_config {
  uint32_t struct_size;  /* sizeof(shm_config) */
  int32_t device;        /* HIP device ordinal */
  uint16_t node_id;      /* GlobalAddress.nodeID of this shard (= GPU id) */
  uint16_t reserved0;
  uint32_t flags;        /* SHM_FLAG_* */
  uint64_t arena_bytes;  /* HBM page arena (1 KB pages), at most 4 TB (else SHM_EINVAL) */
  uint64_t max_batch;    /* ops per device chunk of a batch call (< 2^24) */
  uint32_t num_locks;    /* HBM lock table words (reference: 16384) */
  uint32_t sort_bits;    /* top key bits that order gets: 0 or 16 */
  /* key range hint: this shard's keys lie in [key_lo, key_lo + 2^key_bits)
   * (a range shard of a multi-GPU tree; key_bits = 64: the whole key space).
   * It only steers the get ordering and the leaf directory; keys outside it
   * are still stored and found exactly. */
  uint64_t key_lo;
  uint32_t key_bits;     /* 1..64 (0 is read as 64) */
  uint32_t reserved1;
} shm_config;

typedef struct shm_stats_t {
  uint64_t root_ptr;      /* GlobalAddress of the root page */
  uint32_t root_level;    /* level of the root (leaves are level 0) */
  uint32_t height;        /* root_level + 1 */
  uint64_t pages_used;    /* allocated 1 KB pages (excluding superblock) */
  uint64_t pages_capacity;
  uint64_t arena_bytes;
  uint64_t batches;       /* mutating batches applied */
  uint64_t splits;        /* leaf + internal pages created by splits */
  uint32_t last_error;    /* sticky device error bits (0 = none) */
  uint32_t reserved;
} shm_stats_t;

/* lifecycle ------------------------------------------------------------------ */
int shm_config_init(shm_config *cfg);
int shm_tree_create(const shm_config *cfg, shm_tree **out);
int shm_tree_destroy(shm_tree *t);
/* cfg.max_batch of the handle (the largest chunk one batch call processes) */
uint64_t shm_tree_max_batch(const shm_tree *t);
const char *shm_strerror(int status);
int shm_abi_version(void);

/* batched hot path (device pointers) ------------------------------------------ */
/* vals_out[i] = value of keys[i] (0 if absent); found_out[i] = 1/0.
 * found_out may be NULL. Reads only.
 * Streams: searches issued on distinct streams may run concurrently on the
 * device (an ordered batch uses one of two internal workspaces, alternating,
 * so consecutive batches on two streams overlap one's ordering with the
 * other's walk).  Every other call (insert, delete, range, routing, a
 * directory rebuild) is ordered on the device after all calls issued before
 * it on any stream, and before all calls issued after it: results follow
 * the host's call order. */
int shm_search_batch(shm_tree *t, const uint64_t *keys, uint64_t n,
                     uint64_t *vals_out, uint8_t *found_out, void *stream);
/* Upsert keys[i] -> vals[i] in batch order (last writer in the batch wins).
 * vals[i] == 0 (kValueNull) deletes keys[i]. Mutating calls on one handle are
 * serialised internally. Returns once the batch has been applied on `stream`
 * (one host synchronisation, for the status): SHM_EINVAL if the batch held
 * kKeyMax (the max_batch chunk holding it is rejected whole; the call's other
 * chunks, before and after it, are applied), SHM_ENOMEM if the arena ran out
 * (the splits that did not fit are left unapplied), SHM_EIO on a device fault
 * or a tree inconsistency the kernels detected (shm_last_error names the
 * bits and the chunk that first saw them).  A chunk whose split propagation
 * gave up waiting (a hand-off bound) is completed in the same launch by its
 * last block alone, before any later call reads the tree (counted in
 * shm_error_t.resumed; not an error), as the reference always completes a
 * parent insert (src/Tree.cpp:973-988). */
int shm_insert_batch(shm_tree *t, const uint64_t *keys, const uint64_t *vals,
                     uint64_t n, void *stream);
/* The same batch queued on `stream` without any host wait (the reference's
 * Tree::insert returns nothing either, include/Tree.h:47-48): ordering, leaf
 * upserts, splits, parent levels and root growth all run on the device.  The
 * status of the batch is reported by the next synchronising call on the
 * handle (shm_synchronize, shm_insert_batch, shm_del_batch) as above. */
int shm_insert_batch_async(shm_tree *t, const uint64_t *keys, const uint64_t *vals,
                           uint64_t n, void *stream);
/* shm_insert_batch_async of one chunk (n <= max_batch) split in two calls,
 * so a caller can order the next batch while this one applies:
 * shm_insert_order queues the batch's ordering (last writer per key, sorted,
 * upserts / deletes split; it reads only keys / vals and touches no tree
 * state) on `stream` and returns a ticket; shm_insert_apply queues the tree
 * changes of that ticket (locate, leaf upserts, splits, parent levels,
 * deletes) on its own stream, ordered like any insert (after every earlier
 * call on the handle, before every later one).  At most two tickets are
 * outstanding (SHM_EAGAIN), applied oldest first (else SHM_EINVAL); other
 * insert calls are refused (SHM_EINVAL) while a ticket is outstanding.
 * The ordering reuses the buffers of the chunk two tickets back: when that
 * chunk was applied on another stream, shm_insert_order waits on the host
 * until the device has finished with them (flow control: a pipelined caller
 * stays about two chunks ahead of the device; after 2 s it queues a
 * device-side wait instead and returns).
 * Errors are reported as for shm_insert_batch_async.  Tree::insert
 * (src/Tree.cpp:353-403) for a batch, as shm_insert_batch_async. */
int shm_insert_order(shm_tree *t, const uint64_t *keys, const uint64_t *vals, uint64_t n,
                     void *stream, uint32_t *ticket);
int shm_insert_apply(shm_tree *t, uint32_t ticket, void *stream);
/* One mixed batch of gets and inserts (the reference benchmark's op stream,
 * test/benchmark.cpp:165-188, cut into batches): the gets see the tree as it
 * was before the batch's inserts, the inserts apply as shm_insert_batch_async
 * (the batch's status is reported by the next synchronising call).  Device
 * pointers; found_out nullable. */
int shm_mixed_batch(shm_tree *t, const uint64_t *get_keys, uint64_t n_get, uint64_t *vals_out,
                    uint8_t *found_out, const uint64_t *ins_keys, const uint64_t *ins_vals,
                    uint64_t n_ins, void *stream);
/* Tree::del for every key. */
int shm_del_batch(shm_tree *t, const uint64_t *keys, uint64_t n, void *stream);
/* Batched inclusive range scans [from[i], to[i]]: values of valid entries in
 * leaf order then slot order.  counts_out[i] = number of matches; values are
 * written to vals_out[offsets[i] ...] only when offsets != NULL (call once
 * with offsets == NULL to size, then again with an exclusive scan). */
int shm_range_query(shm_tree *t, const uint64_t *from, const uint64_t *to,
                    uint64_t n, uint64_t *counts_out, const uint64_t *offsets,
                    uint64_t *vals_out, void *stream);
/* The same scans sized in one call: counts_out, offsets_out (exclusive scan
 * of the counts, absolute) and *total_out are always produced (one host
 * synchronisation); the values are written to vals_out when total <=
 * vals_cap, else SHM_ENOSPC is returned and the caller fills a larger buffer
 * with shm_range_query(..., offsets_out, vals). */
int shm_range_query_batch(shm_tree *t, const uint64_t *from, const uint64_t *to,
                          uint64_t n, uint64_t *counts_out, uint64_t *offsets_out,
                          uint64_t *vals_out, uint64_t vals_cap, uint64_t *total_out,
                          void *stream);
/* The same scans without a host synchronisation, for one chunk (n <=
 * cfg.max_batch): total_dev (device, 2 words) receives the total and the
 * device error bits when the call completes on `stream`; values at output
 * index >= vals_cap are dropped, so the caller compares total_dev[0] with
 * vals_cap when it reads the result (the reference leaves sizing the buffer
 * to the caller too, Tree.cpp:513, 532).  Lets a caller queue further work
 * (e.g. the batch's inserts) behind the scans without waiting for them. */
int shm_range_query_batch_async(shm_tree *t, const uint64_t *from, const uint64_t *to,
                                uint64_t n, uint64_t *counts_out, uint64_t *offsets_out,
                                uint64_t *vals_out, uint64_t vals_cap, uint64_t *total_dev,
                                void *stream);
/* Tree::range_query(from, to, Value *buffer) for a batch, each scan with a
 * buffer of its own, as the reference's caller passes one per call
 * (src/Tree.cpp:461-540, include/Tree.h:53): scan i's values, in leaf then
 * slot order, go to vals_out[i * slot_cap ...] (at most slot_cap of them) and
 * counts_out[i] = its number of matches (the reference's return value; more
 * than slot_cap means the buffer was too small and holds the first
 * slot_cap).  One pass over the leaves, no host synchronisation, any n.
 * status_dev (device, 2 words, nullable): the call ADDS the number of scans
 * whose count passed slot_cap to status_dev[0] and ORs its device error bits
 * into status_dev[1] when it completes on `stream` (the caller zeroes the
 * pair; several batches may accumulate into one, checked once). */
int shm_range_query_slots(shm_tree *t, const uint64_t *from, const uint64_t *to,
                          uint64_t n, uint64_t slot_cap, uint64_t *counts_out,
                          uint64_t *vals_out, uint64_t *status_dev, void *stream);

/* introspection / images (host pointers) ------------------------------------- */
int shm_stats(shm_tree *t, shm_stats_t *out);
/* Copy the arena (superblock + pages) to host memory. *bytes_used receives
 * the number of bytes that hold pages; *root_ptr the root GlobalAddress. */
int shm_dump_image(shm_tree *t, void *host_buf, uint64_t cap,
                   uint64_t *bytes_used, uint64_t *root_ptr);
/* Replace the tree with a page image laid out by the reference format
 * (pages at GlobalAddress offsets, nodeID == cfg.node_id). */
int shm_load_image(shm_tree *t, const void *host_buf, uint64_t bytes,
                   uint64_t root_ptr);
/* Structural check on device data: fences, ordering, occupancy. */
int shm_check(shm_tree *t, uint64_t *n_leaves, uint64_t *n_internal,
              uint64_t *n_keys);
int shm_synchronize(shm_tree *t);
/* The device error block as the last synchronising call that found bits in
 * it read it (reset = 1 clears this record).  Errors of asynchronous calls
 * surface at the next synchronising call, whichever it is: `chunk` names the
 * insert chunk that first saw them, so a caller that noted shm_last_chunk()
 * after each async insert knows which batch failed (the reference asserts at
 * the failing operation instead, src/Tree.cpp:220-227, 332-337). */
typedef struct shm_error_t {
  uint32_t bits;     /* device error bits (0 = none was read) */
  uint32_t chunk;    /* insert chunk that first saw them (0: none, e.g. a
                        search's walk bound) */
  int32_t status;    /* the status that call returned */
  uint32_t resumed;  /* chunks whose split propagation gave up waiting and
                        was completed by the launch's last block alone
                        (cumulative) */
} shm_error_t;
int shm_last_error(shm_tree *t, shm_error_t *out, int reset);
/* id of the last insert chunk queued on the handle (1, 2, ...; a batch of n
 * ops is ceil(n / max_batch) chunks) */
uint32_t shm_last_chunk(shm_tree *t);
/* Copy `bytes` (a multiple of 4, <= 1024) of device memory at `src` to
 * host_out once the work queued on `stream` before it has produced them,
 * through the library's zero-copy read-back (one-wave kernel into mapped
 * host memory + a spin on a sequence word) instead of a D2H copy and a stream
 * synchronisation.  Used by the shard router for the RCCL split sizes. */
int shm_read_words(shm_tree *t, const void *src, uint64_t bytes, void *host_out,
                   void *stream);

/* per-kernel timing with HIP events recorded on the launch stream around the
 * hot path's phases (get: order = top-bits sort, walk = the page walk kernel;
 * insert: the whole chunk and its in-place leaf upsert kernel; range: each
 * shm_range_query launch).  Enabled handles pay one event record per phase
 * boundary per call. */
typedef struct shm_profile_t {
  uint64_t calls;        /* search_batch calls (chunks) timed */
  uint64_t queries;      /* queries in those calls */
  double order_ms;       /* sum of get-ordering (partition) time */
  double walk_ms;        /* sum of k_get (page walk) kernel time */
  uint64_t insert_calls; /* insert_batch chunks timed */
  uint64_t insert_ops;   /* ops in those chunks (before dedup) */
  double insert_ms;      /* sum of whole-chunk insert time */
  double upsert_ms;      /* sum of k_leaf_upsert kernel time */
  uint64_t range_calls;  /* shm_range_query launches timed (count + fill) */
  uint64_t range_queries;/* scans in those launches */
  double range_ms;       /* sum of k_range kernel time */
  /* the timed insert chunks' work, counted on the device (ABI 9): the
   * per-touched-leaf algorithmic bytes of bench.py's insert roofline */
  uint64_t insert_unique;/* unique upserts after the batch's last-writer fold */
  uint64_t insert_dels;  /* unique deletes */
  uint64_t insert_staged;/* staged segments: leaves read whole (they get a new key) */
  double walk_kernel_ms; /* sum of the summary walk's device-clock spans (first block
                            start to last wave end: the kernel alone, no launch gap) */
} shm_profile_t;
/* on: bit 0 = the event timing above, bit 1 = the index statistics below */
int shm_profile_enable(shm_tree *t, int on);
int shm_profile_read(shm_tree *t, shm_profile_t *out, int reset);

/* Index statistics of the batched get walk (the role of the reference's
 * Tree::index_cache_statistics / clear_statistics, include/Tree.h:62-63:
 * how often the index cache — here the leaf directory or the LDS replica —
 * took a get straight to its leaf), collected while shm_profile_enable bit
 * 1 is on. */
typedef struct shm_index_stats_t {
  uint64_t gets;            /* queries walked */
  uint64_t start_internal;  /* start page without a leaf summary: a directory
                               miss, or a descent (no directory) */
  uint64_t right_moves;     /* B-link right turns (a stale directory entry) */
  uint64_t page_hops;       /* pages walked from their own bytes */
  uint64_t entry_reads;     /* leaf entries read (fingerprint matches) */
  uint64_t hits;            /* queries found */
  uint64_t dir_fp_hits;     /* found from the directory entry alone (no
                               summary line): its copy of the leaf's
                               fingerprints, or its pair form's slots */
} shm_index_stats_t;
int shm_index_stats(shm_tree *t, shm_index_stats_t *out, int reset);

/* The leaf directory the batched get starts from (the role of the
 * reference's IndexCache, include/IndexCache.h:59-259, whose size and hit
 * counts Tree::index_cache_statistics reports, include/Tree.h:62): its form,
 * the device memory it holds and what its rebuilds cost.  Synchronises with
 * the last rebuild's end (not with other work). */
typedef struct shm_dir_stats_t {
  uint32_t form;              /* 0 none, 1 leaf lists + fingerprints, 2 pair form */
  uint32_t bits;              /* log2 of the entries of the current build */
  uint64_t entries;           /* 2^bits entries of 64 B */
  uint64_t bytes;             /* device bytes held: the allocation (never shrunk)
                                 + the level hints */
  uint64_t builds;            /* builds so far */
  uint64_t pages_at_build;    /* tree pages at the last build */
  uint64_t pages_since_build; /* pages splits added since */
  double last_build_ms;       /* device time of the last build (-1: none yet) */
  double total_build_ms;      /* of every build */
  uint32_t maintained;        /* 1: insert chunks may keep the entries current */
  uint32_t exact;             /* 1: every usable entry equals a fresh build's */
} shm_dir_stats_t;
int shm_dir_stats(shm_tree *t, shm_dir_stats_t *out);

/* multi-GPU routing helpers (range shards: shard s owns
 * [s * 2^64 / P, (s+1) * 2^64 / P)) ------------------------------------------ */
/* Bucket n <= max_batch keys by owning shard (1 <= P <= 64): writes
 * per-shard counts[P], the keys grouped by shard into keys_out, and perm[i] =
 * source position of keys_out[i].  Stable: inside a shard, keys keep their
 * input order (routed insert batches keep last-writer-in-batch-order). */
int shm_route_bucket(shm_tree *t, const uint64_t *keys, uint64_t n,
                     uint32_t num_shards, uint64_t *counts_out,
                     uint64_t *keys_out, uint32_t *perm_out, void *stream);
/* out[i] = in[perm[i]] (carry a companion array, e.g. insert values, along
 * with the bucketed keys). */
int shm_route_permute(shm_tree *t, const uint64_t *in, const uint32_t *perm,
                      uint64_t n, uint64_t *out, void *stream);
/* out[perm[i]] = in[i] (reverse of the bucket permutation). */
int shm_route_unpermute(shm_tree *t, const uint64_t *in, const uint32_t *perm,
                        uint64_t n, uint64_t *out, void *stream);
/* the same for routed get replies, with found_out[perm[i]] = in[i] != 0
 * (Tree::search's bool, Tree.cpp:445-448) in the same pass */
int shm_route_unpermute_found(shm_tree *t, const uint64_t *in, const uint32_t *perm,
                              uint64_t n, uint64_t *out, uint8_t *found_out, void *stream);

/* multi-GPU range shards over RCCL ------------------------------------------
 * Rank r of P (P <= 16) owns keys [r * 2^64 / P, (r+1) * 2^64 / P) in its own
 * shm_tree (create it with key_lo / key_bits of that slice).  One process per
 * GPU; every rank makes the same calls in the same order (collectives).
 * Every rank's tree has the same max_batch (checked at create).
 * A routed get: each key into its owner's run of fixed-size slots
 * (n / P + 6 sqrt(n / P) + 256 keys; the runs' tails padded with kKeyMax
 * once per size, later batches leaving earlier keys of the same owner
 * there), grouped ncclSend / ncclRecv of the runs and of the per-peer
 * counts, local shm_search_batch, results back the same way, gathered to
 * input order; no host wait before the key exchange.  Every rank passes the
 * same n: the slots' size derives from it, and ranks that disagree exchange
 * runs of different sizes.  Keys past their run's slot are answered by an
 * exact second round that end() runs after one read-back of the counts: no
 * lookup is dropped.  A routed insert: stable bucketing, each owner's run
 * in a slot of max_batch / P (kKeyMax padding the receiver skips; a batch
 * holding kKeyMax itself routes nothing and is reported as SHM_EINVAL by the
 * next synchronising call), keys / values / counts exchanged, queued as one
 * insert on the owner with no host wait.  Each rank's ops apply in its own
 * batch order; across ranks the slots apply in rank order, and a run's tail
 * past its slot is sent and applied by the next call on the shard (or
 * shm_shard_synchronize) before anything else, after every rank's slots: one
 * valid linearisation of the ranks' concurrent batches.  Device pointers;
 * n <= the local tree's max_batch. */
typedef struct shm_shard shm_shard;
/* rank 0 makes the id (NCCL_UNIQUE_ID_BYTES = 128), the caller broadcasts it */
int shm_nccl_unique_id(void *id_out, uint64_t bytes);
int shm_shard_create(shm_tree *local, const void *nccl_id, uint64_t id_bytes, uint32_t world,
                     uint32_t rank, shm_shard **out);
/* the same over a caller's communicator (an ncclComm_t as void*; not freed) */
int shm_shard_create_with_comm(shm_tree *local, void *nccl_comm, uint32_t world, uint32_t rank,
                               shm_shard **out);
int shm_shard_destroy(shm_shard *s);
/* vals_out / found_out in input order (Tree::search per key) */
int shm_shard_search(shm_shard *s, const uint64_t *keys, uint64_t n, uint64_t *vals_out,
                     uint8_t *found_out, void *stream);
/* the same in two halves for pipelining: begin = bucketing + the keys'
 * exchange, end = local get + the results' exchange + unpack (neither waits
 * for the device).  Two batches may be begun at once (two slots, each with
 * its own communicator); end them in order.  At world 1 begin does nothing
 * and end is the local get over keys[], so keys[] stays unchanged until
 * end's work has run on the stream. */
int shm_shard_search_begin(shm_shard *s, const uint64_t *keys, uint64_t n, void *stream,
                           uint32_t *ticket);
int shm_shard_search_end(shm_shard *s, uint32_t ticket, uint64_t *vals_out, uint8_t *found_out);
int shm_shard_insert(shm_shard *s, const uint64_t *keys, const uint64_t *vals, uint64_t n,
                     void *stream);
/* Tree::range_query over the shards (src/Tree.cpp:461-540, intended
 * semantics): scan i = [from[i], to[i]] inclusive; its pieces go only to the
 * shards it overlaps (row p of a P x n_cap piece matrix to rank p), the
 * owners scan them, counts come back, and ONE host read-back of the
 * per-peer value totals sizes the value exchange.  counts_out[i], offsets_out
 * (exclusive scan) and *total_out are always produced; values in key order
 * across shards go to vals_out when total <= vals_cap, else SHM_ENOSPC
 * (counts and offsets stay valid, and shm_shard_range_values copies the
 * batch's values into a larger buffer without another exchange).  n_cap:
 * the same on every rank, >= n, P * n_cap <= max_batch. */
int shm_shard_range_query(shm_shard *s, const uint64_t *from, const uint64_t *to, uint64_t n,
                          uint64_t n_cap, uint64_t *counts_out, uint64_t *offsets_out,
                          uint64_t *vals_out, uint64_t vals_cap, uint64_t *total_out,
                          void *stream);
/* The same batch with no host synchronisation: the values
 * travel in fixed runs of peer_cap values per peer each way (the same on
 * every rank), padded on the device, so nothing is read back to size the
 * exchange.  counts_out / offsets_out as above; status (2 device words,
 * written on the stream): status[0] = the batch's total values, status[1] =
 * flags -- 1: a run to or from a peer passed peer_cap (values lost), 2: the
 * scan pass's buffer was short, 4: total > vals_cap (values past vals_cap
 * dropped), 8: a device error of the scans.  Nonzero flags: the batch's
 * values are incomplete; repeat it with shm_shard_range_query (before any
 * tree change).  Sizing: peer_cap ~ 1.25 x the values a rank's scans find
 * on one shard, + a few thousand. */
int shm_shard_range_query_async(shm_shard *s, const uint64_t *from, const uint64_t *to,
                                uint64_t n, uint64_t n_cap, uint64_t *counts_out,
                                uint64_t *offsets_out, uint64_t *vals_out, uint64_t vals_cap,
                                uint64_t peer_cap, uint64_t *status, void *stream);
/* the last shm_shard_range_query batch's values (its offsets_out must still
 * be live), local only: valid until the next call on the shard */
int shm_shard_range_values(shm_shard *s, uint64_t *vals_out, uint64_t vals_cap, void *stream);
/* Apply what a routed insert left for the next call (its overflow tails),
 * then shm_synchronize the local tree: the status of every routed batch. */
int shm_shard_synchronize(shm_shard *s);

/* Tree::lock_bench (include/Tree.h:60, src/Tree.cpp:310-321) for a batch:
 * take and release lock[CityHash64(keys[i]) % num_locks] of the HBM lock
 * table (atomicCAS, try_lock_addr / unlock_addr, Tree.cpp:205-264); keys
 * sharing a word take it in turn.  Ordered like an insert; a spin past its
 * bound is reported at the next synchronising call. */
int shm_lock_bench(shm_tree *t, const uint64_t *keys, uint64_t n, void *stream);

/* workload generators on device (test/benchmark.cpp:43-46, zipf.h) ----------- */
/* keys[j] = CityHash64(i) + 1 (mod keyspace if keyspace != 0), i = first + j */
int shm_gen_keys(shm_tree *t, uint64_t first, uint64_t n, uint64_t keyspace,
                 uint64_t *keys_out, void *stream);
/* keys[j] = CityHash64(ids[j]) + 1 (mod keyspace if keyspace != 0): to_key
 * over an id array, e.g. a zipf stream (test/benchmark.cpp:43-46, 172-173) */
int shm_hash_keys(shm_tree *t, const uint64_t *ids, uint64_t n, uint64_t keyspace,
                  uint64_t *keys_out, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SHERMAN_AMD_H */
