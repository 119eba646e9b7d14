/*
 * sherman_oracle.h — CPU ORACLE (test infrastructure only; never shipped, never
 * on the product path).
 *
 * A from-scratch plain-C restatement of the reference Sherman B+tree hot path
 * (Tree::search / Tree::insert / Tree::del and the *intended* range_query),
 * operating on an in-process page arena that uses the reference's exact 1 KB
 * page byte layout (include/Tree.h:130-336, include/Common.h:112-121) and the
 * GlobalAddress encoding (include/GlobalAddress.h:7-26).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline.
 *
 * Parity pinning: the reference cannot be built in this image (it needs
 * ibverbs/MLNX_OFED, boost_coroutine, libcityhash and libmemcached; stubbing
 * those is not allowed), so this oracle is pinned by the reference's own
 * known-answer test, test/tree_test.cpp:31-68, replayed verbatim in
 * tests/test_oracle.py, plus structural invariants. CityHash64 (third-party,
 * google/cityhash HEAD = v1.1.x, script/installLibs.sh:16-20) is restated from
 * the published algorithm; no reference test pins its outputs, so key streams
 * derived from it are "parity unpinned at the hash" (see DESIGN.md).
 */
#ifndef SHERMAN_ORACLE_H
#define SHERMAN_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_tree orc_tree;

/* tree lifecycle ---------------------------------------------------------- */
/* Tree::Tree (src/Tree.cpp:27-61): empty leaf root, set_consistent. */
orc_tree *orc_tree_create(uint64_t arena_bytes);
void orc_tree_destroy(orc_tree *t);

/* Wrap an externally produced tree image (e.g. a GPU arena copied to host).
 * `image` must stay alive and hold `capacity_bytes` (>= image_bytes): the
 * pages past image_bytes are allocated by later splits; offsets in
 * GlobalAddresses index into it; the node id bits (low 16) of every pointer
 * must equal `node_id`. */
orc_tree *orc_tree_wrap_image(uint8_t *image, uint64_t image_bytes,
                              uint64_t capacity_bytes, uint64_t root_ptr,
                              uint16_t node_id);

/* operations (single op, reference semantics) ------------------------------ */
/* Tree::search  src/Tree.cpp:405-459 */
int orc_search(orc_tree *t, uint64_t k, uint64_t *v);
/* Tree::insert  src/Tree.cpp:353-403 (+ leaf/internal store, new root) */
int orc_insert(orc_tree *t, uint64_t k, uint64_t v);
/* Tree::del     src/Tree.cpp:542-591, 993-1057 */
void orc_del(orc_tree *t, uint64_t k);
/* intended range_query semantics (src/Tree.cpp:461-540 with a working
 * index cache): values of valid entries with from <= key <= to in leaf
 * order then slot order. Returns the count (may exceed cap; only cap
 * values are written). */
uint64_t orc_range_query(orc_tree *t, uint64_t from, uint64_t to,
                         uint64_t *out, uint64_t cap);
uint64_t orc_range_query_batch(orc_tree *t, const uint64_t *from, const uint64_t *to,
                               uint64_t n, uint64_t *counts, uint64_t *out,
                               uint64_t cap);

/* batched helpers ----------------------------------------------------------- */
void orc_search_batch(orc_tree *t, const uint64_t *keys, uint64_t n,
                      uint64_t *vals, uint8_t *found);
/* multi-threaded read-only search (pthreads); returns wall seconds */
double orc_search_batch_mt(orc_tree *t, const uint64_t *keys, uint64_t n,
                           uint64_t *vals, uint8_t *found, int nthreads);
/* sequential insert of a batch in batch order (last writer wins);
 * value 0 means delete (kValueNull, Common.h:117). */
/* the same contents on `nthreads` threads partitioned by page lock word;
 * returns seconds */
double orc_apply_batch_mt(orc_tree *t, const uint64_t *keys, const uint64_t *vals, uint64_t n,
                          int nthreads);
uint64_t orc_range_query_batch_mt(orc_tree *t, const uint64_t *from, const uint64_t *to,
                                  uint64_t n, uint64_t *counts, uint64_t *out, uint64_t cap,
                                  int nthreads, double *secs);
/* the reference benchmark's read phase (test/benchmark.cpp:165-188, 302-341) */
void orc_c1_build(orc_tree *t, uint64_t keyspace, double warm_ratio, uint64_t preload);
void orc_c1_bench(orc_tree *t, int nthreads, uint64_t keyspace, double theta,
                  uint64_t seed_base, int windows, double window_s, double *win_mops);
void orc_apply_batch(orc_tree *t, const uint64_t *keys, const uint64_t *vals,
                     uint64_t n);

/* introspection ------------------------------------------------------------- */
uint64_t orc_root_ptr(const orc_tree *t);
int orc_root_level(const orc_tree *t);
uint64_t orc_pages_used(const orc_tree *t);
const uint8_t *orc_arena(const orc_tree *t);
uint64_t orc_arena_bytes_used(const orc_tree *t);
/* walk every leaf (left to right through sibling links) and emit all valid
 * (key,value) pairs; returns count (writes at most cap). */
uint64_t orc_dump_pairs(orc_tree *t, uint64_t *keys, uint64_t *vals,
                        uint64_t cap);
/* structural check: fences, sortedness of internal pages, occupancy bounds,
 * sibling chain; returns 0 if ok, else a negative code. counts out. */
int orc_check(orc_tree *t, uint64_t *n_leaves, uint64_t *n_internal,
              uint64_t *n_keys, int *height);
/* counters mirroring DSM.cpp:17-21 (page reads during searches) */
uint64_t orc_read_pages(const orc_tree *t);

/* workload generators -------------------------------------------------------- */
/* CityHash64 v1.1 (google/cityhash), lengths 0..16 only. */
uint64_t orc_cityhash64(const void *s, size_t len);
/* benchmark.cpp:43-46 to_key (keyspace 0 => no modulus) */
uint64_t orc_to_key(uint64_t i, uint64_t keyspace);
/* mehcached zipf, test/zipf.h:57-203 */
typedef struct orc_zipf {
  uint64_t n;
  double theta, alpha, thres;
  uint64_t last_n;
  double dbl_n, zetan, eta;
  uint64_t rand_state;
} orc_zipf;
void orc_zipf_init(orc_zipf *z, uint64_t n, double theta, uint64_t seed);
uint64_t orc_zipf_next(orc_zipf *z);
/* fill `out` with n zipf draws */
void orc_zipf_fill(uint64_t n_items, double theta, uint64_t seed, uint64_t *out,
                   uint64_t count);
/* glibc rand_r op stream: is_get[i] = rand_r(&seed) % 100 < read_ratio */
void orc_op_mix(unsigned int seed, int read_ratio, uint8_t *is_get,
                uint64_t count);

#ifdef __cplusplus
}
#endif
#endif
