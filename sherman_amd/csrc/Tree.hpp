// Tree.hpp — host C++ facade with the reference's Tree API
// (include/Tree.h:42-63) over the C-ABI (include/sherman_amd.h).
//
//   Reference                                   Here
//   Tree(DSM*, uint16_t tree_id)                Tree(const shm_config&, uint16_t tree_id = 0)
//   void insert(const Key&, const Value&, ...)  insert(k, v[, cxt, coro_id])
//   bool search(const Key&, Value&, ...)        search(k, v[, cxt, coro_id])
//   void del(const Key&, ...)                   del(k[, cxt, coro_id])
//   uint64_t range_query(from, to, Value* buf)  range_query(from, to, buf[, cxt, coro_id])
//   void print_and_check_tree(...)              print_and_check_tree([cxt, coro_id])
//   void lock_bench(const Key&, ...)            lock_bench(k[, cxt, coro_id])
//   void index_cache_statistics()               index_cache_statistics() (the leaf directory's)
//   void clear_statistics()                     clear_statistics()
//   (new) batched forms on device pointers      search_batch / insert_batch / mixed_batch
//
// The coroutine arguments are accepted and ignored, so call sites of the
// reference's coroutine path (src/Tree.cpp:1088-1093) compile unchanged: a
// GPU batch hides latency with occupancy, not with coroutines.
//
// Single ops are batches of one, staged through small device buffers; the
// batched forms are the hot path.  Errors that the reference turns into
// assert()/infinite retries throw shm::Error here.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/sherman_amd.h"

namespace shm {

// the reference's coroutine context (include/Common.h); only its pointer is
// ever passed here
struct CoroContext;

using Key = uint64_t;    // include/Common.h:113
using Value = uint64_t;  // include/Common.h:114
constexpr Value kValueNull = 0;

struct Error : std::runtime_error {
  int status;
  Error(int s, const std::string& what)
      : std::runtime_error(what + ": " + shm_strerror(s)), status(s) {}
};

inline void check(int s, const char* what) {
  if (s != SHM_OK) throw Error(s, what);
}

class Tree {
 public:
  explicit Tree(const shm_config& cfg, uint16_t tree_id = 0) : tree_id(tree_id) {
    check(shm_tree_create(&cfg, &t_), "shm_tree_create");
    if (hipSetDevice(cfg.device) != hipSuccess ||
        hipMalloc(&d_keys_, 2 * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&d_vals_, 2 * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&d_found_, 8) != hipSuccess) {
      release();  // whichever of them were allocated
      throw Error(SHM_ENOMEM, "staging buffers");
    }
  }
  static shm_config default_config() {
    shm_config c;
    shm_config_init(&c);
    return c;
  }
  ~Tree() { release(); }
  Tree(const Tree&) = delete;
  Tree& operator=(const Tree&) = delete;

  // Tree::insert (Tree.cpp:353-403); v == kValueNull deletes
  void insert(const Key& k, const Value& v, CoroContext* cxt = nullptr, int coro_id = 0) {
    (void)cxt;
    (void)coro_id;
    stage(k, &v);
    check(shm_insert_batch(t_, d_keys_, d_vals_, 1, nullptr), "insert");
  }
  // Tree::search (Tree.cpp:405-459)
  bool search(const Key& k, Value& v, CoroContext* cxt = nullptr, int coro_id = 0) {
    (void)cxt;
    (void)coro_id;
    stage(k, nullptr);
    check(shm_search_batch(t_, d_keys_, 1, d_vals_, d_found_, nullptr), "search");
    uint8_t f = 0;
    if (hipMemcpy(&v, d_vals_, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&f, d_found_, 1, hipMemcpyDeviceToHost) != hipSuccess)
      throw Error(SHM_EIO, "search copy-back");
    return f != 0;
  }
  // Tree::del (Tree.cpp:542-591)
  void del(const Key& k, CoroContext* cxt = nullptr, int coro_id = 0) {
    (void)cxt;
    (void)coro_id;
    stage(k, nullptr);
    check(shm_del_batch(t_, d_keys_, 1, nullptr), "del");
  }
  // Tree::range_query (Tree.cpp:461-540), intended semantics: values of
  // [from, to] in leaf then slot order; `buffer` must hold every match.
  uint64_t range_query(const Key& from, const Key& to, Value* buffer,
                       CoroContext* cxt = nullptr, int coro_id = 0) {
    (void)cxt;
    (void)coro_id;
    uint64_t h[2] = {from, to};
    uint64_t *d_from = d_keys_, *d_to = d_keys_ + 1, *d_cnt = d_vals_;
    if (hipMemcpy(d_keys_, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess)
      throw Error(SHM_EIO, "range stage");
    check(shm_range_query(t_, d_from, d_to, 1, d_cnt, nullptr, nullptr, nullptr),
          "range count");
    uint64_t cnt = 0;
    if (hipMemcpy(&cnt, d_cnt, sizeof(cnt), hipMemcpyDeviceToHost) != hipSuccess)
      throw Error(SHM_EIO, "range count copy");
    if (cnt == 0) return 0;
    uint64_t *d_out = nullptr, *d_off = nullptr;
    if (hipMalloc(&d_out, cnt * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&d_off, sizeof(uint64_t)) != hipSuccess ||
        hipMemset(d_off, 0, sizeof(uint64_t)) != hipSuccess) {
      if (d_out) (void)hipFree(d_out);
      if (d_off) (void)hipFree(d_off);
      throw Error(SHM_ENOMEM, "range buffers");
    }
    int s = shm_range_query(t_, d_from, d_to, 1, d_cnt, d_off, d_out, nullptr);
    if (s == SHM_OK &&
        hipMemcpy(buffer, d_out, cnt * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
      s = SHM_EIO;
    (void)hipFree(d_out);
    (void)hipFree(d_off);
    check(s, "range_query");
    return cnt;
  }

  // batched hot path on device pointers (see include/sherman_amd.h)
  void search_batch(const Key* d_keys, uint64_t n, Value* d_vals,
                    uint8_t* d_found, hipStream_t s = nullptr) {
    check(shm_search_batch(t_, d_keys, n, d_vals, d_found, s), "search_batch");
  }
  void insert_batch(const Key* d_keys, const Value* d_vals, uint64_t n,
                    hipStream_t s = nullptr) {
    check(shm_insert_batch(t_, d_keys, d_vals, n, s), "insert_batch");
  }
  // one mixed batch: the gets see the tree before the batch's inserts
  void mixed_batch(const Key* d_get, uint64_t n_get, Value* d_vals, uint8_t* d_found,
                   const Key* d_ins, const Value* d_ins_vals, uint64_t n_ins,
                   hipStream_t s = nullptr) {
    check(shm_mixed_batch(t_, d_get, n_get, d_vals, d_found, d_ins, d_ins_vals, n_ins, s),
          "mixed_batch");
  }

  // Tree::print_and_check_tree (Tree.cpp:151-203) -> structural check
  void check_tree(uint64_t* leaves = nullptr, uint64_t* internal = nullptr,
                  uint64_t* keys = nullptr) {
    check(shm_check(t_, leaves, internal, keys), "check");
  }
  // the reference's name: checks the tree and prints its shape
  void print_and_check_tree(CoroContext* cxt = nullptr, int coro_id = 0) {
    (void)cxt;
    (void)coro_id;
    uint64_t leaves = 0, internal = 0, keys = 0;
    check_tree(&leaves, &internal, &keys);
    const shm_stats_t st = stats();
    printf("tree %u: height %u, %llu leaves, %llu internal pages, %llu keys\n",
           (unsigned)tree_id, st.height, (unsigned long long)leaves,
           (unsigned long long)internal, (unsigned long long)keys);
  }
  shm_stats_t stats() {
    shm_stats_t s;
    check(shm_stats(t_, &s), "stats");
    return s;
  }
  // Tree::lock_bench (Tree.cpp:310-321): take and release k's lock word
  void lock_bench(const Key& k, CoroContext* cxt = nullptr, int coro_id = 0) {
    (void)cxt;
    (void)coro_id;
    stage(k, nullptr);
    check(shm_lock_bench(t_, d_keys_, 1, nullptr), "lock_bench");
    check(shm_synchronize(t_), "lock_bench");
  }
  // Tree::index_cache_statistics / clear_statistics (Tree.cpp:1175-1185):
  // the index here is the leaf directory (or the LDS replica); its counters
  // are collected while enable_statistics(true)
  void enable_statistics(bool on) { check(shm_profile_enable(t_, on ? 2 : 0), "statistics"); }
  void index_cache_statistics() {
    shm_index_stats_t s;
    check(shm_index_stats(t_, &s, 0), "index statistics");
    const double g = s.gets ? (double)s.gets : 1.0;
    printf("index: %llu gets, %.4f start off a leaf, %.4f right moves, %.4f page hops, "
           "%.3f entry reads per get, %llu hits\n",
           (unsigned long long)s.gets, s.start_internal / g, s.right_moves / g, s.page_hops / g,
           s.entry_reads / g, (unsigned long long)s.hits);
  }
  void clear_statistics() {
    shm_index_stats_t s;
    check(shm_index_stats(t_, &s, 1), "clear statistics");
  }
  shm_tree* handle() { return t_; }

  const uint64_t tree_id;  // include/Tree.h:67 (one tree per handle here)

 private:
  void stage(const Key& k, const Value* v) {
    if (hipMemcpy(d_keys_, &k, sizeof(k), hipMemcpyHostToDevice) != hipSuccess)
      throw Error(SHM_EIO, "stage key");
    if (v && hipMemcpy(d_vals_, v, sizeof(*v), hipMemcpyHostToDevice) != hipSuccess)
      throw Error(SHM_EIO, "stage value");
  }
  void release() {
    if (d_keys_) (void)hipFree(d_keys_);
    if (d_vals_) (void)hipFree(d_vals_);
    if (d_found_) (void)hipFree(d_found_);
    d_keys_ = d_vals_ = nullptr;
    d_found_ = nullptr;
    if (t_) shm_tree_destroy(t_);
    t_ = nullptr;
  }
  shm_tree* t_ = nullptr;
  uint64_t* d_keys_ = nullptr;
  uint64_t* d_vals_ = nullptr;
  uint8_t* d_found_ = nullptr;
};

}  // namespace shm
