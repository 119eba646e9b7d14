// tree_test.cpp — the reference's known-answer test (test/tree_test.cpp:31-68)
// through the host C++ facade (sherman_amd/csrc/Tree.hpp) on one MI355X.
// Single-node: the reference's node-1 spin (tree_test.cpp:25-28) has no
// counterpart.  The delete phase, which the reference only prints, is
// asserted here.  Exit code 0 = pass.
#include <cstdio>
#include <cstdlib>

#include "../../sherman_amd/csrc/Tree.hpp"

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "FAIL %s (%s:%d)\n", #c, __FILE__, __LINE__); \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

int main() {
  shm_config cfg = shm::Tree::default_config();
  cfg.arena_bytes = 64ull << 20;
  cfg.max_batch = 1 << 14;
  shm::Tree tree(cfg, /*tree_id=*/0);
  shm::Value v;
  shm::CoroContext* cxt = nullptr;  // the reference's coroutine arguments compile too
  const uint64_t N = 10240;
  for (uint64_t i = 1; i < N; ++i) tree.insert(i, i * 2);
  for (uint64_t i = N - 1; i >= 1; --i) tree.insert(i, i * 3);
  for (uint64_t i = 1; i < N; ++i) {
    bool res = tree.search(i, v);
    CHECK(res && v == i * 3);
  }
  for (uint64_t i = 1; i < N; ++i) tree.del(i, cxt, 0);
  for (uint64_t i = 1; i < N; ++i) CHECK(!tree.search(i, v));
  for (uint64_t i = N - 1; i >= 1; --i) tree.insert(i, i * 3);
  for (uint64_t i = 1; i < N; ++i) {
    bool res = tree.search(i, v);
    CHECK(res && v == i * 3);
  }
  // range_query over [100, 199]: 100 values, leaf order then slot order
  std::vector<shm::Value> buf(N);
  CHECK(tree.range_query(100, 199, buf.data()) == 100);
  uint64_t sum = 0;
  for (int i = 0; i < 100; ++i) sum += buf[i];
  CHECK(sum == 3 * (100 + 199) * 100 / 2);
  uint64_t leaves = 0, internal = 0, keys = 0;
  tree.check_tree(&leaves, &internal, &keys);
  CHECK(keys == N - 1);
  tree.print_and_check_tree(cxt, 0);
  // the remaining members of the reference's Tree (include/Tree.h:58-63)
  for (uint64_t i = 1; i < 64; ++i) tree.lock_bench(i, cxt, 0);
  tree.clear_statistics();
  tree.enable_statistics(true);
  for (uint64_t i = 1; i < 200; ++i) CHECK(tree.search(i, v) && v == i * 3);
  tree.index_cache_statistics();
  tree.enable_statistics(false);
  tree.insert(5, 55);  // the lock words are free again after lock_bench
  CHECK(tree.search(5, v) && v == 55);
  tree.insert(5, 15);
  std::printf("tree_test ok: %lu keys, %lu leaves, %lu internal pages, height %u\n",
              (unsigned long)keys, (unsigned long)leaves, (unsigned long)internal,
              tree.stats().height);
  return 0;
}
