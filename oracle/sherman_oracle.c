/*
 * sherman_oracle.c — CPU ORACLE (test infrastructure only).
 *
 * Plain-C restatement of the reference Sherman B+tree hot path over a host
 * arena.  Every function cites the reference file:line it follows.  This file
 * is the checker for the HIP product path and the "port" CPU baseline; it is
 * never linked into the product library.  See sherman_oracle.h for the
 * pinning status ("parity unpinned at the hash"; tree semantics pinned by the
 * reference KAT test/tree_test.cpp:31-68).
 */
#define _GNU_SOURCE
#include "sherman_oracle.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---- constants (include/Common.h:80-121, include/Tree.h:189-195) -------- */
#define K_PAGE 1024u             /* kInternalPageSize == kLeafPageSize */
#define K_INTERNAL_CARD 61       /* kInternalCardinality */
#define K_LEAF_CARD 54           /* kLeafCardinality */
#define K_MAX_LEVEL 7            /* define::kMaxLevelOfTree */
#define K_KEY_MAX UINT64_MAX     /* kKeyMax */
#define K_VALUE_NULL 0ull        /* kValueNull */

/* ---- byte layout (include/Tree.h:130-336) ------------ */
#define OFF_LOCK 0          /* union {crc, embedding_lock, index_cache_freq} */
#define OFF_FVER 8          /* front_version */
#define OFF_LEFTMOST 9      /* Header.leftmost_ptr */
#define OFF_SIBLING 17      /* Header.sibling_ptr */
#define OFF_LEVEL 25        /* Header.level (u8) */
#define OFF_LASTIDX 26      /* Header.last_index (i16) */
#define OFF_LOWEST 28       /* Header.lowest */
#define OFF_HIGHEST 36      /* Header.highest */
#define OFF_REC 44          /* records[] */
#define OFF_INT_RVER 1020   /* InternalPage.rear_version */
#define OFF_LEAF_RVER 1016  /* LeafPage.rear_version */
#define INT_ENT 16          /* InternalEntry {key, ptr} */
#define LEAF_ENT 18         /* LeafEntry {f:4, key, value, r:4} */

#define ORC_ASSERT(c)                                                          \
  do {                                                                         \
    if (!(c)) {                                                                \
      fprintf(stderr, "oracle assertion failed: %s (%s:%d)\n", #c, __FILE__,   \
              __LINE__);                                                       \
      abort();                                                                 \
    }                                                                          \
  } while (0)

static inline uint64_t ld64(const uint8_t *p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}
static inline void st64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
static inline int16_t ld16s(const uint8_t *p) {
  int16_t v;
  memcpy(&v, p, 2);
  return v;
}
static inline void st16s(uint8_t *p, int16_t v) { memcpy(p, &v, 2); }

/* page header accessors */
#define P_LEFTMOST(p) ld64((p) + OFF_LEFTMOST)
#define P_SIBLING(p) ld64((p) + OFF_SIBLING)
#define P_LEVEL(p) ((p)[OFF_LEVEL])
#define P_LASTIDX(p) ld16s((p) + OFF_LASTIDX)
#define P_LOWEST(p) ld64((p) + OFF_LOWEST)
#define P_HIGHEST(p) ld64((p) + OFF_HIGHEST)
/* internal records */
#define I_KEY(p, j) ld64((p) + OFF_REC + INT_ENT * (j))
#define I_PTR(p, j) ld64((p) + OFF_REC + INT_ENT * (j) + 8)
/* leaf records */
#define L_BASE(p, i) ((p) + OFF_REC + LEAF_ENT * (i))
#define L_FVER(p, i) (L_BASE(p, i)[0] & 0xF)
#define L_KEY(p, i) ld64(L_BASE(p, i) + 1)
#define L_VAL(p, i) ld64(L_BASE(p, i) + 9)
#define L_RVER(p, i) (L_BASE(p, i)[17] & 0xF)

static inline void set_fver(uint8_t *e, unsigned v) {
  e[0] = (uint8_t)((e[0] & 0xF0) | (v & 0xF));
}
static inline void set_rver(uint8_t *e, unsigned v) {
  e[17] = (uint8_t)((e[17] & 0xF0) | (v & 0xF));
}

/* ---- tree / arena ------------------------------------------------------ */
struct orc_tree {
  uint8_t *arena;
  uint64_t arena_bytes;
  uint64_t next_off; /* bump allocator (LocalAllocator.h:21-38) */
  int owns;
  uint16_t node_id;
  uint64_t root;     /* g_root_ptr / *root_ptr_ptr (Tree.cpp:90-114) */
  int root_level;    /* g_root_level (Directory.cpp:72-79) */
  uint64_t read_pages;
  int mt; /* multi-threaded run in progress: page reads are not counted */
  uint64_t path[K_MAX_LEVEL]; /* path_stack (Tree.cpp:21-22), single coro */
};

/* GlobalAddress{nodeID:16, offset:48} (GlobalAddress.h:7-16) */
static inline uint64_t ga_make(uint16_t node, uint64_t off) {
  return (uint64_t)node | (off << 16);
}
static inline uint64_t ga_off(uint64_t ga) { return ga >> 16; }

static uint8_t *page_at(orc_tree *t, uint64_t ga) {
  uint64_t off = ga_off(ga);
  ORC_ASSERT(ga != 0);
  ORC_ASSERT((uint16_t)(ga & 0xFFFF) == t->node_id);
  ORC_ASSERT(off + K_PAGE <= t->arena_bytes);
  return t->arena + off;
}

/* DSM::alloc (include/DSM.h:198-224) -> bump inside the arena; offset 0 is
 * reserved as Null like chunk 0 (GlobalAllocator.h:24-26). */
static uint64_t orc_alloc(orc_tree *t) {
  if (t->next_off + K_PAGE > t->arena_bytes) {
    fprintf(stderr, "oracle: shared memory space run out\n");
    abort();
  }
  uint64_t off = t->next_off;
  t->next_off += K_PAGE;
  return ga_make(t->node_id, off);
}

/* dsm->read_sync(page_buffer, addr, 1024) */
static void read_page(orc_tree *t, uint64_t ga, uint8_t *buf) {
  memcpy(buf, page_at(t, ga), K_PAGE);
  /* DSM read counter (DSM.cpp:119-120); not kept while threads share the
   * tree, so the threads do not contend on one counter line */
  if (!t->mt) t->read_pages++;
}
static void write_bytes(orc_tree *t, uint64_t ga, const uint8_t *src,
                        uint32_t n) {
  ORC_ASSERT((uint16_t)(ga & 0xFFFF) == t->node_id);
  uint64_t off = ga_off(ga);
  ORC_ASSERT(off + n <= t->arena_bytes);
  memcpy(t->arena + off, src, n);
}

/* LeafPage(uint32_t level) (Tree.h:296-304) with Header() (Tree.h:145-151)
 * and LeafEntry() (Tree.h:181-186); padding bytes zeroed. */
static void init_leaf(uint8_t *p, uint8_t level) {
  memset(p, 0, K_PAGE);
  p[OFF_LEVEL] = level;
  st16s(p + OFF_LASTIDX, -1);
  st64(p + OFF_LOWEST, 0);
  st64(p + OFF_HIGHEST, K_KEY_MAX);
}
/* InternalPage(uint32_t level) (Tree.h:231-239) */
static void init_internal(uint8_t *p, uint8_t level) {
  memset(p, 0, K_PAGE);
  p[OFF_LEVEL] = level;
  st16s(p + OFF_LASTIDX, -1);
  st64(p + OFF_LOWEST, 0);
  st64(p + OFF_HIGHEST, K_KEY_MAX);
}
/* set_consistent (Tree.h:241-248 / 306-313), CRC variant off */
static void set_consistent(uint8_t *p, int is_leaf) {
  p[OFF_FVER] = (uint8_t)(p[OFF_FVER] + 1);
  p[is_leaf ? OFF_LEAF_RVER : OFF_INT_RVER] = p[OFF_FVER];
}
/* check_consistent (Tree.h:250-261 / 315-327) */
static int check_consistent(const uint8_t *p, int is_leaf) {
  return p[OFF_FVER] == p[is_leaf ? OFF_LEAF_RVER : OFF_INT_RVER];
}

orc_tree *orc_tree_create(uint64_t arena_bytes) {
  orc_tree *t = (orc_tree *)calloc(1, sizeof(orc_tree));
  if (arena_bytes < 4 * K_PAGE) arena_bytes = 4 * K_PAGE;
  t->arena = (uint8_t *)calloc(1, arena_bytes);
  if (!t->arena) {
    free(t);
    return NULL;
  }
  t->arena_bytes = arena_bytes;
  t->next_off = K_PAGE; /* offset 0 == Null */
  t->owns = 1;
  t->node_id = 0;
  /* Tree::Tree (Tree.cpp:44-60): empty leaf root, set_consistent, CAS root */
  uint8_t buf[K_PAGE];
  init_leaf(buf, 0);
  set_consistent(buf, 1);
  uint64_t root = orc_alloc(t);
  write_bytes(t, root, buf, K_PAGE);
  t->root = root;
  t->root_level = 0;
  return t;
}

orc_tree *orc_tree_wrap_image(uint8_t *image, uint64_t image_bytes,
                              uint64_t capacity_bytes, uint64_t root_ptr,
                              uint16_t node_id) {
  orc_tree *t = (orc_tree *)calloc(1, sizeof(orc_tree));
  t->arena = image;
  /* pages past image_bytes (up to capacity_bytes) are free for splits */
  t->arena_bytes = capacity_bytes > image_bytes ? capacity_bytes : image_bytes;
  t->next_off = image_bytes;
  t->owns = 0;
  t->node_id = node_id;
  t->root = root_ptr;
  t->root_level = page_at(t, root_ptr)[OFF_LEVEL];
  return t;
}

void orc_tree_destroy(orc_tree *t) {
  if (!t) return;
  if (t->owns) free(t->arena);
  free(t);
}

/* ---- search --------------------------------------------------------------- */
typedef struct {
  int is_leaf;
  uint8_t level;
  uint64_t sibling;
  uint64_t next_level;
  uint64_t val;
} search_result; /* SearchResult (Tree.h:32-38) */

/* internal_page_search (Tree.cpp:665-685) */
static void internal_page_search(const uint8_t *p, uint64_t k,
                                 search_result *r) {
  int cnt = P_LASTIDX(p) + 1;
  if (k < I_KEY(p, 0)) {
    r->next_level = P_LEFTMOST(p);
    return;
  }
  for (int i = 1; i < cnt; ++i) {
    if (k < I_KEY(p, i)) {
      r->next_level = I_PTR(p, i - 1);
      return;
    }
  }
  r->next_level = I_PTR(p, cnt - 1);
}

/* leaf_page_search (Tree.cpp:687-697) */
static void leaf_page_search(const uint8_t *p, uint64_t k, search_result *r) {
  for (int i = 0; i < K_LEAF_CARD; ++i) {
    if (L_KEY(p, i) == k && L_VAL(p, i) != K_VALUE_NULL &&
        L_FVER(p, i) == L_RVER(p, i)) {
      r->val = L_VAL(p, i);
      break;
    }
  }
}

/* page_search (Tree.cpp:593-663); returns 0 on the reference's `false`.
 * `track` mirrors path_stack[coro_id][level] = page_addr (Tree.cpp:610). */
static int page_search(orc_tree *t, uint64_t ga, uint64_t k, search_result *r,
                       int track) {
  uint8_t buf[K_PAGE];
  int counter = 0;
re_read:
  if (++counter > 100) return 0; /* "re read too many times" (Tree.cpp:601) */
  read_page(t, ga, buf);
  memset(r, 0, sizeof(*r));
  r->is_leaf = P_LEFTMOST(buf) == 0;
  r->level = P_LEVEL(buf);
  if (track && r->level < K_MAX_LEVEL) t->path[r->level] = ga;
  if (r->is_leaf) {
    if (!check_consistent(buf, 1)) goto re_read;
    if (k >= P_HIGHEST(buf)) { /* should turn right (Tree.cpp:626-629) */
      r->sibling = P_SIBLING(buf);
      return 1;
    }
    if (k < P_LOWEST(buf)) return 0; /* assert(false) in the reference */
    leaf_page_search(buf, k, r);
  } else {
    if (!check_consistent(buf, 0)) goto re_read;
    if (k >= P_HIGHEST(buf)) { /* Tree.cpp:648-651 */
      r->sibling = P_SIBLING(buf);
      return 1;
    }
    if (k < P_LOWEST(buf)) return 0;
    internal_page_search(buf, k, r);
  }
  return 1;
}

/* Tree::search (Tree.cpp:405-459), index cache disabled (Directory.cpp:8) */
int orc_search(orc_tree *t, uint64_t k, uint64_t *v) {
  uint64_t p = t->root;
  search_result r;
  for (int hops = 0; hops < 1 << 20; ++hops) {
    if (!page_search(t, p, k, &r, 0)) return 0;
    if (r.is_leaf) {
      if (r.val != K_VALUE_NULL) {
        *v = r.val;
        return 1;
      }
      if (r.sibling != 0) { /* turn right */
        p = r.sibling;
        continue;
      }
      return 0;
    }
    p = r.sibling != 0 ? r.sibling : r.next_level;
    if (p == 0) return 0; /* k == kKeyMax: reference would read Null */
  }
  return 0;
}

/* ---- insert ----------------------------------------------------------------- */
static void internal_page_store(orc_tree *t, uint64_t page_addr, uint64_t k,
                                uint64_t v, uint64_t root, int level);

/* update_new_root (Tree.cpp:126-149) + broadcast (Tree.cpp:116-124,
 * Directory.cpp:72-83) */
static int update_new_root(orc_tree *t, uint64_t left, uint64_t k,
                           uint64_t right, int level, uint64_t old_root) {
  uint8_t buf[K_PAGE];
  /* InternalPage(left, key, right, level) (Tree.h:217-229) */
  init_internal(buf, (uint8_t)level);
  st64(buf + OFF_LEFTMOST, left);
  st64(buf + OFF_REC, k);
  st64(buf + OFF_REC + 8, right);
  st16s(buf + OFF_LASTIDX, 0);
  uint64_t new_root = orc_alloc(t);
  set_consistent(buf, 0);
  write_bytes(t, new_root, buf, K_PAGE);
  if (t->root == old_root) { /* cas_sync(root_ptr_ptr, old_root, new_root) */
    t->root = new_root;
    if (t->root_level < level) t->root_level = level;
    return 1;
  }
  return 0;
}

/* internal_page_store (Tree.cpp:699-826) */
static void internal_page_store(orc_tree *t, uint64_t page_addr, uint64_t k,
                                uint64_t v, uint64_t root, int level) {
  uint8_t page[K_PAGE];
  read_page(t, page_addr, page); /* lock_and_read_page (Tree.cpp:716-717) */
  ORC_ASSERT(P_LEVEL(page) == level);
  ORC_ASSERT(check_consistent(page, 0));
  if (k >= P_HIGHEST(page)) { /* Tree.cpp:723-733 */
    ORC_ASSERT(P_SIBLING(page) != 0);
    internal_page_store(t, P_SIBLING(page), k, v, root, level);
    return;
  }
  ORC_ASSERT(k >= P_LOWEST(page));
  int cnt = P_LASTIDX(page) + 1;
  int is_update = 0;
  int insert_index = 0;
  for (int i = cnt - 1; i >= 0; --i) { /* Tree.cpp:740-751 */
    if (I_KEY(page, i) == k) {
      st64(page + OFF_REC + INT_ENT * i + 8, v);
      is_update = 1;
      break;
    }
    if (I_KEY(page, i) < k) {
      insert_index = i + 1;
      break;
    }
  }
  ORC_ASSERT(cnt != K_INTERNAL_CARD);
  if (!is_update) { /* insert and shift (Tree.cpp:755-764) */
    for (int i = cnt; i > insert_index; --i) {
      memcpy(page + OFF_REC + INT_ENT * i, page + OFF_REC + INT_ENT * (i - 1),
             INT_ENT);
    }
    st64(page + OFF_REC + INT_ENT * insert_index, k);
    st64(page + OFF_REC + INT_ENT * insert_index + 8, v);
    st16s(page + OFF_LASTIDX, (int16_t)(P_LASTIDX(page) + 1));
  }
  cnt = P_LASTIDX(page) + 1;
  int need_split = cnt == K_INTERNAL_CARD;
  uint64_t split_key = 0, sibling_addr = 0;
  if (need_split) { /* Tree.cpp:770-801 */
    uint8_t sib[K_PAGE];
    sibling_addr = orc_alloc(t);
    init_internal(sib, P_LEVEL(page));
    int m = cnt / 2;
    split_key = I_KEY(page, m);
    ORC_ASSERT(split_key > P_LOWEST(page));
    ORC_ASSERT(split_key < P_HIGHEST(page));
    for (int i = m + 1; i < cnt; ++i) {
      memcpy(sib + OFF_REC + INT_ENT * (i - m - 1), page + OFF_REC + INT_ENT * i,
             INT_ENT);
    }
    st16s(page + OFF_LASTIDX, (int16_t)(P_LASTIDX(page) - (cnt - m)));
    st16s(sib + OFF_LASTIDX, (int16_t)(P_LASTIDX(sib) + (cnt - m - 1)));
    st64(sib + OFF_LEFTMOST, I_PTR(page, m));
    st64(sib + OFF_LOWEST, I_KEY(page, m));
    st64(sib + OFF_HIGHEST, P_HIGHEST(page));
    st64(page + OFF_HIGHEST, I_KEY(page, m));
    st64(sib + OFF_SIBLING, P_SIBLING(page));
    st64(page + OFF_SIBLING, sibling_addr);
    set_consistent(sib, 0);
    write_bytes(t, sibling_addr, sib, K_PAGE);
  }
  set_consistent(page, 0);
  write_bytes(t, page_addr, page, K_PAGE); /* write_page_and_unlock */
  if (!need_split) return;
  if (root == page_addr) { /* Tree.cpp:810-816 */
    if (update_new_root(t, page_addr, split_key, sibling_addr, level + 1, root))
      return;
  }
  ORC_ASSERT(level + 1 < K_MAX_LEVEL);
  uint64_t up = t->path[level + 1];
  ORC_ASSERT(up != 0); /* assert(false) branch (Tree.cpp:823-825) */
  internal_page_store(t, up, split_key, sibling_addr, root, level + 1);
}

static int cmp_leaf_entry(const void *a, const void *b) {
  uint64_t ka = ld64((const uint8_t *)a + 1), kb = ld64((const uint8_t *)b + 1);
  return ka < kb ? -1 : (ka > kb ? 1 : 0);
}

/* leaf_page_store (Tree.cpp:828-991), non-cache path */
static void leaf_page_store(orc_tree *t, uint64_t page_addr, uint64_t k,
                            uint64_t v, uint64_t root, int level) {
  uint8_t page[K_PAGE];
  read_page(t, page_addr, page); /* lock_and_read_page (Tree.cpp:851-852) */
  ORC_ASSERT(P_LEVEL(page) == level);
  ORC_ASSERT(check_consistent(page, 1));
  if (k >= P_HIGHEST(page)) { /* Tree.cpp:865-872 */
    ORC_ASSERT(P_SIBLING(page) != 0);
    leaf_page_store(t, P_SIBLING(page), k, v, root, level);
    return;
  }
  ORC_ASSERT(k >= P_LOWEST(page));
  int cnt = 0, empty_index = -1, update_index = -1;
  for (int i = 0; i < K_LEAF_CARD; ++i) { /* Tree.cpp:878-893 */
    uint8_t *e = L_BASE(page, i);
    if (L_VAL(page, i) != K_VALUE_NULL) {
      cnt++;
      if (L_KEY(page, i) == k) {
        st64(e + 9, v);
        set_fver(e, (L_FVER(page, i) + 1) & 0xF);
        set_rver(e, L_FVER(page, i));
        update_index = i;
        break;
      }
    } else if (empty_index == -1) {
      empty_index = i;
    }
  }
  ORC_ASSERT(cnt != K_LEAF_CARD);
  if (update_index < 0) { /* insert new item (Tree.cpp:897-912) */
    ORC_ASSERT(empty_index != -1);
    uint8_t *e = L_BASE(page, empty_index);
    st64(e + 1, k);
    st64(e + 9, v);
    set_fver(e, (L_FVER(page, empty_index) + 1) & 0xF);
    set_rver(e, L_FVER(page, empty_index));
    update_index = empty_index;
    cnt++;
  }
  int need_split = cnt == K_LEAF_CARD;
  if (!need_split) { /* write back the 18 B entry only (Tree.cpp:915-921) */
    uint64_t eoff = OFF_REC + LEAF_ENT * (uint64_t)update_index;
    write_bytes(t, page_addr + (eoff << 16), L_BASE(page, update_index),
                LEAF_ENT);
    return;
  }
  /* std::sort by key (Tree.cpp:923-925); keys are unique among 54 valid */
  qsort(page + OFF_REC, K_LEAF_CARD, LEAF_ENT, cmp_leaf_entry);
  uint8_t sib[K_PAGE];
  uint64_t sibling_addr = orc_alloc(t); /* Tree.cpp:930-963 */
  init_leaf(sib, P_LEVEL(page));
  int m = cnt / 2;
  uint64_t split_key = L_KEY(page, m);
  ORC_ASSERT(split_key > P_LOWEST(page));
  ORC_ASSERT(split_key < P_HIGHEST(page));
  for (int i = m; i < cnt; ++i) {
    st64(L_BASE(sib, i - m) + 1, L_KEY(page, i));
    st64(L_BASE(sib, i - m) + 9, L_VAL(page, i));
    st64(L_BASE(page, i) + 1, 0);
    st64(L_BASE(page, i) + 9, K_VALUE_NULL);
  }
  st16s(page + OFF_LASTIDX, (int16_t)(P_LASTIDX(page) - (cnt - m)));
  st16s(sib + OFF_LASTIDX, (int16_t)(P_LASTIDX(sib) + (cnt - m)));
  st64(sib + OFF_LOWEST, split_key);
  st64(sib + OFF_HIGHEST, P_HIGHEST(page));
  st64(page + OFF_HIGHEST, split_key);
  st64(sib + OFF_SIBLING, P_SIBLING(page));
  st64(page + OFF_SIBLING, sibling_addr);
  set_consistent(sib, 1);
  write_bytes(t, sibling_addr, sib, K_PAGE);
  set_consistent(page, 1);
  write_bytes(t, page_addr, page, K_PAGE);
  if (root == page_addr) { /* Tree.cpp:973-978 */
    if (update_new_root(t, page_addr, split_key, sibling_addr, level + 1, root))
      return;
  }
  uint64_t up = t->path[level + 1];
  ORC_ASSERT(up != 0); /* assert(from_cache) (Tree.cpp:986) */
  internal_page_store(t, up, split_key, sibling_addr, root, level + 1);
}

/* Tree::insert (Tree.cpp:353-403).  Returns 0 ok, -1 if k == kKeyMax (which
 * the reference cannot store: root highest is exclusive kKeyMax). */
int orc_insert(orc_tree *t, uint64_t k, uint64_t v) {
  if (k == K_KEY_MAX) return -1;
  for (int i = 0; i < K_MAX_LEVEL; ++i) t->path[i] = 0; /* before_operation */
  uint64_t root = t->root;
  uint64_t p = root;
  search_result r;
  for (;;) {
    if (!page_search(t, p, k, &r, 1)) {
      ORC_ASSERT(0 && "SEARCH WARNING insert");
    }
    if (!r.is_leaf) {
      ORC_ASSERT(r.level != 0);
      if (r.sibling != 0) {
        p = r.sibling;
        continue;
      }
      p = r.next_level;
      if (r.level != 1) continue;
    }
    break;
  }
  leaf_page_store(t, p, k, v, root, 0);
  return 0;
}

/* leaf_page_del (Tree.cpp:993-1057) */
static void leaf_page_del(orc_tree *t, uint64_t page_addr, uint64_t k) {
  uint8_t page[K_PAGE];
  read_page(t, page_addr, page);
  ORC_ASSERT(check_consistent(page, 1));
  if (k >= P_HIGHEST(page)) {
    ORC_ASSERT(P_SIBLING(page) != 0);
    leaf_page_del(t, P_SIBLING(page), k);
    return;
  }
  for (int i = 0; i < K_LEAF_CARD; ++i) {
    uint8_t *e = L_BASE(page, i);
    if (L_KEY(page, i) == k && L_VAL(page, i) != K_VALUE_NULL) {
      st64(e + 9, K_VALUE_NULL);
      set_fver(e, (L_FVER(page, i) + 1) & 0xF);
      set_rver(e, L_FVER(page, i));
      uint64_t eoff = OFF_REC + LEAF_ENT * (uint64_t)i;
      write_bytes(t, page_addr + (eoff << 16), e, LEAF_ENT);
      return;
    }
  }
}

/* Tree::del (Tree.cpp:542-591) */
void orc_del(orc_tree *t, uint64_t k) {
  if (k == K_KEY_MAX) return;
  uint64_t p = t->root;
  search_result r;
  for (;;) {
    if (!page_search(t, p, k, &r, 1)) ORC_ASSERT(0 && "SEARCH WARNING del");
    if (!r.is_leaf) {
      if (r.sibling != 0) {
        p = r.sibling;
        continue;
      }
      p = r.next_level;
      if (r.level != 1) continue;
    }
    break;
  }
  leaf_page_del(t, p, k);
}

/* intended range_query (Tree.cpp:461-540 with a working cache): leaves in
 * key order (sibling chain), valid slots in slot order. */
uint64_t orc_range_query(orc_tree *t, uint64_t from, uint64_t to,
                         uint64_t *out, uint64_t cap) {
  if (from > to) return 0;
  /* descend to the leaf containing `from` */
  uint64_t p = t->root;
  uint8_t buf[K_PAGE];
  for (;;) {
    read_page(t, p, buf);
    if (from >= P_HIGHEST(buf) && P_SIBLING(buf) != 0) {
      p = P_SIBLING(buf);
      continue;
    }
    if (P_LEFTMOST(buf) == 0) break;
    search_result r;
    memset(&r, 0, sizeof(r));
    internal_page_search(buf, from, &r);
    p = r.next_level;
  }
  uint64_t counter = 0;
  for (;;) {
    for (int i = 0; i < K_LEAF_CARD; ++i) { /* Tree.cpp:509-516 */
      if (L_VAL(buf, i) != K_VALUE_NULL && L_FVER(buf, i) == L_RVER(buf, i)) {
        uint64_t k = L_KEY(buf, i);
        if (k >= from && k <= to) {
          if (counter < cap) out[counter] = L_VAL(buf, i);
          counter++;
        }
      }
    }
    uint64_t sib = P_SIBLING(buf);
    if (sib == 0 || P_HIGHEST(buf) > to) break;
    read_page(t, sib, buf);
  }
  return counter;
}

/* ---- batched helpers ------------------------------------------------------- */
/* scans i = 0..n-1 one after the other: counts[i] = matches of scan i, values
 * concatenated into out (truncated at cap); returns the total count */
uint64_t orc_range_query_batch(orc_tree *t, const uint64_t *from, const uint64_t *to,
                               uint64_t n, uint64_t *counts, uint64_t *out,
                               uint64_t cap) {
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t room = total < cap ? cap - total : 0;
    counts[i] = orc_range_query(t, from[i], to[i], out + (room ? total : 0), room);
    total += counts[i];
  }
  return total;
}

void orc_search_batch(orc_tree *t, const uint64_t *keys, uint64_t n,
                      uint64_t *vals, uint8_t *found) {
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t v = 0;
    int f = orc_search(t, keys[i], &v);
    vals[i] = f ? v : 0;
    found[i] = (uint8_t)f;
  }
}

typedef struct {
  orc_tree *t;
  const uint64_t *keys;
  uint64_t *vals;
  uint8_t *found;
  uint64_t lo, hi;
  int cpu;
} mt_arg;

static void *mt_worker(void *a_) {
  mt_arg *a = (mt_arg *)a_;
  /* bindCore (Common.cpp:11-20): pin 1:1 */
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(a->cpu, &set);
  pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
  for (uint64_t i = a->lo; i < a->hi; ++i) {
    uint64_t v = 0;
    int f = orc_search(a->t, a->keys[i], &v);
    a->vals[i] = f ? v : 0;
    a->found[i] = (uint8_t)f;
  }
  return NULL;
}

double orc_search_batch_mt(orc_tree *t, const uint64_t *keys, uint64_t n,
                           uint64_t *vals, uint8_t *found, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  t->mt = 1;
  pthread_t th[256];
  mt_arg args[256];
  if (nthreads > 256) nthreads = 256;
  cpu_set_t avail;
  CPU_ZERO(&avail);
  sched_getaffinity(0, sizeof(avail), &avail);
  int cpus[1024], ncpu = 0;
  for (int c = 0; c < CPU_SETSIZE && ncpu < 1024; ++c)
    if (CPU_ISSET(c, &avail)) cpus[ncpu++] = c;
  if (ncpu == 0) cpus[ncpu++] = 0;
  struct timespec s, e;
  clock_gettime(CLOCK_MONOTONIC, &s);
  for (int i = 0; i < nthreads; ++i) {
    args[i].t = t;
    args[i].keys = keys;
    args[i].vals = vals;
    args[i].found = found;
    args[i].lo = n * (uint64_t)i / nthreads;
    args[i].hi = n * (uint64_t)(i + 1) / nthreads;
    args[i].cpu = cpus[i % ncpu];
    pthread_create(&th[i], NULL, mt_worker, &args[i]);
  }
  for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
  clock_gettime(CLOCK_MONOTONIC, &e);
  t->mt = 0;
  return (double)(e.tv_sec - s.tv_sec) + 1e-9 * (double)(e.tv_nsec - s.tv_nsec);
}

void orc_apply_batch(orc_tree *t, const uint64_t *keys, const uint64_t *vals,
                     uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) {
    if (vals[i] == K_VALUE_NULL)
      orc_del(t, keys[i]);
    else
      orc_insert(t, keys[i], vals[i]);
  }
}

/* ---- introspection ---------------------------------------------------------- */
uint64_t orc_root_ptr(const orc_tree *t) { return t->root; }
int orc_root_level(const orc_tree *t) { return t->root_level; }
uint64_t orc_pages_used(const orc_tree *t) { return t->next_off / K_PAGE - 1; }
const uint8_t *orc_arena(const orc_tree *t) { return t->arena; }
uint64_t orc_arena_bytes_used(const orc_tree *t) { return t->next_off; }
uint64_t orc_read_pages(const orc_tree *t) { return t->read_pages; }

static uint64_t leftmost_leaf(orc_tree *t) {
  uint64_t p = t->root;
  for (;;) {
    uint8_t *pg = page_at(t, p);
    if (P_LEFTMOST(pg) == 0) return p;
    p = P_LEFTMOST(pg);
  }
}

uint64_t orc_dump_pairs(orc_tree *t, uint64_t *keys, uint64_t *vals,
                        uint64_t cap) {
  uint64_t cnt = 0;
  uint64_t p = leftmost_leaf(t);
  while (p) {
    uint8_t *pg = page_at(t, p);
    for (int i = 0; i < K_LEAF_CARD; ++i) {
      if (L_VAL(pg, i) != K_VALUE_NULL && L_FVER(pg, i) == L_RVER(pg, i)) {
        if (cnt < cap) {
          keys[cnt] = L_KEY(pg, i);
          vals[cnt] = L_VAL(pg, i);
        }
        cnt++;
      }
    }
    p = P_SIBLING(pg);
  }
  return cnt;
}

/* Structural invariants of a quiescent B-link tree. */
int orc_check(orc_tree *t, uint64_t *n_leaves, uint64_t *n_internal,
              uint64_t *n_keys, int *height) {
  uint64_t leaves = 0, internals = 0, keys = 0;
  uint64_t level_head = t->root;
  int top = page_at(t, t->root)[OFF_LEVEL];
  if (height) *height = top + 1;
  for (int lvl = top; lvl >= 0; --lvl) {
    uint64_t p = level_head;
    uint64_t expect_low = 0;
    uint64_t next_head = 0;
    while (p) {
      uint8_t *pg = page_at(t, p);
      int is_leaf = P_LEFTMOST(pg) == 0;
      if (P_LEVEL(pg) != lvl) return -1;
      if ((lvl == 0) != is_leaf) return -2;
      if (!check_consistent(pg, is_leaf)) return -3;
      if (P_LOWEST(pg) != expect_low) return -4;
      if (P_HIGHEST(pg) <= P_LOWEST(pg)) return -5;
      if (is_leaf) {
        int c = 0;
        for (int i = 0; i < K_LEAF_CARD; ++i) {
          if (L_VAL(pg, i) == K_VALUE_NULL) continue;
          uint64_t k = L_KEY(pg, i);
          if (k < P_LOWEST(pg) || k >= P_HIGHEST(pg)) return -6;
          c++;
        }
        if (c > K_LEAF_CARD - 1) return -7;
        keys += (uint64_t)c;
        leaves++;
      } else {
        int cnt = P_LASTIDX(pg) + 1;
        if (cnt < 0 || cnt > K_INTERNAL_CARD - 1) return -8;
        uint64_t prev = P_LOWEST(pg);
        uint64_t child = P_LEFTMOST(pg);
        if (!next_head) next_head = child;
        uint8_t *cp = page_at(t, child);
        if (P_LOWEST(cp) != P_LOWEST(pg)) return -9;
        for (int j = 0; j < cnt; ++j) {
          uint64_t k = I_KEY(pg, j);
          if (!(k > prev || (j == 0 && k > P_LOWEST(pg)))) return -10;
          if (k >= P_HIGHEST(pg)) return -11;
          prev = k;
          cp = page_at(t, I_PTR(pg, j));
          if (P_LOWEST(cp) != k) return -12;
          if ((int)P_LEVEL(cp) != lvl - 1) return -13;
        }
        internals++;
      }
      expect_low = P_HIGHEST(pg);
      p = P_SIBLING(pg);
    }
    if (expect_low != K_KEY_MAX) return -14;
    level_head = next_head;
  }
  if (n_leaves) *n_leaves = leaves;
  if (n_internal) *n_internal = internals;
  if (n_keys) *n_keys = keys;
  return 0;
}

/* ---- generators --------------------------------------------------------------- */
/* CityHash64 v1.1 (google/cityhash city.cc, lengths <= 16), restated. */
static const uint64_t kC0 = 0xc3a5c85c97cb3127ULL;
static const uint64_t kC2 = 0x9ae16a3b2f90404fULL;
static inline uint64_t rot64(uint64_t v, int s) {
  return s == 0 ? v : ((v >> s) | (v << (64 - s)));
}
static inline uint64_t shift_mix(uint64_t v) { return v ^ (v >> 47); }
static inline uint64_t hash_len16_mul(uint64_t u, uint64_t v, uint64_t mul) {
  uint64_t a = (u ^ v) * mul;
  a ^= (a >> 47);
  uint64_t b = (v ^ a) * mul;
  b ^= (b >> 47);
  b *= mul;
  return b;
}
static inline uint32_t ld32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
uint64_t orc_cityhash64(const void *s_, size_t len) {
  const uint8_t *s = (const uint8_t *)s_;
  ORC_ASSERT(len <= 16);
  if (len >= 8) {
    uint64_t mul = kC2 + len * 2;
    uint64_t a = ld64(s) + kC2;
    uint64_t b = ld64(s + len - 8);
    uint64_t c = rot64(b, 37) * mul + a;
    uint64_t d = (rot64(a, 25) + b) * mul;
    return hash_len16_mul(c, d, mul);
  }
  if (len >= 4) {
    uint64_t mul = kC2 + len * 2;
    uint64_t a = ld32(s);
    return hash_len16_mul(len + (a << 3), ld32(s + len - 4), mul);
  }
  if (len > 0) {
    uint8_t a = s[0], b = s[len >> 1], c = s[len - 1];
    uint32_t y = (uint32_t)a + ((uint32_t)b << 8);
    uint32_t z = (uint32_t)len + ((uint32_t)c << 2);
    return shift_mix(y * kC2 ^ z * kC0) * kC2;
  }
  return kC2;
}

/* to_key (test/benchmark.cpp:43-46) */
uint64_t orc_to_key(uint64_t i, uint64_t keyspace) {
  uint64_t h = orc_cityhash64(&i, sizeof(i)) + 1;
  return keyspace ? h % keyspace : h;
}

/* mehcached_rand_d (zipf.h:57-61) */
static double rand_d(uint64_t *state) {
  *state = (*state * 0x5deece66dULL + 0xbULL) & ((1ULL << 48) - 1);
  return (double)*state / (double)((1ULL << 48) - 1);
}
/* mehcached_pow_approx (zipf.h:65-91) */
static double pow_approx(double a, double b) {
  int e = (int)b;
  union {
    double d;
    int x[2];
  } u = {a};
  u.x[1] = (int)((b - (double)e) * (double)(u.x[1] - 1072632447) + 1072632447.);
  u.x[0] = 0;
  double r = 1.;
  while (e) {
    if (e & 1) r *= a;
    a *= a;
    e >>= 1;
  }
  return r * u.d;
}
/* mehcached_zeta (zipf.h:149-160) */
static double zeta(uint64_t last_n, double last_sum, uint64_t n, double theta) {
  if (last_n > n) {
    last_n = 0;
    last_sum = 0.;
  }
  while (last_n < n) {
    last_sum += 1. / pow_approx((double)last_n + 1., theta);
    last_n++;
  }
  return last_sum;
}
/* mehcached_zipf_init (zipf.h:96-126) */
void orc_zipf_init(orc_zipf *z, uint64_t n, double theta, uint64_t seed) {
  ORC_ASSERT(n > 0);
  ORC_ASSERT(theta == -1. || (theta >= 0. && theta < 1.) || theta >= 40.);
  ORC_ASSERT(seed < (1ULL << 48));
  memset(z, 0, sizeof(*z));
  z->n = n;
  z->theta = theta;
  if (theta == -1.)
    seed = seed % n;
  else if (theta > 0. && theta < 1.) {
    z->alpha = 1. / (1. - theta);
    z->thres = 1. + pow_approx(0.5, theta);
  }
  z->rand_state = seed;
}
/* mehcached_zipf_next (zipf.h:163-203) */
uint64_t orc_zipf_next(orc_zipf *z) {
  if (z->last_n != z->n) {
    if (z->theta > 0. && z->theta < 1.) {
      z->zetan = zeta(z->last_n, z->zetan, z->n, z->theta);
      z->eta = (1. - pow_approx(2. / (double)z->n, 1. - z->theta)) /
               (1. - zeta(0, 0., 2, z->theta) / z->zetan);
    }
    z->last_n = z->n;
    z->dbl_n = (double)z->n;
  }
  if (z->theta == -1.) {
    uint64_t v = z->rand_state;
    if (++z->rand_state >= z->n) z->rand_state = 0;
    return v;
  } else if (z->theta == 0.) {
    double u = rand_d(&z->rand_state);
    return (uint64_t)(z->dbl_n * u);
  } else if (z->theta >= 40.) {
    return 0;
  } else {
    double u = rand_d(&z->rand_state);
    double uz = u * z->zetan;
    if (uz < 1.) return 0;
    if (uz < z->thres) return 1;
    return (uint64_t)(z->dbl_n * pow_approx(z->eta * (u - 1.) + 1., z->alpha));
  }
}
void orc_zipf_fill(uint64_t n_items, double theta, uint64_t seed, uint64_t *out,
                   uint64_t count) {
  orc_zipf z;
  orc_zipf_init(&z, n_items, theta, seed);
  for (uint64_t i = 0; i < count; ++i) out[i] = orc_zipf_next(&z);
}
/* op mix (benchmark.cpp:173): glibc rand_r */
void orc_op_mix(unsigned int seed, int read_ratio, uint8_t *is_get,
                uint64_t count) {
  for (uint64_t i = 0; i < count; ++i)
    is_get[i] = (uint8_t)(rand_r(&seed) % 100 < read_ratio);
}

/* ---- multi-threaded CPU baseline (the reference benchmark's thread model) --
 * Threads pinned 1:1 to the CPUs of the affinity mask (bindCore,
 * src/Common.cpp:11-20; test/benchmark.cpp:96). */
static int avail_cpus(int *cpus, int max) {
  cpu_set_t avail;
  CPU_ZERO(&avail);
  sched_getaffinity(0, sizeof(avail), &avail);
  int n = 0;
  for (int c = 0; c < CPU_SETSIZE && n < max; ++c)
    if (CPU_ISSET(c, &avail)) cpus[n++] = c;
  if (n == 0) cpus[n++] = 0;
  return n;
}
static void pin_cpu(int cpu) {
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(cpu, &set);
  pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}
static double now_s(void) {
  struct timespec s;
  clock_gettime(CLOCK_MONOTONIC, &s);
  return (double)s.tv_sec + 1e-9 * (double)s.tv_nsec;
}

/* Tree::insert's descent to the leaf (Tree.cpp:353-403), read-only */
static uint64_t locate_leaf(orc_tree *t, uint64_t k) {
  uint64_t p = t->root;
  search_result r;
  for (int hops = 0; hops < 1 << 20; ++hops) {
    if (!page_search(t, p, k, &r, 0)) return 0;
    if (r.is_leaf) {
      if (r.sibling != 0) { /* k >= highest: turn right */
        p = r.sibling;
        continue;
      }
      return p;
    }
    p = r.sibling != 0 ? r.sibling : r.next_level;
    if (p == 0) return 0;
  }
  return 0;
}

/* leaf_page_store's no-split path (Tree.cpp:875-921) applied in place by the
 * thread that owns the page's lock word; 0 when the insert would reach 54
 * entries (the split point, Tree.cpp:914): the page is left untouched */
static int leaf_store_inplace(orc_tree *t, uint64_t page_addr, uint64_t k, uint64_t v) {
  uint8_t *page = page_at(t, page_addr);
  int cnt = 0, empty_index = -1;
  for (int i = 0; i < K_LEAF_CARD; ++i) {
    uint8_t *e = L_BASE(page, i);
    if (L_VAL(page, i) != K_VALUE_NULL) {
      cnt++;
      if (L_KEY(page, i) == k) {
        st64(e + 9, v);
        set_fver(e, (L_FVER(page, i) + 1) & 0xF);
        set_rver(e, L_FVER(page, i));
        return 1;
      }
    } else if (empty_index == -1) {
      empty_index = i;
    }
  }
  if (cnt + 1 >= K_LEAF_CARD || empty_index < 0) return 0;
  uint8_t *e = L_BASE(page, empty_index);
  st64(e + 1, k);
  st64(e + 9, v);
  set_fver(e, (L_FVER(page, empty_index) + 1) & 0xF);
  set_rver(e, L_FVER(page, empty_index));
  return 1;
}

/* leaf_page_del's body (Tree.cpp:1037-1055) on the located leaf */
static void leaf_del_inplace(orc_tree *t, uint64_t page_addr, uint64_t k) {
  uint8_t *page = page_at(t, page_addr);
  for (int i = 0; i < K_LEAF_CARD; ++i) {
    uint8_t *e = L_BASE(page, i);
    if (L_KEY(page, i) == k && L_VAL(page, i) != K_VALUE_NULL) {
      st64(e + 9, K_VALUE_NULL);
      set_fver(e, (L_FVER(page, i) + 1) & 0xF);
      set_rver(e, L_FVER(page, i));
      return;
    }
  }
}

typedef struct {
  orc_tree *t;
  const uint64_t *keys, *vals;
  uint64_t n;
  uint64_t *leaf;
  uint16_t *owner;
  uint8_t *defer;
  int tid, nthreads, cpu;
  pthread_barrier_t *bar;
} am_arg;

/* tiny open-addressing set of page addresses (per thread) */
typedef struct {
  uint64_t *slot;
  uint64_t cap, n;
} pset;
static int pset_has(const pset *s, uint64_t x) {
  if (!s->cap) return 0;
  for (uint64_t h = (x * 0x9E3779B97F4A7C15ull) & (s->cap - 1);; h = (h + 1) & (s->cap - 1)) {
    if (s->slot[h] == x) return 1;
    if (s->slot[h] == 0) return 0;
  }
}
static void pset_add(pset *s, uint64_t x) {
  if (2 * (s->n + 1) > s->cap) {
    pset o = *s;
    s->cap = o.cap ? 2 * o.cap : 64;
    s->slot = (uint64_t *)calloc(s->cap, 8);
    s->n = 0;
    for (uint64_t i = 0; i < o.cap; ++i)
      if (o.slot[i]) pset_add(s, o.slot[i]);
    free(o.slot);
  }
  uint64_t h = (x * 0x9E3779B97F4A7C15ull) & (s->cap - 1);
  while (s->slot[h] != 0 && s->slot[h] != x) h = (h + 1) & (s->cap - 1);
  if (s->slot[h] == 0) {
    s->slot[h] = x;
    s->n++;
  }
}

static void *am_worker(void *a_) {
  am_arg *a = (am_arg *)a_;
  pin_cpu(a->cpu);
  /* 1. every op's leaf (a read-only descent; no page splits yet) and the
   *    thread owning its lock word lock[CityHash64(page) % kNumOfLock]
   *    (Tree.cpp:832-842, kNumOfLock = 16384, include/Common.h:87-93) */
  const uint64_t lo = a->n * (uint64_t)a->tid / a->nthreads;
  const uint64_t hi = a->n * (uint64_t)(a->tid + 1) / a->nthreads;
  for (uint64_t i = lo; i < hi; ++i) {
    const uint64_t k = a->keys[i];
    const uint64_t lf = k == K_KEY_MAX ? 0 : locate_leaf(a->t, k);
    a->leaf[i] = lf;
    a->owner[i] = (uint16_t)(lf ? (orc_cityhash64(&lf, 8) % 16384) % (uint64_t)a->nthreads : 0);
  }
  pthread_barrier_wait(a->bar);
  /* 2. this thread's pages, in batch order: in place, or (the page would
   *    split) left for the serial pass together with every later op on it */
  pset deferred = {0, 0, 0};
  for (uint64_t i = 0; i < a->n; ++i) {
    if (a->owner[i] != (uint16_t)a->tid) continue;
    const uint64_t lf = a->leaf[i];
    if (!lf || pset_has(&deferred, lf)) {
      a->defer[i] = 1;
      continue;
    }
    if (a->vals[i] == K_VALUE_NULL) {
      leaf_del_inplace(a->t, lf, a->keys[i]);
    } else if (!leaf_store_inplace(a->t, lf, a->keys[i], a->vals[i])) {
      pset_add(&deferred, lf);
      a->defer[i] = 1;
    }
  }
  free(deferred.slot);
  return NULL;
}

/* The batch applied in order (Tree::insert / Tree::del per op) by `nthreads`
 * threads partitioned by page lock word, as concurrent Sherman clients
 * serialise on those words; ops on a page that must split run afterwards in
 * batch order on one thread (splits touch parents).  Same key->value
 * contents as orc_apply_batch.  Returns seconds. */
double orc_apply_batch_mt(orc_tree *t, const uint64_t *keys, const uint64_t *vals, uint64_t n,
                          int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 1024) nthreads = 1024;
  static int cpus[1024];
  const int ncpu = avail_cpus(cpus, 1024);
  uint64_t *leaf = (uint64_t *)malloc(8 * (n ? n : 1));
  uint16_t *owner = (uint16_t *)malloc(2 * (n ? n : 1));
  uint8_t *defer = (uint8_t *)calloc(n ? n : 1, 1);
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
  am_arg *args = (am_arg *)malloc(sizeof(am_arg) * nthreads);
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
  const double t0 = now_s();
  t->mt = 1;
  for (int i = 0; i < nthreads; ++i) {
    args[i] = (am_arg){t, keys, vals, n, leaf, owner, defer, i, nthreads, cpus[i % ncpu], &bar};
    pthread_create(&th[i], NULL, am_worker, &args[i]);
  }
  for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
  t->mt = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (!defer[i]) continue;
    if (vals[i] == K_VALUE_NULL)
      orc_del(t, keys[i]);
    else
      orc_insert(t, keys[i], vals[i]);
  }
  const double secs = now_s() - t0;
  pthread_barrier_destroy(&bar);
  free(leaf);
  free(owner);
  free(defer);
  free(th);
  free(args);
  return secs;
}

typedef struct {
  orc_tree *t;
  const uint64_t *from, *to;
  uint64_t lo, hi;
  uint64_t *counts;
  const uint64_t *offs;
  uint64_t *out;
  int cpu;
} rq_arg;
static void *rq_worker(void *a_) {
  rq_arg *a = (rq_arg *)a_;
  pin_cpu(a->cpu);
  for (uint64_t i = a->lo; i < a->hi; ++i) {
    if (a->offs)
      (void)orc_range_query(a->t, a->from[i], a->to[i], a->out + a->offs[i], a->counts[i]);
    else
      a->counts[i] = orc_range_query(a->t, a->from[i], a->to[i], NULL, 0);
  }
  return NULL;
}

/* orc_range_query_batch on `nthreads` threads: counts, then the values at
 * their offsets (out must hold the total, which is returned).  Seconds in
 * *secs. */
uint64_t orc_range_query_batch_mt(orc_tree *t, const uint64_t *from, const uint64_t *to,
                                  uint64_t n, uint64_t *counts, uint64_t *out, uint64_t cap,
                                  int nthreads, double *secs) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 1024) nthreads = 1024;
  static int cpus[1024];
  const int ncpu = avail_cpus(cpus, 1024);
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
  rq_arg *args = (rq_arg *)malloc(sizeof(rq_arg) * nthreads);
  uint64_t *offs = (uint64_t *)malloc(8 * (n ? n : 1));
  const double t0 = now_s();
  t->mt = 1;
  uint64_t total = 0;
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1) {
      for (uint64_t i = 0; i < n; ++i) {
        offs[i] = total;
        total += counts[i];
      }
      if (total > cap) break;
    }
    for (int i = 0; i < nthreads; ++i) {
      args[i] = (rq_arg){t, from, to, n * (uint64_t)i / nthreads, n * (uint64_t)(i + 1) / nthreads,
                         counts, pass ? offs : NULL, out, cpus[i % ncpu]};
      pthread_create(&th[i], NULL, rq_worker, &args[i]);
    }
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
  }
  t->mt = 0;
  if (secs) *secs = now_s() - t0;
  free(th);
  free(args);
  free(offs);
  return total;
}

typedef struct {
  orc_tree *t;
  uint64_t keyspace;
  double theta;
  uint64_t seed;
  int cpu;
  volatile int *stop;
  volatile int *ready;
  volatile uint64_t *count; /* this thread's op counter (own cache line) */
} c1_arg;
static void *c1_worker(void *a_) {
  c1_arg *a = (c1_arg *)a_;
  pin_cpu(a->cpu);
  orc_zipf z;
  orc_zipf_init(&z, a->keyspace, a->theta, a->seed);
  __atomic_fetch_add(a->ready, 1, __ATOMIC_RELEASE);
  uint64_t done = 0;
  while (!__atomic_load_n(a->stop, __ATOMIC_RELAXED)) {
    for (int j = 0; j < 256; ++j) {
      /* key = to_key(zipf_next()), a search (kReadRatio = 100),
       * test/benchmark.cpp:165-177 */
      const uint64_t key = orc_to_key(orc_zipf_next(&z), a->keyspace);
      uint64_t v;
      (void)orc_search(a->t, key, &v);
    }
    done += 256;
    *a->count = done;  /* tp[id][0] (test/benchmark.cpp:186) */
  }
  return NULL;
}

/* The reference benchmark's measured phase on `nthreads` pinned threads
 * (test/benchmark.cpp:165-188 with kReadRatio = 100): every thread draws
 * key = to_key(zipf_next()) over `keyspace` with its own generator (seed
 * seed_base + thread id) and searches it; the main thread samples the
 * threads' op counters every window_s seconds (test/benchmark.cpp:302-341)
 * and writes each window's Mops/s to win_mops[0 .. windows). */
/* The tree test/benchmark.cpp builds before its measured phase, one
 * Tree::insert at a time as the reference does (27/27 leaf splits,
 * Tree.cpp:914-968): node 0's preload to_key(i) -> 2i for i = 1..preload
 * (benchmark.cpp:269-274), then the warm-up to_key(i) -> 2i for
 * i in [1, warm_ratio * keyspace) (benchmark.cpp:114-120; the reference's
 * threads take i % T == id concurrently: one thread here takes every i in
 * order, the order a round-robin interleaving of those threads gives). */
void orc_c1_build(orc_tree *t, uint64_t keyspace, double warm_ratio, uint64_t preload) {
  for (uint64_t i = 1; i <= preload; ++i) orc_insert(t, orc_to_key(i, keyspace), i * 2);
  const uint64_t end = (uint64_t)(warm_ratio * (double)keyspace);
  for (uint64_t i = 1; i < end; ++i) orc_insert(t, orc_to_key(i, keyspace), i * 2);
}

void orc_c1_bench(orc_tree *t, int nthreads, uint64_t keyspace, double theta,
                  uint64_t seed_base, int windows, double window_s, double *win_mops) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 1024) nthreads = 1024;
  static int cpus[1024];
  const int ncpu = avail_cpus(cpus, 1024);
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
  c1_arg *args = (c1_arg *)malloc(sizeof(c1_arg) * nthreads);
  volatile uint64_t *cnt = (volatile uint64_t *)calloc((size_t)nthreads * 8, 8);
  volatile int stop = 0, ready = 0;
  t->mt = 1;
  for (int i = 0; i < nthreads; ++i) {
    args[i] = (c1_arg){t, keyspace, theta, (seed_base + (uint64_t)i) & 0xFFFFFFFFFFFFull,
                       cpus[i % ncpu], &stop, &ready, cnt + 8 * i};
    pthread_create(&th[i], NULL, c1_worker, &args[i]);
  }
  while (__atomic_load_n(&ready, __ATOMIC_ACQUIRE) < nthreads) {
  }
  uint64_t prev = 0;
  double ts = now_s();
  for (int w = 0; w < windows; ++w) {
    const double until = ts + window_s;
    while (now_s() < until) {
      struct timespec nap = {0, 2000000};
      nanosleep(&nap, NULL);
    }
    const double te = now_s();
    uint64_t all = 0;
    for (int i = 0; i < nthreads; ++i) all += cnt[8 * i];
    win_mops[w] = (double)(all - prev) / (te - ts) / 1e6;
    prev = all;
    ts = te;
  }
  __atomic_store_n(&stop, 1, __ATOMIC_RELAXED);
  for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
  t->mt = 0;
  free(th);
  free(args);
  free((void *)cnt);
}
