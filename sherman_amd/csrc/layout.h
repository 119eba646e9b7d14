// layout.h — Sherman page layout, constants and GlobalAddress, shared by the
// HIP kernels and the host runtime.  Byte offsets restate the packed C++ layout
// of include/Tree.h:130-336 (probe-verified in SURVEY.md Appendix A); they are
// spelled out as offsets because the kernels move whole 1 KB pages through
// registers/LDS and never materialise the packed structs.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SHM_HD __host__ __device__ __forceinline__
#else
#define SHM_HD inline
#endif

namespace shm {

// include/Common.h:113-121
constexpr uint64_t kKeyMin = 0;
constexpr uint64_t kKeyMax = ~0ull;
constexpr uint64_t kValueNull = 0;
constexpr uint32_t kPageSize = 1024;  // kInternalPageSize == kLeafPageSize

// include/Tree.h:189-195
constexpr int kInternalCardinality = 61;
constexpr int kLeafCardinality = 54;
constexpr int kMaxLevelOfTree = 7;  // include/Common.h:96

// Batched multi-way split targets (reference splits one page at a time at
// exactly 54 / 61 and leaves halves of 27 / 30, src/Tree.cpp:939, 779).  A
// batch may overflow a page by many entries; it is then cut into
// ceil(T / fill) pages so a 54-entry overflow still yields 27 + 27.
constexpr int kLeafSplitFill = 36;      // entries per leaf after a k-way split
constexpr int kInternalSplitFill = 40;  // records per internal page

// byte offsets inside a page (Tree.h:197-336)
constexpr int kOffLock = 0;        // union {crc, embedding_lock, freq}
constexpr int kOffFrontVer = 8;    // front_version
constexpr int kOffLeftmost = 9;    // Header.leftmost_ptr
constexpr int kOffSibling = 17;    // Header.sibling_ptr
constexpr int kOffLevel = 25;      // Header.level
constexpr int kOffLastIndex = 26;  // Header.last_index (int16)
constexpr int kOffLowest = 28;     // Header.lowest
constexpr int kOffHighest = 36;    // Header.highest
constexpr int kOffRecords = 44;    // records[]
constexpr int kOffInternalRear = 1020;
constexpr int kOffLeafRear = 1016;
constexpr int kInternalEntry = 16;  // {key, ptr}
constexpr int kLeafEntry = 18;      // {f:4, key, value, r:4}

static_assert(kOffRecords + kInternalCardinality * kInternalEntry ==
                  kOffInternalRear,
              "internal layout");
static_assert(kOffRecords + kLeafCardinality * kLeafEntry == kOffLeafRear,
              "leaf layout");

// Per-page occupancy bound (a side array, not part of the page bytes): for a
// leaf, every slot >= hw holds value 0 (empty, Tree.cpp:881), so a reader may
// stop its page read after slot hw - 1.  kLeafHwFull = unknown (internal
// pages, pages of a loaded image): read the whole page.
constexpr uint8_t kLeafHwFull = 0xFF;
// 16 B lanes of a page DMA covering the header and slots [0, hw); the last
// lane (rear_version, byte 1016) is loaded as well
SHM_HD int hw_dma_lanes(uint32_t hw) {
  return hw >= (uint32_t)kLeafCardinality ? 64 : (kOffRecords + kLeafEntry * (int)hw + 15) / 16;
}

// Leaf summary (a side line per arena page, 64 B, not part of the page
// bytes): what a get needs of a leaf in one HBM request instead of the
// page's 1 KB.  The highest fence (u64) at 0; byte 8 = kSumLeaf while the
// line describes the current leaf (0 for internal pages and pages never
// written as leaves); fp[slot] (u8) at 9 + slot = key_fp of the slot's key for
// a valid slot (value != 0), 0 for an empty one.  A get reads the line, turns
// right on k >= highest (the sibling from the page header: a stale start,
// rare), and reads only the entries whose fp matches (false positives
// ~ 40 / 255 per leaf).  Every leaf writer keeps the line.  At 64 B per page
// the lines of a 2^26-key shard (119 MB) and its leaf directory (64 MB) fit
// the 256 MB Infinity Cache together.
constexpr uint32_t kSumBytes = 64;
constexpr uint32_t kSumOffHighest = 0;
constexpr uint32_t kSumOffTag = 8;
constexpr uint32_t kSumOffFp = 9;
constexpr uint8_t kSumLeaf = 0xA5;
static_assert(kSumOffFp + kLeafCardinality <= kSumBytes, "summary line");
// leaf directory entries (leafdir.hip): 64 B = kDirWords u64 each; count
// word flag: the entry is in fingerprint form (device_common.h dir_fp_cand)
constexpr uint64_t kDirWords = 8;
constexpr uint32_t kDirFp = 0x100u;
// pair form (a read phase's build, leafdir.hip k_dir_pairs): the leaf list
// of the first 32 B stays valid, and bytes 32..63 list up to kDirPairMax
// (fingerprint, slot | leaf << 6) u16 pairs of the keys inside the prefix;
// the pair count in bits 16..23 of the count word; kDirPairsBad: a key of
// the prefix was found in a leaf the list does not name (not usable)
constexpr uint32_t kDirPairs = 0x200u;
constexpr uint32_t kDirPairsBad = 0x400u;
constexpr uint32_t kDirPairMax = 16;
// count word flag: an insert chunk's writer listed the entry for repair
// after the chunk (dir_upkeep.h, leafdir.hip k_dir_repair); the walks ignore it
constexpr uint32_t kDirFix = 0x800u;
SHM_HD uint32_t key_fp(uint64_t k) {
  const uint32_t f = (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> 56);
  return f ? f : 1u;
}

// GlobalAddress{nodeID:16, offset:48} (include/GlobalAddress.h:7-16).
// nodeID = GPU / shard id, offset = byte offset into that GPU's page arena.
SHM_HD uint64_t ga_make(uint16_t node, uint64_t off) {
  return (uint64_t)node | (off << 16);
}
SHM_HD uint64_t ga_offset(uint64_t ga) { return ga >> 16; }
SHM_HD uint16_t ga_node(uint64_t ga) { return (uint16_t)(ga & 0xFFFF); }
// leaf-directory page index <-> GlobalAddress (1 KB pages, offset < 4 TB)
SHM_HD uint64_t dir_page_ga(uint32_t pg, uint16_t node) {
  return ((uint64_t)pg << 26) | (uint64_t)node;
}
SHM_HD uint32_t dir_page_index(uint64_t ga) { return (uint32_t)(ga_offset(ga) >> 10); }

// Superblock in page 0 of the arena (offset 0 is Null, like chunk 0 in
// GlobalAllocator.h:24-26); it plays the role of root_ptr_ptr
// (src/Tree.cpp:90-97) and of the Directory's g_root_ptr / g_root_level
// (src/Directory.cpp:72-79).
struct Superblock {
  uint64_t magic;
  uint64_t root_ptr;
  uint64_t root_level;
  uint64_t next_page;  // bump allocator, in pages (page 0 = superblock)
  uint64_t capacity_pages;
  uint64_t node_id;
  uint64_t batches;
  uint64_t splits;
};
constexpr uint64_t kSuperMagic = 0x5348524d414d4431ull;  // "SHRMAMD1"

// device error bits (word 0 of the tree's error block; word 1 = the tag of
// the first insert chunk that saw a bit other than kErrKeyMax, tree.cpp
// check_err).  Every bound that can stop a kernel has a bit of its own, so a
// record names the kernel that hit it.
constexpr uint32_t kErrBadPtr = 1u << 0;       // pointer outside arena / node
constexpr uint32_t kErrInconsistent = 1u << 1; // version mismatch persisted
constexpr uint32_t kErrRounds = 1u << 2;       // k_upper: a parent / delete walk did not converge
constexpr uint32_t kErrFence = 1u << 3;        // k < lowest on a walk
constexpr uint32_t kErrLock = 1u << 4;         // lock spin bound exceeded
constexpr uint32_t kErrPlan = 1u << 5;         // page changed between plan/apply
constexpr uint32_t kErrOverflow = 1u << 6;     // page overfull at apply
constexpr uint32_t kErrNoMem = 1u << 7;        // page arena exhausted (splits left unapplied)
constexpr uint32_t kErrHandoff = 1u << 8;      // k_upper: a phase hand-off wait timed out
                                               // (the chunk's levels / deletes resume later)
constexpr uint32_t kErrSegSpin = 1u << 9;      // retired (k_seg_fill counts a late tile itself)
constexpr uint32_t kErrScanSpin = 1u << 10;    // k_scan_u64: look-back spin bound
constexpr uint32_t kErrBinSpin = 1u << 11;     // k_bin_unique: look-back spin bound
constexpr uint32_t kErrGetHops = 1u << 12;     // a get walk (k_get / k_get_sum) hop bound
constexpr uint32_t kErrLocateHops = 1u << 13;  // k_locate: walk hop bound
constexpr uint32_t kErrFanIn = 1u << 14;       // k_upper: a large split's fan-in wait bound

// CityHash64 v1.1 (google/cityhash, city.cc HashLen0to16 for len == 8).
// Third-party dependency of the reference (script/installLibs.sh:16-20, HEAD,
// unpinned); used by to_key (test/benchmark.cpp:43-46) and the lock index
// (src/Tree.cpp:832-833).
SHM_HD uint64_t rot64(uint64_t v, int s) {
  return s == 0 ? v : ((v >> s) | (v << (64 - s)));
}
SHM_HD uint64_t cityhash64_u64(uint64_t x) {
  const uint64_t k2 = 0x9ae16a3b2f90404full;
  const uint64_t len = 8;
  const uint64_t mul = k2 + len * 2;
  const uint64_t a = x + k2;
  const uint64_t b = x;  // Fetch64(s + len - 8) == Fetch64(s)
  const uint64_t c = rot64(b, 37) * mul + a;
  const uint64_t d = (rot64(a, 25) + b) * mul;
  uint64_t h = (c ^ d) * mul;  // HashLen16(c, d, mul)
  h ^= (h >> 47);
  uint64_t g = (d ^ h) * mul;
  g ^= (g >> 47);
  g *= mul;
  return g;
}

}  // namespace shm
