// shard.cpp — the multi-GPU boundary of the C-ABI: range shards over RCCL.
//
// Replaces the reference's memory-node placement (pages spread over memory
// nodes in 32 MB chunks, include/DSM.h:198-224; every Tree::search walks
// remote pages over RDMA, src/Tree.cpp:405-459) with key-range shards: rank
// r owns [r * 2^64 / P, (r+1) * 2^64 / P) and holds a complete B-link tree of
// its slice, so no page pointer crosses GPUs and a query touches one shard.
// One exchange each way per batch, over RCCL (xGMI between the GPUs of a
// node):
//
//   search : every key straight into its owner's run of fixed-capacity
//            slots (cap = 1.25 n / P + 256, kKeyMax padding; a per-peer
//            cursor places it, spos records where) -> ncclAllToAll of the
//            slots -> local batched get over all received slots (a kKeyMax
//            finds nothing) -> ncclAllToAll of the results back -> gather to
//            input order through spos (found = value != 0, Tree.cpp:445-448).
//            No count exchange, no bucketing pass and no host wait: the whole
//            routed get is queued on the stream.  A key whose run is full
//            (keys far from uniform over the shards) finds nothing and is
//            reported as kErrOverflow at the tree's next synchronising call.
//   insert : the same bucketing, the values permuted alongside, keys and
//            values exchanged, then a local insert queued without a host
//            wait; received runs arrive in source-rank order and bucketing
//            is stable, so a shard applies the union of the ranks' batches
//            in rank-major batch order (last writer wins), one valid
//            linearisation of Sherman's concurrent inserts.
//
// A search is split in two calls so a caller can pipeline batches: begin
// (bucketing + count exchange, no host wait) and end (the rest).  Each of the
// handle's two slots has its own buffers and its own communicator (split
// from the first), so a begun batch's count exchange is never queued behind
// the other slot's value exchange.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "../../include/sherman_amd.h"
#include "kernels.h"

// library-internal (tree.cpp): the tree's sticky device error word
extern "C" uint32_t* shm__error_word(shm_tree* t);

namespace {

constexpr int kSlots = 2;

struct Slot {
  ncclComm_t comm = nullptr;
  uint64_t* cnts = nullptr;   // device: send counts [P], receive counts [P]
  uint64_t* kb = nullptr;     // keys bucketed by owner
  uint64_t* vb = nullptr;     // insert values, permuted alongside
  uint32_t* perm = nullptr;   // insert: source position of kb[i]; get: slot of input i
  uint64_t* rk = nullptr;     // received keys
  uint64_t* rv = nullptr;     // received insert values / local get results
  uint64_t* back = nullptr;   // results returned to this rank (bucketed order)
  // fixed-capacity get exchange: P slots of up to pcap keys each way; a
  // batch of n uses slots of ncap = min(pcap, 1.25 n / P + 256) (every rank
  // passes the same n: the exchange is a collective)
  uint64_t pcap = 0;
  uint64_t ncap = 0;
  uint64_t* pk = nullptr;     // packed keys to send
  uint64_t* pr = nullptr;     // keys received
  uint64_t* pv = nullptr;     // local results for them
  uint64_t* pb = nullptr;     // results returned
  uint64_t cap = 0;           // send-side capacity (the local max_batch)
  uint64_t rcap = 0;          // receive-side capacity (grows)
  const uint64_t* keys = nullptr;
  uint64_t n = 0;
  hipStream_t stream = nullptr;
  bool busy = false;
};

}  // namespace

struct shm_shard {
  shm_tree* local = nullptr;
  uint32_t world = 1, rank = 0;
  bool own_comm = false;
  Slot slot[kSlots];
  int next = 0;
};

namespace {

int nccl_ok(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return SHM_OK;
  fprintf(stderr, "sherman_amd: %s failed: %s\n", what, ncclGetErrorString(r));
  return SHM_EIO;
}
#define NCCL_OK(expr)                                 \
  do {                                                \
    const int _rc = nccl_ok((expr), #expr);           \
    if (_rc) return _rc;                              \
  } while (0)
#define HIP_OK2(expr)                                 \
  do {                                                \
    if ((expr) != hipSuccess) return SHM_EIO;         \
  } while (0)

template <class T>
int dalloc(T** p, uint64_t count) {
  if (hipMalloc((void**)p, sizeof(T) * std::max<uint64_t>(count, 1)) != hipSuccess) {
    *p = nullptr;
    return SHM_ENOMEM;
  }
  return SHM_OK;
}

void free_slot(Slot& s, bool own) {
  for (void* p : {(void*)s.cnts, (void*)s.kb, (void*)s.vb, (void*)s.perm, (void*)s.rk,
                  (void*)s.rv, (void*)s.back, (void*)s.pk, (void*)s.pr, (void*)s.pv,
                  (void*)s.pb})
    if (p) (void)hipFree(p);
  if (own && s.comm) (void)ncclCommDestroy(s.comm);
  s = Slot{};
}

int alloc_slot(Slot& s, uint64_t cap, uint32_t world) {
  s.cap = cap;
  s.rcap = cap + cap / 4;
  int rc = SHM_OK;
  rc |= dalloc(&s.cnts, 2 * (uint64_t)world);
  rc |= dalloc(&s.kb, cap);
  rc |= dalloc(&s.vb, cap);
  rc |= dalloc(&s.perm, cap);
  rc |= dalloc(&s.back, cap);
  rc |= dalloc(&s.rk, s.rcap);
  rc |= dalloc(&s.rv, s.rcap);
  // a peer's share of a uniform batch is cap / P; 25 % + 256 of slack
  s.pcap = world == 1 ? cap : std::min<uint64_t>(cap, (cap + cap / 4) / world + 256);
  const uint64_t slots = (uint64_t)world * s.pcap;
  rc |= dalloc(&s.pk, slots);
  rc |= dalloc(&s.pr, slots);
  rc |= dalloc(&s.pv, slots);
  rc |= dalloc(&s.pb, slots);
  return rc ? SHM_ENOMEM : SHM_OK;
}

// receive buffers for `need` keys (rare regrowth: waits for the slot's stream)
int ensure_recv(Slot& s, uint64_t need) {
  if (need <= s.rcap) return SHM_OK;
  HIP_OK2(hipStreamSynchronize(s.stream));
  (void)hipFree(s.rk);
  (void)hipFree(s.rv);
  s.rk = s.rv = nullptr;
  s.rcap = need + need / 4;
  if (dalloc(&s.rk, s.rcap) || dalloc(&s.rv, s.rcap)) return SHM_ENOMEM;
  return SHM_OK;
}

// bucket the slot's keys by owner and exchange the per-peer counts
int begin(shm_shard* h, Slot& s) {
  const uint32_t P = h->world;
  int rc = shm_route_bucket(h->local, s.keys, s.n, P, s.cnts, s.kb, s.perm, s.stream);
  if (rc) return rc;
  NCCL_OK(ncclAllToAll(s.cnts, s.cnts + P, 1, ncclUint64, s.comm, s.stream));
  return SHM_OK;
}

// both count vectors on the host (one zero-copy read-back); offsets
int counts(shm_shard* h, Slot& s, std::vector<uint64_t>& cnt, std::vector<uint64_t>& rcnt,
           std::vector<uint64_t>& soff, std::vector<uint64_t>& roff, uint64_t* nrecv) {
  const uint32_t P = h->world;
  std::vector<uint64_t> both(2 * P);
  const int rc = shm_read_words(h->local, s.cnts, 16ull * P, both.data(), s.stream);
  if (rc) return rc;
  cnt.assign(both.begin(), both.begin() + P);
  rcnt.assign(both.begin() + P, both.end());
  soff.assign(P + 1, 0);
  roff.assign(P + 1, 0);
  for (uint32_t p = 0; p < P; ++p) {
    soff[p + 1] = soff[p] + cnt[p];
    roff[p + 1] = roff[p] + rcnt[p];
  }
  *nrecv = roff[P];
  return SHM_OK;
}

// grouped point-to-point exchange: send[p] (cnt) -> peer p, recv[p] (rcnt) <- peer p
int exchange(shm_shard* h, Slot& s, const uint64_t* send, const std::vector<uint64_t>& cnt,
             const std::vector<uint64_t>& soff, uint64_t* recv,
             const std::vector<uint64_t>& rcnt, const std::vector<uint64_t>& roff) {
  NCCL_OK(ncclGroupStart());
  for (uint32_t p = 0; p < h->world; ++p) {
    if (cnt[p]) NCCL_OK(ncclSend(send + soff[p], cnt[p], ncclUint64, (int)p, s.comm, s.stream));
    if (rcnt[p]) NCCL_OK(ncclRecv(recv + roff[p], rcnt[p], ncclUint64, (int)p, s.comm, s.stream));
  }
  NCCL_OK(ncclGroupEnd());
  return SHM_OK;
}

int make_shard(shm_tree* local, ncclComm_t comm, uint32_t world, uint32_t rank, bool own,
               shm_shard** out) {
  shm_shard* h = new shm_shard();
  h->local = local;
  h->world = world;
  h->rank = rank;
  h->own_comm = own;
  h->slot[0].comm = comm;
  // a second communicator for the second slot, split from the first (same
  // ranks, same order) so the two slots' collectives never serialise
  ncclComm_t c2 = nullptr;
  if (nccl_ok(ncclCommSplit(comm, 0, (int)rank, &c2, nullptr), "ncclCommSplit") || !c2) {
    delete h;
    return SHM_EIO;
  }
  h->slot[1].comm = c2;
  // the send side holds at most one max_batch chunk of the local tree
  const uint64_t cap = shm_tree_max_batch(local);
  for (int i = 0; i < kSlots; ++i) {
    if (alloc_slot(h->slot[i], cap, world)) {
      for (int j = 0; j < kSlots; ++j) free_slot(h->slot[j], j > 0 || own);
      delete h;
      return SHM_ENOMEM;
    }
  }
  *out = h;
  return SHM_OK;
}

}  // namespace

extern "C" {

int shm_nccl_unique_id(void* id_out, uint64_t bytes) {
  if (!id_out || bytes < sizeof(ncclUniqueId)) return SHM_EINVAL;
  ncclUniqueId id;
  NCCL_OK(ncclGetUniqueId(&id));
  memcpy(id_out, &id, sizeof(id));
  return SHM_OK;
}

int shm_shard_create(shm_tree* local, const void* nccl_id, uint64_t id_bytes, uint32_t world,
                     uint32_t rank, shm_shard** out) {
  if (!local || !nccl_id || id_bytes < sizeof(ncclUniqueId) || !out || world == 0 ||
      world > 16 || rank >= world)
    return SHM_EINVAL;
  ncclUniqueId id;
  memcpy(&id, nccl_id, sizeof(id));
  ncclComm_t comm = nullptr;
  NCCL_OK(ncclCommInitRank(&comm, (int)world, id, (int)rank));
  const int rc = make_shard(local, comm, world, rank, true, out);
  if (rc) (void)ncclCommDestroy(comm);
  return rc;
}

int shm_shard_create_with_comm(shm_tree* local, void* nccl_comm, uint32_t world, uint32_t rank,
                               shm_shard** out) {
  if (!local || !nccl_comm || !out || world == 0 || world > 16 || rank >= world)
    return SHM_EINVAL;
  return make_shard(local, (ncclComm_t)nccl_comm, world, rank, false, out);
}

int shm_shard_destroy(shm_shard* h) {
  if (!h) return SHM_EINVAL;
  (void)hipDeviceSynchronize();
  for (int i = 0; i < kSlots; ++i) free_slot(h->slot[i], i > 0 || h->own_comm);
  delete h;
  return SHM_OK;
}

int shm_shard_search_begin(shm_shard* h, const uint64_t* keys, uint64_t n, void* stream,
                           uint32_t* ticket) {
  if (!h || !ticket || (n && !keys)) return SHM_EINVAL;
  const int i = h->next;
  Slot& s = h->slot[i];
  if (s.busy) return SHM_EINVAL;  // end the slot's batch first
  if (n > s.cap) return SHM_E2BIG;
  h->next = (i + 1) % kSlots;
  s.keys = keys;
  s.n = n;
  s.stream = (hipStream_t)stream;
  s.busy = true;
  *ticket = (uint32_t)i;
  const uint32_t P = h->world;
  s.ncap = P == 1 ? n : std::min<uint64_t>(s.pcap, (n + n / 4) / P + 256);
  shm::dev::launch_route_slots(s.keys, s.n, P, s.ncap, reinterpret_cast<uint32_t*>(s.cnts), s.pk,
                               s.perm, shm__error_word(h->local), s.stream);
  int rc = hipGetLastError() == hipSuccess ? SHM_OK : SHM_EIO;
  if (rc == SHM_OK)
    rc = nccl_ok(ncclAllToAll(s.pk, s.pr, s.ncap, ncclUint64, s.comm, s.stream),
                 "ncclAllToAll(keys)");
  if (rc) s.busy = false;
  return rc;
}

int shm_shard_search_end(shm_shard* h, uint32_t ticket, uint64_t* vals_out, uint8_t* found_out) {
  if (!h || ticket >= (uint32_t)kSlots || !h->slot[ticket].busy) return SHM_EINVAL;
  Slot& s = h->slot[ticket];
  if (s.n && (!vals_out || !found_out)) return SHM_EINVAL;
  s.busy = false;
  const uint32_t P = h->world;
  int rc = shm_search_batch(h->local, s.pr, (uint64_t)P * s.ncap, s.pv, nullptr, s.stream);
  if (rc) return rc;
  // the results go back the way the keys came, slot for slot
  NCCL_OK(ncclAllToAll(s.pv, s.pb, s.ncap, ncclUint64, s.comm, s.stream));
  shm::dev::launch_route_gather(s.pb, s.perm, s.n, vals_out, found_out, s.stream);
  return hipGetLastError() == hipSuccess ? SHM_OK : SHM_EIO;
}

int shm_shard_search(shm_shard* h, const uint64_t* keys, uint64_t n, uint64_t* vals_out,
                     uint8_t* found_out, void* stream) {
  uint32_t ticket = 0;
  const int rc = shm_shard_search_begin(h, keys, n, stream, &ticket);
  if (rc) return rc;
  return shm_shard_search_end(h, ticket, vals_out, found_out);
}

int shm_shard_insert(shm_shard* h, const uint64_t* keys, const uint64_t* vals, uint64_t n,
                     void* stream) {
  if (!h || (n && (!keys || !vals))) return SHM_EINVAL;
  const int i = h->next;
  Slot& s = h->slot[i];
  if (s.busy) return SHM_EINVAL;
  if (n > s.cap) return SHM_E2BIG;
  h->next = (i + 1) % kSlots;
  s.keys = keys;
  s.n = n;
  s.stream = (hipStream_t)stream;
  int rc = begin(h, s);
  if (rc) return rc;
  if ((rc = shm_route_permute(h->local, vals, s.perm, n, s.vb, s.stream))) return rc;
  std::vector<uint64_t> cnt, rcnt, soff, roff;
  uint64_t nrecv = 0;
  if ((rc = counts(h, s, cnt, rcnt, soff, roff, &nrecv))) return rc;
  if ((rc = ensure_recv(s, nrecv))) return rc;
  if ((rc = exchange(h, s, s.kb, cnt, soff, s.rk, rcnt, roff))) return rc;
  if ((rc = exchange(h, s, s.vb, cnt, soff, s.rv, rcnt, roff))) return rc;
  return shm_insert_batch_async(h->local, s.rk, s.rv, nrecv, s.stream);
}

// Library-internal test hooks, not part of include/sherman_amd.h: the routed
// get's slot placement and result gather for P shards, so the P > 1 path can
// be checked on one GPU (tests/test_gpu_shard.py) without P ranks.  cursor:
// P u32 of device scratch; the overflow bit goes to t's error word.
int shm__route_slots(shm_tree* t, const uint64_t* keys, uint64_t n, uint32_t P, uint64_t cap,
                     uint32_t* cursor, uint64_t* slots, uint32_t* spos, void* stream) {
  if (!t || !cursor || !slots || !spos || P == 0 || P > 64 || (n && !keys) ||
      (uint64_t)P * cap >= ~0u)
    return SHM_EINVAL;
  shm::dev::launch_route_slots(keys, n, P, cap, cursor, slots, spos, shm__error_word(t),
                               (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? SHM_OK : SHM_EIO;
}
int shm__route_gather(const uint64_t* in, const uint32_t* spos, uint64_t n, uint64_t* vals_out,
                      uint8_t* found_out, void* stream) {
  if (n && (!in || !spos || !vals_out)) return SHM_EINVAL;
  shm::dev::launch_route_gather(in, spos, n, vals_out, found_out, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? SHM_OK : SHM_EIO;
}

}  // extern "C"
