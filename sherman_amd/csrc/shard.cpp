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
//            cursor places it, spos records where; this rank's own run is
//            placed straight into its receive slot) -> grouped ncclSend /
//            ncclRecv of the P - 1 peers' runs and key counts (nothing at
//            P = 1) -> local batched get over all received slots (a kKeyMax
//            finds nothing) -> the peers' results back the same way ->
//            gather to input order through spos, the own run's results
//            read in place (found = value != 0, Tree.cpp:445-448).  No host wait before the key
//            exchange.  A run longer than its slot (keys far from uniform
//            over the shards, e.g. a zipf hot key) puts the rest of its keys
//            on an overflow list; end() reads the key counts back once (they
//            are ready as soon as the key exchange is), and where a count
//            passed the slot both sides know it and run a second, exact
//            round: grouped ncclSend / ncclRecv of the cut keys, a local get,
//            the values back and scattered to their inputs.  No lookup is
//            ever dropped (Tree::search always answers, Tree.cpp:405-459).
//   insert : stable bucketing by owner, the values permuted alongside, each
//            owner's run packed into a slot of max_batch / P (kKeyMax
//            padding), keys / values / counts exchanged, then the received
//            slots queued as one local insert that skips the padding: no
//            host wait (a batch holding kKeyMax routes nothing and reports
//            SHM_EINVAL, as a local insert rejects its chunk).  Received
//            slots arrive in source-rank order and the bucketing is stable,
//            so the slots apply in rank-major batch order.  A run longer
//            than its slot keeps its tail, which the next call on the shard
//            (or shm_shard_synchronize) sends in an exact second round and
//            applies before anything else; each rank's ops stay in its own
//            order, but a tail applies after every rank's slots, so across
//            ranks the result is one valid linearisation of the ranks'
//            concurrent batches (Sherman's clients are not ordered either),
//            not strict rank-major order.
//   range  : scan j's overlap with shard p is piece (p, j) of a P x n_cap
//            matrix (empty where it misses the shard); row p goes to rank p
//            (ncclAllToAll, no count exchange), the owner scans the pieces
//            (count, offsets, staged fill), the counts come back, and ONE
//            read-back of the per-peer value totals sizes the grouped
//            ncclSend / ncclRecv of the values; scan j's values are its
//            pieces' values in shard order = key order (Tree::range_query,
//            Tree.cpp:461-540, intended semantics).
//
// A search is split in two calls so a caller can pipeline batches: begin
// (placement + key exchange) and end (the rest).  Each of the handle's two
// search slots has its own buffers and its own communicator (split from the
// first), so a begun batch's key exchange is never queued behind the other
// slot's value exchange; inserts and range scans use a third communicator
// and buffers of their own.
//
// The transport is an interface: RCCL (one process per GPU, the product
// path), or an in-process group of P handles on one GPU whose collectives are
// device copies between the ranks' buffers (library-internal test hook: the
// routing logic above at P = 8 on the one GPU of a test box).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <vector>

#include "../../include/sherman_amd.h"
#include "kernels.h"

// library-internal (tree.cpp)
extern "C" uint32_t* shm__error_word(shm_tree* t);
extern "C" int shm__insert_batch_padded(shm_tree* t, const uint64_t* keys, const uint64_t* vals,
                                        uint64_t n, void* stream);
extern "C" int shm__route_bucket_insert(shm_tree* t, const uint64_t* keys, uint64_t n,
                                        uint32_t num_shards, uint64_t* counts_out,
                                        uint64_t* keys_out, uint32_t* perm_out, void* stream);
extern "C" int shm__scan_u64(shm_tree* t, const uint64_t* in, uint64_t* out, uint64_t n,
                             uint64_t* tot_dev, void* stream);

namespace {

// A routed get's slot per peer: n / P + 6 sigma of the binomial count of
// keys a peer gets from n uniform (hashed) keys, + 256.  Past it a run's
// tail takes the exact overflow round (get_overflow), so a skewed batch is
// slower, never wrong; at C4's 2^20 keys and P = 8 the slots carry 1.9 %
// padding where 1.25 n / P + 256 carried 25 % (fewer bytes over xGMI, fewer
// padding lanes in the walk).
uint64_t get_slot_cap(uint64_t n, uint32_t P) {
  const uint64_t m = n / P;
  return m + 6 * (uint64_t)std::sqrt((double)m) + 256;
}


constexpr uint32_t kMaxWorld = 16;

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
#define RC_OK(expr)                                   \
  do {                                                \
    const int _rc = (expr);                           \
    if (_rc) return _rc;                              \
  } while (0)

template <class T>
int dalloc(T** p, uint64_t count) {
  if (hipMalloc((void**)p, sizeof(T) * std::max<uint64_t>(count, 1)) != hipSuccess) {
    *p = nullptr;
    return SHM_ENOMEM;
  }
  return SHM_OK;
}
template <class T>
void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}
// grow a device buffer to >= need elements (waits for the stream first)
template <class T>
int ensure(T*& p, uint64_t& cap, uint64_t need, hipStream_t s) {
  if (need <= cap && p) return SHM_OK;
  HIP_OK2(hipStreamSynchronize(s));
  dfree(p);
  cap = need + need / 4 + 1024;
  return dalloc(&p, cap);
}

// ---- transports ---------------------------------------------------------------
struct Xport {
  uint32_t P = 1, rank = 0;
  // a2a_peers also exchanges this rank's own part with itself (shm__shard_
  // force_route: a world-1 shard's routed path through the transport)
  bool self_too = false;
  virtual ~Xport() = default;
  virtual int group_start() { return SHM_OK; }
  virtual int group_end() { return SHM_OK; }
  // `count` elements of eb (4 or 8) bytes to and from every peer: peer p's
  // part of send / recv at p * count
  virtual int a2a(const void* send, void* recv, uint64_t count, int eb, hipStream_t s) = 0;
  // a2a without this rank's own part (it never leaves the rank: the callers
  // place it straight where the local kernel reads it); nothing at P = 1
  virtual int a2a_peers(const void* send, void* recv, uint64_t count, int eb, hipStream_t s) = 0;
  // grouped point-to-point: scnt[p] elements at send + soff[p] to peer p,
  // rcnt[p] elements from peer p to recv + roff[p] (both sides know both)
  virtual int p2p(const void* send, const uint64_t* scnt, const uint64_t* soff, void* recv,
                  const uint64_t* rcnt, const uint64_t* roff, int eb, hipStream_t s) = 0;
};

ncclDataType_t nccl_type(int eb) { return eb == 8 ? ncclUint64 : ncclUint32; }

struct RcclXport : Xport {
  ncclComm_t comm = nullptr;
  bool own = false;
  ~RcclXport() override {
    if (own && comm) (void)ncclCommDestroy(comm);
  }
  int group_start() override { return nccl_ok(ncclGroupStart(), "ncclGroupStart"); }
  int group_end() override { return nccl_ok(ncclGroupEnd(), "ncclGroupEnd"); }
  int a2a(const void* send, void* recv, uint64_t count, int eb, hipStream_t s) override {
    return nccl_ok(ncclAllToAll(send, recv, count, nccl_type(eb), comm, s), "ncclAllToAll");
  }
  int a2a_peers(const void* send, void* recv, uint64_t count, int eb, hipStream_t s) override {
    if ((P == 1 && !self_too) || count == 0) return SHM_OK;
    NCCL_OK(ncclGroupStart());
    for (uint32_t p = 0; p < P; ++p) {
      if (p == rank && !self_too) continue;
      NCCL_OK(ncclSend(static_cast<const char*>(send) + (uint64_t)p * count * eb, count,
                       nccl_type(eb), (int)p, comm, s));
      NCCL_OK(ncclRecv(static_cast<char*>(recv) + (uint64_t)p * count * eb, count, nccl_type(eb),
                       (int)p, comm, s));
    }
    NCCL_OK(ncclGroupEnd());
    return SHM_OK;
  }
  int p2p(const void* send, const uint64_t* scnt, const uint64_t* soff, void* recv,
          const uint64_t* rcnt, const uint64_t* roff, int eb, hipStream_t s) override {
    NCCL_OK(ncclGroupStart());
    for (uint32_t p = 0; p < P; ++p) {
      if (scnt[p])
        NCCL_OK(ncclSend(static_cast<const char*>(send) + soff[p] * eb, scnt[p], nccl_type(eb),
                         (int)p, comm, s));
      if (rcnt[p])
        NCCL_OK(ncclRecv(static_cast<char*>(recv) + roff[p] * eb, rcnt[p], nccl_type(eb), (int)p,
                         comm, s));
    }
    NCCL_OK(ncclGroupEnd());
    return SHM_OK;
  }
};

// In-process group of P ranks on one device, each driven by its own host
// thread (test hook).  A collective: every rank posts its buffers and an
// event recorded after their producers, a host barrier, every rank copies
// its parts out of the peers' send buffers on its stream (after their
// events), a barrier, every rank's stream waits for the peers' copies before
// its send buffer may change, a barrier before the posts are reused.
struct LocalGroup {
  uint32_t P;
  std::mutex mu;
  std::condition_variable cv;
  uint64_t gen = 0;
  uint32_t arrived = 0;
  struct Post {
    const char* send = nullptr;
    const uint64_t* scnt = nullptr;
    const uint64_t* soff = nullptr;
    uint64_t count = 0;
    hipEvent_t ready = nullptr, done = nullptr;
  };
  std::vector<Post> post;
  // point-to-point mailboxes [src * P + dst]: only the pairs with data meet
  // (as ncclSend / ncclRecv), so a rank with nothing to exchange skips it
  struct Mail {
    const char* send = nullptr;
    uint64_t bytes = 0;
    hipEvent_t ready = nullptr;  // sender: its data produced
    hipEvent_t done = nullptr;   // receiver: its copy queued
    int state = 0;               // 0 empty, 1 posted, 2 consumed
  };
  std::vector<Mail> mail;
  explicit LocalGroup(uint32_t p) : P(p), post(p), mail((size_t)p * p) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t g = gen;
    if (++arrived == P) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

struct LocalXport : Xport {
  LocalGroup* g = nullptr;
  hipEvent_t ready = nullptr, done = nullptr;
  std::vector<hipEvent_t> sev, rev;  // per peer: p2p send-ready / receive-done
  ~LocalXport() override {
    if (ready) (void)hipEventDestroy(ready);
    if (done) (void)hipEventDestroy(done);
    for (hipEvent_t e : sev) (void)hipEventDestroy(e);
    for (hipEvent_t e : rev) (void)hipEventDestroy(e);
  }
  int init() {
    HIP_OK2(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    HIP_OK2(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    sev.assign(g->P, nullptr);
    rev.assign(g->P, nullptr);
    for (uint32_t p = 0; p < g->P; ++p) {
      HIP_OK2(hipEventCreateWithFlags(&sev[p], hipEventDisableTiming));
      HIP_OK2(hipEventCreateWithFlags(&rev[p], hipEventDisableTiming));
    }
    return SHM_OK;
  }
  // copy(p) enqueues the part from peer p; then the hand-back protocol
  template <class F>
  int run(const LocalGroup::Post& mine, hipStream_t s, F copy) {
    int rc = SHM_OK;
    if (hipEventRecord(ready, s) != hipSuccess) rc = SHM_EIO;
    LocalGroup::Post m = mine;
    m.ready = ready;
    m.done = done;
    g->post[rank] = m;
    g->barrier();
    for (uint32_t p = 0; p < P; ++p) {
      if (hipStreamWaitEvent(s, g->post[p].ready, 0) != hipSuccess) rc = SHM_EIO;
      if (copy(p, g->post[p])) rc = SHM_EIO;
    }
    if (hipEventRecord(done, s) != hipSuccess) rc = SHM_EIO;
    g->barrier();
    for (uint32_t p = 0; p < P; ++p)
      if (hipStreamWaitEvent(s, g->post[p].done, 0) != hipSuccess) rc = SHM_EIO;
    g->barrier();
    return rc;
  }
  int a2a(const void* send, void* recv, uint64_t count, int eb, hipStream_t s) override {
    LocalGroup::Post m;
    m.send = static_cast<const char*>(send);
    m.count = count;
    return run(m, s, [&](uint32_t p, const LocalGroup::Post& q) {
      if (!count) return 0;
      return hipMemcpyAsync(static_cast<char*>(recv) + (uint64_t)p * count * eb,
                            q.send + (uint64_t)rank * count * eb, count * eb,
                            hipMemcpyDeviceToDevice, s) != hipSuccess ? 1 : 0;
    });
  }
  int a2a_peers(const void* send, void* recv, uint64_t count, int eb, hipStream_t s) override {
    LocalGroup::Post m;
    m.send = static_cast<const char*>(send);
    m.count = count;
    return run(m, s, [&](uint32_t p, const LocalGroup::Post& q) {
      if (!count || (p == rank && !self_too)) return 0;
      return hipMemcpyAsync(static_cast<char*>(recv) + (uint64_t)p * count * eb,
                            q.send + (uint64_t)rank * count * eb, count * eb,
                            hipMemcpyDeviceToDevice, s) != hipSuccess ? 1 : 0;
    });
  }
  // post every send, take every receive, then wait until the sends were taken
  // (no rank blocks before all of its sends are posted: no cycle)
  int p2p(const void* send, const uint64_t* scnt, const uint64_t* soff, void* recv,
          const uint64_t* rcnt, const uint64_t* roff, int eb, hipStream_t s) override {
    const uint32_t P = g->P;
    int rc = SHM_OK;
    std::unique_lock<std::mutex> lk(g->mu);
    for (uint32_t p = 0; p < P; ++p) {
      if (!scnt[p]) continue;
      LocalGroup::Mail& m = g->mail[(size_t)rank * P + p];
      g->cv.wait(lk, [&] { return m.state == 0; });
      if (hipEventRecord(sev[p], s) != hipSuccess) rc = SHM_EIO;
      m.send = static_cast<const char*>(send) + soff[p] * eb;
      m.bytes = scnt[p] * eb;
      m.ready = sev[p];
      m.state = 1;
    }
    g->cv.notify_all();
    for (uint32_t p = 0; p < P; ++p) {
      if (!rcnt[p]) continue;
      LocalGroup::Mail& m = g->mail[(size_t)p * P + rank];
      g->cv.wait(lk, [&] { return m.state == 1; });
      if (m.bytes != rcnt[p] * eb) rc = SHM_EIO;  // the two sides disagree on a count
      if (hipStreamWaitEvent(s, m.ready, 0) != hipSuccess ||
          hipMemcpyAsync(static_cast<char*>(recv) + roff[p] * eb, m.send,
                         std::min<uint64_t>(m.bytes, rcnt[p] * eb), hipMemcpyDeviceToDevice,
                         s) != hipSuccess ||
          hipEventRecord(rev[p], s) != hipSuccess)
        rc = SHM_EIO;
      m.done = rev[p];
      m.state = 2;
      g->cv.notify_all();
    }
    for (uint32_t p = 0; p < P; ++p) {
      if (!scnt[p]) continue;
      LocalGroup::Mail& m = g->mail[(size_t)rank * P + p];
      g->cv.wait(lk, [&] { return m.state == 2; });
      // the receiver's copy out of our buffer precedes anything we queue next
      if (hipStreamWaitEvent(s, m.done, 0) != hipSuccess) rc = SHM_EIO;
      m.state = 0;
    }
    g->cv.notify_all();
    return rc;
  }
};

// ---- per-context state ------------------------------------------------------------
// a search slot: one routed get in flight
struct GetSlot {
  Xport* x = nullptr;
  uint64_t pcap = 0;          // slot capacity per peer (allocated)
  uint64_t ncap = 0;          // this batch's: min(pcap, get_slot_cap(n, P))
  uint32_t* cw = nullptr;     // [P] keys routed to each peer, [P] overflow count, [P + 1 ..] received counts
  uint32_t* ctr = nullptr;    // the placement's claim words (route_ctr_words), zero at rest
  uint64_t filled = 0;        // the capacity the runs were last padded at (0: never)
  uint64_t *pk = nullptr, *pr = nullptr, *pv = nullptr, *pb = nullptr;  // P * pcap
  uint32_t* spos = nullptr;   // input -> slot
  uint64_t* ovk = nullptr;    // overflow list: keys, their inputs
  uint32_t* ovi = nullptr;
  uint64_t* ocnt = nullptr;   // overflow round: bucket counts [P], keys by owner, permutation, results
  uint64_t* okb = nullptr;
  uint32_t* operm = nullptr;
  uint64_t* ores = nullptr;
  uint64_t *ork = nullptr, *orv = nullptr;  // received overflow keys / their values
  uint64_t orcap = 0, orvcap = 0;
  hipEvent_t ev_keys = nullptr;
  const uint64_t* keys = nullptr;
  uint64_t n = 0;
  hipStream_t stream = nullptr;
  bool busy = false;
};

// inserts and range scans (exclusive calls on the tree)
struct ExclCtx {
  Xport* x = nullptr;
  uint64_t icap = 0;          // insert slot per peer: max_batch / P
  uint64_t* icnt = nullptr;   // bucket counts: [P] sent, [P] received
  uint64_t *kb = nullptr, *vb = nullptr;
  uint32_t* perm = nullptr;
  uint64_t *pk = nullptr, *pv = nullptr, *rk = nullptr, *rv = nullptr;  // P * icap
  uint64_t *ork = nullptr, *orv = nullptr;  // overflow tails received
  uint64_t orcap = 0, orvcap = 0;
  hipEvent_t ev_ins = nullptr;
  bool pending = false;       // an insert whose overflow check is still due
  hipStream_t pstream = nullptr;
  // range scans: P x n_cap piece matrices (grown on demand)
  uint64_t pcap = 0;
  uint64_t *plo = nullptr, *phi = nullptr, *rlo = nullptr, *rhi = nullptr;
  uint64_t *rc = nullptr, *roff = nullptr, *bc = nullptr, *bsc = nullptr;
  uint64_t* rvals = nullptr;  // the values this rank's scans of received pieces found
  uint64_t rvcap = 0;
  uint64_t* bv = nullptr;     // the values received back
  uint64_t bvcap = 0;
  uint64_t* pvs = nullptr;    // async scans: the values to send, peer_cap per peer
  uint64_t pvscap = 0;
  uint64_t* rw = nullptr;     // [2P + 8] small words read back once per scan batch
  // the last batch, for shm_shard_range_values after SHM_ENOSPC
  uint64_t last_n = 0, last_ncap = 0, last_total = 0;
  const uint64_t* last_off = nullptr;
  bool last_ok = false;
};

}  // namespace

struct shm_shard {
  shm_tree* local = nullptr;
  uint32_t world = 1, rank = 0;
  uint64_t cap = 0;               // the local tree's max_batch
  Xport* xp[3] = {nullptr, nullptr, nullptr};  // search slots 0 / 1, exclusive calls
  GetSlot slot[2];
  int next = 0;
  ExclCtx ex;
  hipStream_t side = nullptr;     // read-backs that wait on an event
  shm::dev::ShardBounds bnd{};
  // shm__shard_force_route: even at world 1 every get and insert takes the
  // routed path -- slot placement, the exchange through the transport (each
  // rank's own run included, so RCCL sends it to itself), the local batch,
  // the results back, the gather -- as at world > 1
  bool force_route = false;
};

namespace {

void free_shard(shm_shard* h) {
  for (GetSlot& s : h->slot) {
    dfree(s.cw); dfree(s.ctr); dfree(s.pk); dfree(s.pr); dfree(s.pv); dfree(s.pb); dfree(s.spos);
    dfree(s.ovk); dfree(s.ovi); dfree(s.ocnt); dfree(s.okb); dfree(s.operm); dfree(s.ores);
    dfree(s.ork); dfree(s.orv);
    if (s.ev_keys) (void)hipEventDestroy(s.ev_keys);
  }
  ExclCtx& e = h->ex;
  dfree(e.icnt); dfree(e.kb); dfree(e.vb); dfree(e.perm); dfree(e.pk); dfree(e.pv); dfree(e.rk);
  dfree(e.rv); dfree(e.ork); dfree(e.orv); dfree(e.plo); dfree(e.phi); dfree(e.rlo); dfree(e.rhi);
  dfree(e.rc); dfree(e.roff); dfree(e.bc); dfree(e.bsc); dfree(e.rvals); dfree(e.bv); dfree(e.pvs); dfree(e.rw);
  if (e.ev_ins) (void)hipEventDestroy(e.ev_ins);
  if (h->side) (void)hipStreamDestroy(h->side);
  // xp[0] may own the base communicator: destroy the splits first
  for (int i = 2; i >= 0; --i) delete h->xp[i];
  delete h;
}

int alloc_shard(shm_shard* h) {
  const uint32_t P = h->world;
  const uint64_t cap = h->cap;
  int rc = SHM_OK;
  for (GetSlot& s : h->slot) {
    // a peer's share of a uniform batch is cap / P; 25 % + 256 of slack
    s.pcap = P == 1 ? cap : std::min<uint64_t>(cap, get_slot_cap(cap, P));
    const uint64_t slots = (uint64_t)P * s.pcap;
    rc |= dalloc(&s.cw, 2 * (uint64_t)P + 2);
    rc |= dalloc(&s.ctr, shm::dev::route_ctr_words(P));
    if (s.ctr && hipMemset(s.ctr, 0, 4 * shm::dev::route_ctr_words(P)) != hipSuccess) rc |= SHM_EIO;
    rc |= dalloc(&s.pk, slots);
    rc |= dalloc(&s.pr, slots);
    rc |= dalloc(&s.pv, slots);
    rc |= dalloc(&s.pb, slots);
    rc |= dalloc(&s.spos, cap);
    rc |= dalloc(&s.ovk, cap);
    rc |= dalloc(&s.ovi, cap);
    rc |= dalloc(&s.ocnt, P);
    rc |= dalloc(&s.okb, cap);
    rc |= dalloc(&s.operm, cap);
    rc |= dalloc(&s.ores, cap);
    if (hipEventCreateWithFlags(&s.ev_keys, hipEventDisableTiming) != hipSuccess) rc |= SHM_EIO;
  }
  ExclCtx& e = h->ex;
  e.icap = P == 1 ? cap : cap / P;
  rc |= dalloc(&e.icnt, 2 * (uint64_t)P);
  rc |= dalloc(&e.kb, cap);
  rc |= dalloc(&e.vb, cap);
  rc |= dalloc(&e.perm, cap);
  rc |= dalloc(&e.pk, (uint64_t)P * e.icap);
  rc |= dalloc(&e.pv, (uint64_t)P * e.icap);
  rc |= dalloc(&e.rk, (uint64_t)P * e.icap);
  rc |= dalloc(&e.rv, (uint64_t)P * e.icap);
  rc |= dalloc(&e.rw, 2 * (uint64_t)P + 8);
  if (hipEventCreateWithFlags(&e.ev_ins, hipEventDisableTiming) != hipSuccess) rc |= SHM_EIO;
  if (hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking) != hipSuccess) rc |= SHM_EIO;
  // shard p owns [ceil(p 2^64 / P), ceil((p + 1) 2^64 / P))
  for (uint32_t p = 0; p < P; ++p)
    h->bnd.b[p] = (uint64_t)((((unsigned __int128)p << 64) + P - 1) / P);
  return rc ? SHM_ENOMEM : SHM_OK;
}

// `bytes` of device words at src, once event ev has completed (the side
// stream waits for it; the caller's stream keeps going)
int read_after(shm_shard* h, hipEvent_t ev, const void* src, uint64_t bytes, void* out) {
  HIP_OK2(hipStreamWaitEvent(h->side, ev, 0));
  return shm_read_words(h->local, src, bytes, out, h->side);
}

// Every rank must have created its tree with the same max_batch: the slot
// sizes of the exchanges derive from it (one read-back, at creation)
int check_caps(shm_shard* h) {
  const uint32_t P = h->world;
  std::vector<uint64_t> w(2 * P, h->cap);
  uint64_t* d = h->ex.rw;  // 2P + 8 words
  HIP_OK2(hipMemcpyAsync(d, w.data(), 8ull * P, hipMemcpyHostToDevice, h->side));
  RC_OK(h->xp[2]->a2a(d, d + P, 1, 8, h->side));
  RC_OK(shm_read_words(h->local, d, 16ull * P, w.data(), h->side));
  for (uint32_t p = 0; p < P; ++p)
    if (w[P + p] != h->cap) {
      fprintf(stderr, "sherman_amd: shard %u has max_batch %llu, rank %u %llu: they must match\n",
              p, (unsigned long long)w[P + p], h->rank, (unsigned long long)h->cap);
      return SHM_EINVAL;
    }
  return SHM_OK;
}

int make_shard(shm_tree* local, Xport* x0, Xport* x1, Xport* x2, uint32_t world, uint32_t rank,
               shm_shard** out) {
  shm_shard* h = new shm_shard();
  h->local = local;
  h->world = world;
  h->rank = rank;
  h->cap = shm_tree_max_batch(local);
  h->xp[0] = x0;
  h->xp[1] = x1;
  h->xp[2] = x2;
  for (int i = 0; i < 3; ++i) {
    h->xp[i]->P = world;
    h->xp[i]->rank = rank;
  }
  h->slot[0].x = x0;
  h->slot[1].x = x1;
  h->ex.x = x2;
  int rc = alloc_shard(h);
  if (rc == SHM_OK) rc = check_caps(h);
  if (rc) {
    free_shard(h);
    return rc;
  }
  *out = h;
  return SHM_OK;
}

int rccl_shard(shm_tree* local, ncclComm_t comm, uint32_t world, uint32_t rank, bool own,
               shm_shard** out) {
  // two more communicators split from the first (same ranks, same order), so
  // the two search slots and the exclusive calls never serialise on one
  ncclComm_t c[3] = {comm, nullptr, nullptr};
  for (int i = 1; i < 3; ++i)
    if (nccl_ok(ncclCommSplit(comm, 0, (int)rank, &c[i], nullptr), "ncclCommSplit") || !c[i]) {
      for (int j = 1; j < i; ++j) (void)ncclCommDestroy(c[j]);
      if (own) (void)ncclCommDestroy(comm);
      return SHM_EIO;
    }
  RcclXport* x[3];
  for (int i = 0; i < 3; ++i) {
    x[i] = new RcclXport();
    x[i]->comm = c[i];
    x[i]->own = i > 0 || own;
  }
  return make_shard(local, x[0], x[1], x[2], world, rank, out);
}

// ---- routed insert: the overflow tails of the last insert ------------------------
// Called before anything else the shard does (and by shm_shard_synchronize):
// one read-back of the last insert's sent and received counts (ready once its
// key exchange has run); where a run passed its slot, both sides send /
// receive the tail in an exact second round, applied behind the slots.
int flush(shm_shard* h) {
  ExclCtx& e = h->ex;
  if (!e.pending) return SHM_OK;
  e.pending = false;
  const uint32_t P = h->world;
  std::vector<uint64_t> c(2 * P);
  RC_OK(read_after(h, e.ev_ins, e.icnt, 16ull * P, c.data()));
  std::vector<uint64_t> scnt(P, 0), soff(P, 0), rcnt(P, 0), roff(P, 0);
  uint64_t base = 0, nr = 0, ns = 0;
  for (uint32_t p = 0; p < P; ++p) {
    if (c[p] > e.icap) {
      scnt[p] = c[p] - e.icap;
      soff[p] = base + e.icap;  // the tail of run p in kb / vb
    }
    base += c[p];
    ns += scnt[p];
    const uint64_t got = p == h->rank ? c[p] : c[P + p];  // own run: never exchanged
    if (got > e.icap) rcnt[p] = got - e.icap;
    roff[p] = nr;
    nr += rcnt[p];
  }
  if (ns == 0 && nr == 0) return SHM_OK;
  hipStream_t s = e.pstream;
  RC_OK(ensure(e.ork, e.orcap, nr, s));
  RC_OK(ensure(e.orv, e.orvcap, nr, s));
  RC_OK(e.x->group_start());
  RC_OK(e.x->p2p(e.kb, scnt.data(), soff.data(), e.ork, rcnt.data(), roff.data(), 8, s));
  RC_OK(e.x->p2p(e.vb, scnt.data(), soff.data(), e.orv, rcnt.data(), roff.data(), 8, s));
  RC_OK(e.x->group_end());
  return nr ? shm_insert_batch_async(h->local, e.ork, e.orv, nr, s) : SHM_OK;
}

// ---- routed get: the overflow round of one slot --------------------------------------
int get_overflow(shm_shard* h, GetSlot& s, uint64_t* vals_out, uint8_t* found_out) {
  const uint32_t P = h->world;
  std::vector<uint32_t> w(2 * P + 1);
  RC_OK(read_after(h, s.ev_keys, s.cw, 4ull * (2 * P + 1), w.data()));
  std::vector<uint64_t> scnt(P, 0), soff(P, 0), rcnt(P, 0), roff(P, 0);
  uint64_t m = 0, mr = 0;
  for (uint32_t p = 0; p < P; ++p) {
    scnt[p] = w[p] > s.ncap ? w[p] - s.ncap : 0;
    soff[p] = m;
    m += scnt[p];
    const uint32_t got = p == h->rank ? w[p] : w[P + 1 + p];  // own run: never exchanged
    rcnt[p] = got > s.ncap ? got - s.ncap : 0;
    roff[p] = mr;
    mr += rcnt[p];
  }
  if (m != w[P]) return SHM_EIO;  // the overflow list disagrees with the counts
  if (m == 0 && mr == 0) return SHM_OK;
  hipStream_t st = s.stream;
  // the cut keys grouped by owner (stable), exchanged exactly, searched, and
  // their values sent back and scattered to the inputs they came from
  if (m) RC_OK(shm_route_bucket(h->local, s.ovk, m, P, s.ocnt, s.okb, s.operm, st));
  RC_OK(ensure(s.ork, s.orcap, mr, st));
  RC_OK(ensure(s.orv, s.orvcap, mr, st));
  RC_OK(s.x->p2p(s.okb, scnt.data(), soff.data(), s.ork, rcnt.data(), roff.data(), 8, st));
  if (mr) RC_OK(shm_search_batch(h->local, s.ork, mr, s.orv, nullptr, st));
  RC_OK(s.x->p2p(s.orv, rcnt.data(), roff.data(), s.ores, scnt.data(), soff.data(), 8, st));
  shm::dev::launch_route_ov_scatter(s.ores, s.operm, s.ovi, m, vals_out, found_out, st);
  return hipGetLastError() == hipSuccess ? SHM_OK : SHM_EIO;
}

// range scans: piece buffers for P x n_cap
int ensure_pieces(shm_shard* h, uint64_t m, hipStream_t s) {
  ExclCtx& e = h->ex;
  if (m <= e.pcap && e.plo) return SHM_OK;
  HIP_OK2(hipStreamSynchronize(s));
  for (uint64_t** p : {&e.plo, &e.phi, &e.rlo, &e.rhi, &e.rc, &e.roff, &e.bc, &e.bsc}) dfree(*p);
  e.pcap = m;
  int rc = SHM_OK;
  for (uint64_t** p : {&e.plo, &e.phi, &e.rlo, &e.rhi, &e.rc, &e.roff, &e.bc, &e.bsc})
    rc |= dalloc(p, m);
  return rc ? SHM_ENOMEM : SHM_OK;
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
      world > kMaxWorld || rank >= world)
    return SHM_EINVAL;
  ncclUniqueId id;
  memcpy(&id, nccl_id, sizeof(id));
  ncclComm_t comm = nullptr;
  NCCL_OK(ncclCommInitRank(&comm, (int)world, id, (int)rank));
  return rccl_shard(local, comm, world, rank, true, out);
}

int shm_shard_create_with_comm(shm_tree* local, void* nccl_comm, uint32_t world, uint32_t rank,
                               shm_shard** out) {
  if (!local || !nccl_comm || !out || world == 0 || world > kMaxWorld || rank >= world)
    return SHM_EINVAL;
  return rccl_shard(local, (ncclComm_t)nccl_comm, world, rank, false, out);
}

int shm_shard_destroy(shm_shard* h) {
  if (!h) return SHM_EINVAL;
  const int rc = flush(h);  // a collective: every rank destroys its handle
  (void)hipDeviceSynchronize();
  free_shard(h);
  return rc;
}

int shm_shard_synchronize(shm_shard* h) {
  if (!h) return SHM_EINVAL;
  const int rc = flush(h);
  const int rs = shm_synchronize(h->local);
  return rc ? rc : rs;
}

int shm_shard_search_begin(shm_shard* h, const uint64_t* keys, uint64_t n, void* stream,
                           uint32_t* ticket) {
  if (!h || !ticket || (n && !keys)) return SHM_EINVAL;
  const int i = h->next;
  GetSlot& s = h->slot[i];
  if (s.busy) return SHM_EINVAL;  // end the slot's batch first
  if (n > h->cap) return SHM_E2BIG;
  RC_OK(flush(h));
  h->next = (i + 1) % 2;
  s.keys = keys;
  s.n = n;
  s.stream = (hipStream_t)stream;
  *ticket = (uint32_t)i;
  const uint32_t P = h->world;
  s.ncap = P == 1 ? n : std::min<uint64_t>(s.pcap, get_slot_cap(n, P));
  // this rank's own run goes straight into its receive slot (s.pr), so only
  // the P - 1 peers' runs cross the collective (none at P = 1)
  const uint32_t me = h->rank;
  s.busy = true;
  if (P == 1 && !h->force_route) return SHM_OK;  // nothing to route: _end is the local get
  // (forced: the own run crosses the transport like the peers')
  // the runs are padded once per capacity: later batches leave earlier keys
  // of the same owner in the tails (searched, never gathered)
  const bool fill = s.filled != s.ncap;
  s.filled = s.ncap;
  shm::dev::launch_route_slots(s.keys, s.n, P, s.ncap, s.cw, s.ctr, s.pk, s.spos, s.ovk, s.ovi,
                               shm__error_word(h->local), s.stream, me,
                               h->force_route ? nullptr : s.pr + (uint64_t)me * s.ncap, fill);
  HIP_OK2(hipGetLastError());
  RC_OK(s.x->group_start());
  RC_OK(s.x->a2a_peers(s.pk, s.pr, s.ncap, 8, s.stream));
  RC_OK(s.x->a2a_peers(s.cw, s.cw + P + 1, 1, 4, s.stream));  // keys routed to each peer
  RC_OK(s.x->group_end());
  HIP_OK2(hipEventRecord(s.ev_keys, s.stream));
  return SHM_OK;
}

int shm_shard_search_end(shm_shard* h, uint32_t ticket, uint64_t* vals_out, uint8_t* found_out) {
  if (!h || ticket >= 2u || !h->slot[ticket].busy) return SHM_EINVAL;
  GetSlot& s = h->slot[ticket];
  if (s.n && (!vals_out || !found_out)) return SHM_EINVAL;
  s.busy = false;
  const uint32_t P = h->world;
  // one shard: the batch is all this rank's, searched where it lies
  if (P == 1 && !h->force_route)
    return shm_search_batch(h->local, s.keys, s.n, vals_out, found_out, s.stream);
  RC_OK(shm_search_batch(h->local, s.pr, (uint64_t)P * s.ncap, s.pv, nullptr, s.stream));
  // the results go back the way the keys came, slot for slot; the own run's
  // are gathered straight from the local results (forced: exchanged as well)
  RC_OK(s.x->a2a_peers(s.pv, s.pb, s.ncap, 8, s.stream));
  shm::dev::launch_route_gather(s.pb, s.spos, s.n, vals_out, found_out, s.stream, h->rank, s.ncap,
                                h->force_route ? nullptr : s.pv);
  HIP_OK2(hipGetLastError());
  return get_overflow(h, s, vals_out, found_out);
}

int shm_shard_search(shm_shard* h, const uint64_t* keys, uint64_t n, uint64_t* vals_out,
                     uint8_t* found_out, void* stream) {
  uint32_t ticket = 0;
  RC_OK(shm_shard_search_begin(h, keys, n, stream, &ticket));
  return shm_shard_search_end(h, ticket, vals_out, found_out);
}

int shm_shard_insert(shm_shard* h, const uint64_t* keys, const uint64_t* vals, uint64_t n,
                     void* stream) {
  if (!h || (n && (!keys || !vals))) return SHM_EINVAL;
  if (n > h->cap) return SHM_E2BIG;
  RC_OK(flush(h));
  ExclCtx& e = h->ex;
  hipStream_t s = (hipStream_t)stream;
  const uint32_t P = h->world;
  // a batch holding kKeyMax routes nothing (SHM_EINVAL at the next
  // synchronising call), as a local insert rejects its chunk
  RC_OK(shm__route_bucket_insert(h->local, keys, n, P, e.icnt, e.kb, e.perm, s));
  RC_OK(shm_route_permute(h->local, vals, e.perm, n, e.vb, s));
  // this rank's own run is packed straight into its receive slot (forced:
  // it crosses the transport like the peers')
  const uint64_t mine = (uint64_t)h->rank * e.icap;
  const bool fr = h->force_route;
  shm::dev::launch_route_pack(e.kb, e.vb, e.icnt, P, e.icap, e.pk, e.pv, s, h->rank,
                              fr ? nullptr : e.rk + mine, fr ? nullptr : e.rv + mine);
  HIP_OK2(hipGetLastError());
  RC_OK(e.x->group_start());
  RC_OK(e.x->a2a_peers(e.pk, e.rk, e.icap, 8, s));
  RC_OK(e.x->a2a_peers(e.pv, e.rv, e.icap, 8, s));
  RC_OK(e.x->a2a_peers(e.icnt, e.icnt + P, 1, 8, s));
  RC_OK(e.x->group_end());
  HIP_OK2(hipEventRecord(e.ev_ins, s));
  e.pending = P > 1 || fr;
  e.pstream = s;
  return shm__insert_batch_padded(h->local, e.rk, e.rv, (uint64_t)P * e.icap, s);
}

}  // extern "C"

namespace {
// steps 1-3 of a routed range scan batch, all on the device: pieces to their
// shards, the local scans of the received pieces (values packed in rvals,
// row p = rank p's), counts back, per-peer totals (rw), counts_out,
// offsets_out and the received runs' offsets (bsc)
int range_scan_pieces(shm_shard* h, const uint64_t* from, const uint64_t* to, uint64_t n,
                      uint64_t n_cap, uint64_t* counts_out, uint64_t* offsets_out, hipStream_t s) {
  const uint32_t P = h->world;
  const uint64_t m = (uint64_t)P * n_cap;
  ExclCtx& e = h->ex;
  uint64_t* rw = e.rw;  // [0, P) sent, [P, 2P) received, scanner {total, err}, scans {total, err}, bsc {total, err}
  // 1. pieces, row p to rank p
  shm::dev::launch_range_pieces(from, to, n, n_cap, P, h->bnd, e.plo, e.phi, s);
  HIP_OK2(hipGetLastError());
  RC_OK(e.x->group_start());
  RC_OK(e.x->a2a(e.plo, e.rlo, n_cap, 8, s));
  RC_OK(e.x->a2a(e.phi, e.rhi, n_cap, 8, s));
  RC_OK(e.x->group_end());
  // 2. this shard scans every received piece (count, offsets, staged fill)
  RC_OK(shm_range_query_batch_async(h->local, e.rlo, e.rhi, m, e.rc, e.roff, e.rvals, e.rvcap,
                                    rw + 2 * P, s));
  // 3. piece counts back; per-peer totals, per-scan counts and offsets
  RC_OK(e.x->a2a(e.rc, e.bc, n_cap, 8, s));
  shm::dev::launch_range_sums(e.rc, e.bc, n, n_cap, P, rw, counts_out, s);
  HIP_OK2(hipGetLastError());
  RC_OK(shm__scan_u64(h->local, counts_out, offsets_out, n, rw + 2 * P + 2, s));
  RC_OK(shm__scan_u64(h->local, e.bc, e.bsc, m, rw + 2 * P + 4, s));
  return SHM_OK;
}
}  // namespace

extern "C" {

int shm_shard_range_query(shm_shard* h, const uint64_t* from, const uint64_t* to, uint64_t n,
                          uint64_t n_cap, uint64_t* counts_out, uint64_t* offsets_out,
                          uint64_t* vals_out, uint64_t vals_cap, uint64_t* total_out,
                          void* stream) {
  if (!h || !total_out || n > n_cap || (n && (!from || !to || !counts_out || !offsets_out)) ||
      (vals_cap && !vals_out))
    return SHM_EINVAL;
  const uint32_t P = h->world;
  const uint64_t m = (uint64_t)P * n_cap;
  if (m > h->cap) return SHM_E2BIG;
  RC_OK(flush(h));
  ExclCtx& e = h->ex;
  e.last_ok = false;
  hipStream_t s = (hipStream_t)stream;
  RC_OK(ensure_pieces(h, m, s));
  // about n_cap non-empty pieces of ~100 values (C5): grown when a batch needs more
  if (!e.rvals) RC_OK(ensure(e.rvals, e.rvcap, std::max<uint64_t>(n_cap * 160, 1u << 20), s));
  uint64_t* rw = e.rw;
  RC_OK(range_scan_pieces(h, from, to, n, n_cap, counts_out, offsets_out, s));
  // 4. the one host synchronisation: the value counts each way
  std::vector<uint64_t> w(2 * P + 6);
  RC_OK(shm_read_words(h->local, rw, 8ull * (2 * P + 6), w.data(), s));
  const uint64_t scanned = w[2 * P], total = w[2 * P + 2];
  if (scanned > e.rvcap) {
    // the fill pass dropped values past its buffer: grow it, fill again
    RC_OK(ensure(e.rvals, e.rvcap, scanned, s));
    RC_OK(shm_range_query(h->local, e.rlo, e.rhi, m, e.rc, e.roff, e.rvals, s));
  }
  std::vector<uint64_t> scnt(P), soff(P), rcnt(P), roff(P);
  uint64_t so = 0, ro = 0;
  for (uint32_t p = 0; p < P; ++p) {
    scnt[p] = w[p];
    soff[p] = so;
    so += w[p];
    rcnt[p] = w[P + p];
    roff[p] = ro;
    ro += w[P + p];
  }
  if (so != scanned || ro != total) return SHM_EIO;
  RC_OK(ensure(e.bv, e.bvcap, ro, s));
  RC_OK(e.x->p2p(e.rvals, scnt.data(), soff.data(), e.bv, rcnt.data(), roff.data(), 8, s));
  *total_out = total;
  e.last_n = n;
  e.last_ncap = n_cap;
  e.last_total = total;
  e.last_off = offsets_out;
  e.last_ok = true;
  // counts / offsets stay valid; shm_shard_range_values fills a larger buffer
  if (total > vals_cap) return SHM_ENOSPC;
  shm::dev::launch_range_assemble(e.bv, e.bc, e.bsc, n, n_cap, P, offsets_out, vals_out, vals_cap,
                                  s);
  return hipGetLastError() == hipSuccess ? SHM_OK : SHM_EIO;
}

int shm_shard_range_query_async(shm_shard* h, const uint64_t* from, const uint64_t* to,
                                uint64_t n, uint64_t n_cap, uint64_t* counts_out,
                                uint64_t* offsets_out, uint64_t* vals_out, uint64_t vals_cap,
                                uint64_t peer_cap, uint64_t* status, void* stream) {
  if (!h || !status || n > n_cap || (n && (!from || !to || !counts_out || !offsets_out)) ||
      (vals_cap && !vals_out) || peer_cap == 0)
    return SHM_EINVAL;
  const uint32_t P = h->world;
  const uint64_t m = (uint64_t)P * n_cap;
  if (m > h->cap) return SHM_E2BIG;
  RC_OK(flush(h));
  ExclCtx& e = h->ex;
  e.last_ok = false;
  hipStream_t s = (hipStream_t)stream;
  RC_OK(ensure_pieces(h, m, s));
  // fixed runs of peer_cap values per peer each way: the scan pass's buffer
  // holds every run that fits (a longer one is flagged, not grown)
  const uint64_t runs = (uint64_t)P * peer_cap;
  RC_OK(ensure(e.rvals, e.rvcap, runs, s));
  RC_OK(ensure(e.pvs, e.pvscap, runs, s));
  RC_OK(ensure(e.bv, e.bvcap, runs, s));
  RC_OK(range_scan_pieces(h, from, to, n, n_cap, counts_out, offsets_out, s));
  // 4. the runs padded to peer_cap on the device, exchanged whole
  shm::dev::launch_range_pitch(e.rvals, e.rw, P, peer_cap, e.pvs, e.rvcap, vals_cap, status, s);
  HIP_OK2(hipGetLastError());
  RC_OK(e.x->a2a(e.pvs, e.bv, peer_cap, 8, s));
  e.last_n = n;
  e.last_ncap = n_cap;
  e.last_total = 0;  // on the device (status[0])
  e.last_off = offsets_out;
  e.last_ok = false;  // shm_shard_range_values needs the host total: not after this call
  shm::dev::launch_range_assemble(e.bv, e.bc, e.bsc, n, n_cap, P, offsets_out, vals_out, vals_cap,
                                  s, peer_cap);
  return hipGetLastError() == hipSuccess ? SHM_OK : SHM_EIO;
}

int shm_shard_range_values(shm_shard* h, uint64_t* vals_out, uint64_t vals_cap, void* stream) {
  if (!h || !h->ex.last_ok || (h->ex.last_total && !vals_out)) return SHM_EINVAL;
  const ExclCtx& e = h->ex;
  if (e.last_total > vals_cap) return SHM_ENOSPC;
  shm::dev::launch_range_assemble(e.bv, e.bc, e.bsc, e.last_n, e.last_ncap, h->world, e.last_off,
                                  vals_out, vals_cap, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? SHM_OK : SHM_EIO;
}

// Library-internal test hooks, not part of include/sherman_amd.h.
// (1) The routed get's slot placement and result gather for P shards, so the
// placement can be checked on one GPU without P ranks (tests/test_gpu_shard.py).
// cursor: P + 1 u32 of device scratch; ovk / ovi nullable (then the overflow
// bit goes to t's error word).
// the claim words of the hooks' placements (zero at rest; one call at a time)
uint32_t* hook_ctr() {
  static uint32_t* c = nullptr;
  if (!c) {
    const uint64_t bytes = 4 * shm::dev::route_ctr_words(64);
    if (hipMalloc((void**)&c, bytes) != hipSuccess) return c = nullptr;
    if (hipMemset(c, 0, bytes) != hipSuccess) {
      (void)hipFree(c);
      c = nullptr;
    }
  }
  return c;
}
int shm__route_slots(shm_tree* t, const uint64_t* keys, uint64_t n, uint32_t P, uint64_t cap,
                     uint32_t* cursor, uint64_t* slots, uint32_t* spos, uint64_t* ovk,
                     uint32_t* ovi, void* stream) {
  if (!t || !cursor || !slots || !spos || P == 0 || P > 64 || (n && !keys) ||
      (uint64_t)P * cap >= ~0u)
    return SHM_EINVAL;
  uint32_t* ctr = hook_ctr();
  if (!ctr) return SHM_ENOMEM;
  shm::dev::launch_route_slots(keys, n, P, cap, cursor, ctr, slots, spos, ovk, ovi,
                               shm__error_word(t), (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? SHM_OK : SHM_EIO;
}
// ... and the shard's own form of it: the runs padded only when fill
int shm__route_slots_ex(shm_tree* t, const uint64_t* keys, uint64_t n, uint32_t P, uint64_t cap,
                        uint32_t* cursor, uint64_t* slots, uint32_t* spos, uint64_t* ovk,
                        uint32_t* ovi, int fill, void* stream) {
  if (!t || !cursor || !slots || !spos || P == 0 || P > 64 || (n && !keys) ||
      (uint64_t)P * cap >= ~0u)
    return SHM_EINVAL;
  uint32_t* ctr = hook_ctr();
  if (!ctr) return SHM_ENOMEM;
  shm::dev::launch_route_slots(keys, n, P, cap, cursor, ctr, slots, spos, ovk, ovi,
                               shm__error_word(t), (hipStream_t)stream, 0, nullptr, fill != 0);
  return hipGetLastError() == hipSuccess ? SHM_OK : SHM_EIO;
}
int shm__route_gather(const uint64_t* in, const uint32_t* spos, uint64_t n, uint64_t* vals_out,
                      uint8_t* found_out, void* stream) {
  if (n && (!in || !spos || !vals_out)) return SHM_EINVAL;
  shm::dev::launch_route_gather(in, spos, n, vals_out, found_out, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? SHM_OK : SHM_EIO;
}

// (3) The routed path at world 1 (force_route above): every call through the
// transport, RCCL sending each run to this rank itself (tests/test_gpu_shard.py
// [nccl-1-routed]), so ncclSend / ncclRecv run on a one-GPU box.
int shm__shard_force_route(shm_shard* h, int on) {
  if (!h) return SHM_EINVAL;
  h->force_route = on != 0;
  for (Xport* x : h->xp)
    if (x) x->self_too = on != 0;
  return SHM_OK;
}

// (2) An in-process group of P shard handles on one device (P trees, one host
// thread per rank, every rank's calls on ONE shared stream so the trees'
// persistent kernels never share the device): the whole routed path —
// slots, overflow rounds, padded inserts and their tails, range pieces — with
// device copies for the collectives (tests/test_gpu_shard.py at P = 8).
int shm__local_group_create(uint32_t world, void** out) {
  if (!out || world == 0 || world > kMaxWorld) return SHM_EINVAL;
  *out = new LocalGroup(world);
  return SHM_OK;
}
int shm__local_group_destroy(void* g) {
  delete static_cast<LocalGroup*>(g);
  return SHM_OK;
}
int shm__shard_create_local(shm_tree* local, void* group, uint32_t rank, shm_shard** out) {
  LocalGroup* g = static_cast<LocalGroup*>(group);
  if (!local || !g || !out || rank >= g->P) return SHM_EINVAL;
  LocalXport* x[3];
  for (int i = 0; i < 3; ++i) {
    x[i] = new LocalXport();
    x[i]->g = g;
    x[i]->rank = rank;
    x[i]->P = g->P;
    if (x[i]->init()) {
      for (int j = 0; j <= i; ++j) delete x[j];
      return SHM_EIO;
    }
  }
  return make_shard(local, x[0], x[1], x[2], g->P, rank, out);
}

}  // extern "C"
