// upper_quick.h — the part of k_upper a chunk needs when nothing is left to
// split and nothing to delete (insert.hip's quick path): the next chunk's
// counters zeroed, the superblock's batch count, the host mirror's tags.
// Shared by k_upper and by the segmentation kernel, whose block 0 completes
// a chunk without a new key or a delete (C3's chunks) so that the upsert
// kernel and k_upper return at once (util.hip k_seg_fill).
#pragma once
#include "device_common.h"
#include "kernels.h"

namespace shm {
namespace dev {

// the other parity's counters and hand-off words start the next chunk at 0
// (threads z0, z0 + zs, ... of the caller)
__device__ __forceinline__ void upper_zero_next(UpperCtl* ctl, uint32_t par, uint64_t z0,
                                                uint64_t zs) {
  for (uint64_t j = z0; j < (uint64_t)kMaxUpper; j += zs) {
    ctl->leaf_np[par ^ 1][j] = 0;
    ctl->leaf_ns[par ^ 1][j] = 0;
    ctl->leaf_nb[par ^ 1][j] = 0;
  }
  for (uint64_t j = z0; j < (uint64_t)kUpPhases * 32; j += zs) {
    (&ctl->tk[par ^ 1][0][0])[j] = 0;
    (&ctl->dn[par ^ 1][0][0])[j] = 0;
  }
  if (z0 < 16) ctl->lvl_sep[par ^ 1][z0] = 0;
  if (z0 == 0) {
    ctl->late[par ^ 1][0] = 0;
    ctl->abort[par ^ 1][0] = 0;
    ctl->alloc[par ^ 1][0] = 0;
    ctl->made[par ^ 1][0] = 0;
    ctl->root_new[par ^ 1][0] = 0;
    ctl->done[par ^ 1][0] = 0;
    ctl->ualloc[par ^ 1][0] = 0;
  }
}

// One thread: a chunk that made no page.  The error attribution first (no
// load or returning atomic after the host mirror's PCIe stores), then the
// superblock's batch count and the mirror's tags (the chunk's tag while the
// host's directory is behind; the applied tag that insert_order waits for).
__device__ __forceinline__ void upper_finish_unchanged(const UpperArgs& a, uint32_t err_bits) {
  if (err_bits & ~kErrKeyMax) atomicCAS(a.err + 1, 0u, (uint32_t)a.batch);
  Superblock* sb = reinterpret_cast<Superblock*>(a.arena);
  sb->batches = a.batch;
  if (a.pub) {
    if (a.pub_always)
      __hip_atomic_store(a.pub + 0, a.batch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(a.pub + kPubApplied, a.batch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}


// A chunk without a new key (every op applied in place by k_locate, C3's
// chunks): block 0 also completes it when it has no delete either -- k_upper's
// quick path (upper_quick.h) -- and tags it in UpperCtl.skip, so the upsert
// kernel (no segment) and k_upper return after one load
__device__ __forceinline__ void seg_complete_unchanged(const UpperArgs& q) {
  if (*q.n_del != 0) return;  // the deletes are k_upper's
  upper_zero_next(q.ctl, q.par, threadIdx.x, blockDim.x);
  if (threadIdx.x == 0) {
    if (q.prof)  // the chunk's unique upserts (profiling; no delete, nothing staged)
      atomicAdd(reinterpret_cast<unsigned long long*>(q.prof), (unsigned long long)q.n_del[-1]);
    upper_finish_unchanged(q, __hip_atomic_load(q.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    q.ctl->skip[q.par][0] = q.batch;
  }
}

}  // namespace dev
}  // namespace shm
