"""Range-sharded batched get / insert over P ranks (one process per GPU).

Replaces Sherman's memory-node placement (chunks round-robin over nodes,
include/DSM.h:198-224; every Tree::search walks remote pages over RDMA,
src/Tree.cpp:405-459) with key-range shards: shard s owns
[s * 2^64 / P, (s+1) * 2^64 / P) and holds a complete B-link tree of its
slice, so no page pointer crosses GPUs and each query touches exactly one
shard.  One exchange step each way per batch (RCCL all-to-all over xGMI on
the GPU box, gloo in the CPU tests):

  get    : bucket keys by owner (stable) -> all_to_all counts -> all_to_all
           keys -> local search_batch -> all_to_all values back -> un-permute
  insert : bucket keys by owner (stable), carry values with the same
           permutation -> all_to_all counts / keys / values -> local
           insert_batch.  Received segments arrive in source-rank order and
           bucketing is stable, so the receiver applies the union of all
           ranks' batches in rank-major batch order (last writer wins), which
           is one valid linearisation of Sherman's concurrent inserts.

`local` is the per-rank shard: a sherman_amd.Tree on the GPU path.  Any
object with the same five methods works (the multi-rank CPU tests plug in an
oracle-backed shard to check the exchange logic itself).
"""
import torch


def owner_of(keys, world):
    """floor(k * P / 2^64) for u64 keys held as int64 (== __umul64hi(k, P))."""
    hi = (keys >> 32) & 0xFFFFFFFF
    lo = keys & 0xFFFFFFFF
    return (hi * world + ((lo * world) >> 32)) >> 32


def shard_range(rank, world):
    """(key_lo, key_bits) hint for shard `rank` of `world`: its keys lie in
    [ceil(rank * 2^64 / P), ...) within 2^key_bits of key_lo (shm_config)."""
    lo = (rank * (1 << 64) + world - 1) // world
    bits = 64 - (world.bit_length() - 1)  # 2^bits >= 2^64 / P
    return lo, bits


class ShardRouter:
    def __init__(self, local, world, dist, group=None):
        self.local, self.world, self.dist, self.group = local, world, dist, group
        self._bufs = {}

    def _buf(self, name, n, dtype, device):
        b = self._bufs.get(name)
        if b is None or b.numel() < n or b.device != torch.device(device) or b.dtype != dtype:
            b = torch.empty(max(n, 1), dtype=dtype, device=device)
            self._bufs[name] = b
        return b[:n]

    def _a2a(self, out, inp, out_splits=None, in_splits=None):
        self.dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def _bucket(self, keys):
        n, dev = keys.numel(), keys.device
        kb = self._buf("kb", n, torch.int64, dev)
        perm = self._buf("perm", n, torch.int32, dev)
        cnt = self._buf("cnt", self.world, torch.int64, dev)
        self.local.route_bucket(keys, self.world, kb, perm, cnt)
        rcnt = self._buf("rcnt", self.world, torch.int64, dev)
        self._a2a(rcnt, cnt)
        return kb, perm, cnt.tolist(), rcnt.tolist()

    def search(self, keys, vals_out, found_out):
        """Batched get of this rank's keys; results land in input order."""
        n, dev = keys.numel(), keys.device
        kb, perm, cnt, rcnt = self._bucket(keys)
        nrecv = sum(rcnt)
        recv = self._buf("recv", nrecv, torch.int64, dev)
        self._a2a(recv, kb, rcnt, cnt)
        rv = self._buf("rv", nrecv, torch.int64, dev)
        rf = self._buf("rf", nrecv, torch.uint8, dev)
        self.local.search_batch(recv, rv, rf)
        back = self._buf("back", n, torch.int64, dev)
        self._a2a(back, rv, cnt, rcnt)
        self.local.route_unpermute(back, perm, vals_out)
        # value 0 is kValueNull: found <=> value != 0 (Tree.cpp:445-448)
        torch.ne(vals_out, 0, out=found_out)

    def insert(self, keys, vals):
        """Batched insert (value 0 deletes) of this rank's (key, value) pairs."""
        dev = keys.device
        kb, perm, cnt, rcnt = self._bucket(keys)
        vb = self._buf("vb", keys.numel(), torch.int64, dev)
        self.local.route_permute(vals, perm, vb)
        nrecv = sum(rcnt)
        rk = self._buf("rk", nrecv, torch.int64, dev)
        rv = self._buf("rvi", nrecv, torch.int64, dev)
        self._a2a(rk, kb, rcnt, cnt)
        self._a2a(rv, vb, rcnt, cnt)
        self.local.insert_batch(rk, rv)
