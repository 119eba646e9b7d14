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
  range  : a scan [lo, hi] is cut at shard boundaries into pieces, each piece
           goes to its owner (all_to_all of bounds), the owners scan their
           trees (range_query_batch), and counts then values come back
           (all_to_all); scan i's values are its pieces' values in shard
           order, i.e. in key order across shards (Tree::range_query,
           Tree.cpp:461-540, intended semantics).

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


_SIGN = -(1 << 63)  # int64 bit pattern of 2^63


def _u64(x):
    """Python int in [0, 2^64) -> the int64 holding the same bits."""
    return x - (1 << 64) if x >= (1 << 63) else x


def shard_bounds(world, device):
    """int64 tensor of the P + 1 u64 shard boundaries ceil(s * 2^64 / P)."""
    b = [_u64((s * (1 << 64) + world - 1) // world) for s in range(world)] + [_u64((1 << 64) - 1)]
    return torch.tensor(b, dtype=torch.int64, device=device)


def umax(a, b):
    """element-wise max of u64 values held as int64 (compare with the sign bit flipped)"""
    return torch.where((a ^ _SIGN) >= (b ^ _SIGN), a, b)


def umin(a, b):
    return torch.where((a ^ _SIGN) <= (b ^ _SIGN), a, b)


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
        self._pending = False  # a search_begin not yet ended (it owns kb / perm)

    def _buf(self, name, n, dtype, device):
        b = self._bufs.get(name)
        if b is None or b.numel() < n or b.device != torch.device(device) or b.dtype != dtype:
            b = torch.empty(max(n, 1), dtype=dtype, device=device)
            self._bufs[name] = b
        return b[:n]

    def _a2a(self, out, inp, out_splits=None, in_splits=None):
        self.dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def _bucket_async(self, keys):
        """Bucket by owner and exchange the counts; nothing waits for them."""
        n, dev = keys.numel(), keys.device
        kb = self._buf("kb", n, torch.int64, dev)
        perm = self._buf("perm", n, torch.int32, dev)
        # send and receive counts side by side (one read-back fetches both);
        # a fresh buffer per batch, so a pending batch keeps its own counts
        cnts = torch.empty(2 * self.world, dtype=torch.int64, device=dev)
        cnt, rcnt = cnts[:self.world], cnts[self.world:2 * self.world]
        self.local.route_bucket(keys, self.world, kb, perm, cnt)
        self._a2a(rcnt, cnt)
        return kb, perm, cnts

    def _counts(self, cnts):
        """Both count vectors of one batch (its own `cnts` buffer: sent, then
        received) on the host, the RCCL split sizes: one zero-copy read-back
        (Tree.read_i64) on a GPU."""
        w = self.world
        rd = getattr(self.local, "read_i64", None)
        if rd is not None and cnts.device.type == "cuda" and w <= 16:
            both = rd(cnts[:2 * w])
        else:
            both = cnts[:2 * w].tolist()
        return both[:w], both[w:]

    def _bucket(self, keys):
        kb, perm, cnts = self._bucket_async(keys)
        return (kb, perm) + self._counts(cnts)

    def search(self, keys, vals_out, found_out):
        """Batched get of this rank's keys; results land in input order."""
        self.search_end(self.search_begin(keys), vals_out, found_out)

    def search_begin(self, keys):
        """First half of search(): bucketing and the count exchange, issued
        without waiting for them.  A pipelined caller begins batch i + 1
        before it ends batch i, so batch i + 1's counts are on the host by
        the time they are needed instead of queueing behind batch i's walk
        (bench.py, N > 1).  Every rank must begin and end the same batches
        in the same order (collectives)."""
        # the bucketed keys and permutation live in this router's buffers: one
        # batch in flight per router (bench.py alternates two routers)
        assert not self._pending, "ShardRouter: search_begin while a batch is in flight"
        self._pending = True
        return (keys,) + self._bucket_async(keys)

    def search_end(self, pending, vals_out, found_out):
        """Second half: key exchange, local batched get, value exchange,
        un-permute into vals_out / found_out (input order)."""
        keys, kb, perm, cnts = pending
        self._pending = False
        n, dev = keys.numel(), keys.device
        cnt, rcnt = self._counts(cnts)
        nrecv = sum(rcnt)
        recv = self._buf("recv", nrecv, torch.int64, dev)
        self._a2a(recv, kb, rcnt, cnt)
        rv = self._buf("rv", nrecv, torch.int64, dev)
        rf = self._buf("rf", nrecv, torch.uint8, dev)
        self.local.search_batch(recv, rv, rf)
        back = self._buf("back", n, torch.int64, dev)
        self._a2a(back, rv, cnt, rcnt)
        # value 0 is kValueNull: found <=> value != 0 (Tree.cpp:445-448),
        # written by the same un-permute pass
        self.local.route_unpermute(back, perm, vals_out, found=found_out)

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
        # queued without a host wait where the shard supports it (the
        # status surfaces at the shard's next synchronising call)
        getattr(self.local, "insert_batch_async", self.local.insert_batch)(rk, rv)

    def range_query(self, lo, hi):
        """Batched range scans [lo_i, hi_i] (inclusive, u64 held as int64).
        Returns (counts[n] int64, values): scan i's values are
        values[sum(counts[:i]) : sum(counts[:i+1])], in key order across shards
        (leaf order, then slot order, inside a shard)."""
        n, dev, P = lo.numel(), lo.device, self.world
        s0 = owner_of(lo, P)
        s1 = torch.maximum(owner_of(hi, P), s0)        # lo > hi: one empty piece
        s1 = torch.where((lo ^ _SIGN) > (hi ^ _SIGN), s0, s1)
        npc = s1 - s0 + 1
        total = int(npc.sum().item()) if n else 0
        scan = torch.repeat_interleave(torch.arange(n, device=dev), npc)
        first = torch.cumsum(npc, 0) - npc
        shard = s0[scan] + (torch.arange(total, device=dev) - first[scan])
        bnd = shard_bounds(P, dev)
        plo = umax(lo[scan], bnd[shard])
        last = torch.where(shard + 1 < P, bnd[(shard + 1).clamp(max=P - 1)] - 1, bnd[P])
        phi = umin(hi[scan], last)
        # bucket the pieces by owner (stable) and exchange their bounds
        kb, perm, cnt, rcnt = self._bucket(plo)
        hb = self._buf("rq_hb", total, torch.int64, dev)
        self.local.route_permute(phi, perm, hb)
        nrecv = sum(rcnt)
        rlo = self._buf("rq_rlo", nrecv, torch.int64, dev)
        rhi = self._buf("rq_rhi", nrecv, torch.int64, dev)
        self._a2a(rlo, kb, rcnt, cnt)
        self._a2a(rhi, hb, rcnt, cnt)
        rc, rv = self.local.range_query_batch(rlo, rhi)
        # counts back (piece order as sent), then values with per-rank splits
        bc = self._buf("rq_bc", total, torch.int64, dev)
        self._a2a(bc, rc.to(torch.int64), cnt, rcnt)
        seg = torch.repeat_interleave(torch.arange(P, device=dev),
                                      torch.tensor(rcnt, device=dev))
        vsend = torch.zeros(P, dtype=torch.int64, device=dev).index_add_(0, seg, rc.to(torch.int64))
        vrecv = self._buf("rq_vr", P, torch.int64, dev)
        self._a2a(vrecv, vsend)
        vs, vr = vsend.tolist(), vrecv.tolist()
        bv = self._buf("rq_bv", sum(vr), torch.int64, dev)
        self._a2a(bv, rv, vr, vs)
        # bucketed piece p is original piece perm[p]; reorder values to scan order
        pc = torch.empty(total, dtype=torch.int64, device=dev)
        pc[perm.long()] = bc
        src_off = torch.cumsum(bc, 0) - bc                # offsets in bv (bucketed order)
        src_of_orig = torch.empty(total, dtype=torch.int64, device=dev)
        src_of_orig[perm.long()] = src_off
        dst_off = torch.cumsum(pc, 0) - pc
        nv = int(pc.sum().item()) if total else 0
        shift = torch.repeat_interleave(src_of_orig - dst_off, pc)
        values = bv[torch.arange(nv, device=dev) + shift] if nv else bv[:0]
        counts = torch.zeros(n, dtype=torch.int64, device=dev).index_add_(0, scan, pc)
        return counts, values

