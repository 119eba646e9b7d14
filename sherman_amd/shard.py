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

With `cshard` (a sherman_amd.CShard) the get, insert and range routes run in
C++ behind the C-ABI (include/sherman_amd.h shm_shard_*, csrc/shard.cpp)
over their own RCCL communicators, and this class only forwards to them; the
Python exchange below remains the logic the gloo tests check.
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
    def __init__(self, local, world, dist, group=None, cshard=None):
        self.local, self.world, self.dist, self.group = local, world, dist, group
        self.cshard = cshard
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
        if self.cshard is not None:
            self.cshard.search(keys, vals_out, found_out)
            return
        self.search_end(self.search_begin(keys), vals_out, found_out)

    def search_begin(self, keys):
        """First half of search(): bucketing and the count exchange, issued
        without waiting for them.  A pipelined caller begins batch i + 1
        before it ends batch i, so batch i + 1's counts are on the host by
        the time they are needed instead of queueing behind batch i's walk
        (bench.py, N > 1).  Every rank must begin and end the same batches
        in the same order (collectives)."""
        if self.cshard is not None:  # two batches in flight per C shard
            return ("cabi", keys, self.cshard.search_begin(keys))
        # the bucketed keys and permutation live in this router's buffers: one
        # batch in flight per router (bench.py alternates two routers)
        assert not self._pending, "ShardRouter: search_begin while a batch is in flight"
        self._pending = True
        return (keys,) + self._bucket_async(keys)

    def search_end(self, pending, vals_out, found_out):
        """Second half: key exchange, local batched get, value exchange,
        un-permute into vals_out / found_out (input order)."""
        if pending[0] == "cabi":
            self.cshard.search_end(pending[2], vals_out, found_out)
            return
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

    def synchronize(self):
        """Status of every routed batch (the C shard first applies what its
        last insert left for the next call)."""
        if self.cshard is not None:
            self.cshard.synchronize()
        else:
            self.local.synchronize()

    def insert(self, keys, vals):
        """Batched insert (value 0 deletes) of this rank's (key, value) pairs."""
        if self.cshard is not None:
            self.cshard.insert(keys, vals)
            return
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

    def range_query(self, lo, hi, n_cap=None):
        """Batched range scans [lo_i, hi_i] (inclusive, u64 held as int64).
        Returns (counts[n] int64, values): scan i's values are
        values[sum(counts[:i]) : sum(counts[:i+1])], in key order across shards
        (leaf order, then slot order, inside a shard).  n_cap (C shard only):
        the same on every rank, >= n (shm_shard_range_query).

        Every scan is cut into P pieces, piece s = its overlap with shard s
        (empty, lo > hi, where it misses the shard), and row s of the P x n
        piece matrix goes to rank s: no bucketing and no key-count exchange.
        Host synchronisations: the ranks' scan counts (the receive splits) and
        the ranks' value totals (the value splits), each one read-back."""
        if self.cshard is not None:
            return self.cshard.range_query(lo, hi, n_cap)
        n, dev, P = lo.numel(), lo.device, self.world
        bnd = shard_bounds(P, dev)
        first = bnd[:P]
        last = torch.cat([bnd[1:P] - 1, bnd[P:P + 1]])  # inclusive top of shard s
        plo = umax(lo.unsqueeze(0).expand(P, n), first.unsqueeze(1).expand(P, n)).contiguous()
        phi = umin(hi.unsqueeze(0).expand(P, n), last.unsqueeze(1).expand(P, n)).contiguous()
        # scan counts of every rank (receive splits)
        cn = torch.full((2 * P,), n, dtype=torch.int64, device=dev)
        self._a2a(cn[P:], cn[:P])
        nr = self._counts(cn)[1]
        nrecv = sum(nr)
        rlo = self._buf("rq_rlo", nrecv, torch.int64, dev)
        rhi = self._buf("rq_rhi", nrecv, torch.int64, dev)
        self._a2a(rlo, plo.view(-1), nr, [n] * P)
        self._a2a(rhi, phi.view(-1), nr, [n] * P)
        rc, rv = self.local.range_query_batch(rlo, rhi)
        rc = rc.to(torch.int64)
        # counts back: row s of c = this rank's piece counts on shard s
        c = self._buf("rq_bc", P * n, torch.int64, dev)
        self._a2a(c, rc, [n] * P, nr)
        # value totals per peer (sent, received), one read-back for both
        seg = torch.repeat_interleave(torch.arange(P, device=dev),
                                      torch.tensor(nr, device=dev))
        vt = torch.zeros(2 * P, dtype=torch.int64, device=dev)
        vt[:P].index_add_(0, seg, rc)
        self._a2a(vt[P:], vt[:P].clone())
        vs, vr = self._counts(vt)
        nv = sum(vr)
        bv = self._buf("rq_bv", nv, torch.int64, dev)
        self._a2a(bv, rv, vr, vs)
        # bv holds piece (s, i) at src_off[s, i] (shard-major); scan i takes
        # its pieces s = 0 .. P - 1 in that order (key order across shards)
        c = c.view(P, n)
        src_off = (torch.cumsum(c.reshape(-1), 0) - c.reshape(-1)).view(P, n)
        ct = c.t().contiguous()                       # [n, P], scan-major
        dst_off = (torch.cumsum(ct.reshape(-1), 0) - ct.reshape(-1))
        shift = torch.repeat_interleave(src_off.t().reshape(-1) - dst_off, ct.reshape(-1),
                                        output_size=nv)
        values = bv[torch.arange(nv, device=dev) + shift] if nv else bv[:0]
        counts = ct.sum(1)
        return counts, values
