"""N>1 path on CPU: world_size-2 (and 3) gloo process groups driving
sherman_amd.shard.ShardRouter, the exchange logic bench.py runs over RCCL.

Each rank's shard is an oracle tree (test infrastructure) behind the same
five-method interface the GPU Tree exposes; bucketing is the stable
owner-partition the device kernel implements (checked bit-for-bit against
this restatement in test_gpu_parity.test_route_bucket_roundtrip).

Checked against ONE unsharded oracle tree:
  * routed inserts (duplicates inside a batch, the same key from several
    ranks, deletes as value 0) leave the union of the shards with exactly the
    contents of applying rank 0's batch, then rank 1's, ... in batch order;
  * every shard holds only keys of its own range;
  * routed gets (hits and misses) return the unsharded tree's answers in
    input order;
  * routed range scans (boundary-crossing, whole-space, empty, single-key)
    return the unsharded tree's values per scan.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.pyoracle import OracleTree, to_key
from sherman_amd.shard import ShardRouter, owner_of

U64 = np.uint64


class OracleShard:
    """CPU stand-in for sherman_amd.Tree's routing + batch methods."""

    def __init__(self):
        self.t = OracleTree(64 << 20)

    def route_bucket(self, keys, world, keys_out, perm_out, counts_out):
        own = owner_of(keys, world)
        order = torch.argsort(own, stable=True)
        keys_out.copy_(keys[order])
        perm_out.copy_(order.to(torch.int32))
        counts_out.copy_(torch.bincount(own, minlength=world))

    def route_permute(self, vals, perm, out):
        out.copy_(vals[perm.long()])

    def route_unpermute(self, vals, perm, out, found=None):
        out[perm.long()] = vals
        if found is not None:
            torch.ne(out, 0, out=found)

    def search_batch(self, keys, vals_out, found_out):
        v, f = self.t.search_batch(keys.numpy().view(U64))
        vals_out.copy_(torch.from_numpy(v.view(np.int64)))
        found_out.copy_(torch.from_numpy(f))

    def insert_batch(self, keys, vals):
        self.t.apply_batch(keys.numpy().view(U64), vals.numpy().view(U64))

    def range_query_batch(self, lo, hi):
        c, v = self.t.range_query_batch(lo.numpy().view(U64), hi.numpy().view(U64))
        return torch.from_numpy(c.view(np.int64)), torch.from_numpy(v.view(np.int64))


def rank_batches(rank, rounds=3, n=3000):
    """Insert batches of one rank: a key pool shared by all ranks (cross-rank
    conflicts), in-batch duplicates and some deletes."""
    rng = np.random.default_rng(100 + rank)
    pool = np.array([to_key(i) for i in range(1, 4001)], dtype=U64)
    out = []
    for r in range(rounds):
        k = pool[rng.integers(0, pool.size, n)]
        v = (np.arange(n, dtype=U64) + U64(1 + 10 ** 6 * (10 * rank + r)))
        v[rng.random(n) < 0.05] = 0  # deletes
        out.append((k, v))
    return out


def query_batch(rank, n=5000):
    rng = np.random.default_rng(900 + rank)
    ids = rng.integers(1, 6001, n)  # ids > 4000 never inserted: misses
    return np.array([to_key(int(i)) for i in ids], dtype=U64)


def scan_batch(rank, world, n=60):
    """Range scans of one rank: short and long spans, spans crossing one or
    several shard boundaries, the whole key space, lo > hi (empty), and
    single-key scans."""
    rng = np.random.default_rng(700 + rank)
    lo, hi = [], []
    top = (1 << 64) - 1
    bnd = [(s * (1 << 64) + world - 1) // world for s in range(1, world)] or [1 << 63]
    for i in range(n):
        c = i % 6
        if c == 0:
            a = int(rng.integers(0, 1 << 63)) * 2
            b = min(top, a + (1 << 58))
        elif c == 1:    # straddle a shard boundary
            m = bnd[int(rng.integers(0, len(bnd)))]
            a, b = m - (1 << 57), m + (1 << 57)
        elif c == 2:    # cover everything
            a, b = 0, top
        elif c == 3:    # inverted: empty
            a = int(rng.integers(1 << 40, 1 << 62))
            b = a - 1
        elif c == 4:    # one stored key exactly
            a = b = int(to_key(int(rng.integers(1, 4001))))
        else:           # from a boundary to the top
            a, b = bnd[-1], top
        lo.append(a)
        hi.append(b)
    return np.array(lo, dtype=U64), np.array(hi, dtype=U64)


def worker(rank, world, port, outdir):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}",
                            rank=rank, world_size=world)
    shard = OracleShard()
    router = ShardRouter(shard, world, dist)
    for rnd in range(3):
        # every rank inserts its round-rnd batch; rounds are separate batches
        k, v = rank_batches(rank)[rnd]
        router.insert(torch.from_numpy(k.view(np.int64)), torch.from_numpy(v.view(np.int64)))
    q = query_batch(rank)
    vals = torch.empty(q.size, dtype=torch.int64)
    found = torch.empty(q.size, dtype=torch.uint8)
    router.search(torch.from_numpy(q.view(np.int64)), vals, found)
    slo, shi = scan_batch(rank, world)
    counts, svals = router.range_query(torch.from_numpy(slo.view(np.int64)),
                                       torch.from_numpy(shi.view(np.int64)))
    keys, values = shard.t.dump()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), keys=keys, values=values,
             vals=vals.numpy(), found=found.numpy(), check=np.array([shard.t.check()[0]]),
             scounts=counts.numpy(), svals=svals.numpy())
    shard.t.close()
    dist.barrier()
    dist.destroy_process_group()


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_insert_and_get_match_unsharded_oracle(world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(worker, args=(world, free_port(), d), nprocs=world, join=True)
        verify_against_unsharded(d, world)


def verify_against_unsharded(d, world):
    """Compare the ranks' saved results (rank{r}.npz in `d`) with ONE
    unsharded oracle tree fed the same batches."""
    if True:
        res = [np.load(os.path.join(d, f"rank{r}.npz")) for r in range(world)]

        # expected: one tree, batches applied round by round, rank-major
        ref = OracleTree(64 << 20)
        batches = [rank_batches(r) for r in range(world)]
        for rnd in range(3):
            for r in range(world):
                ref.apply_batch(*batches[r][rnd])
        rk, rv = ref.dump()  # leaf order; slots inside a leaf are unsorted
        ro = np.argsort(rk)
        rk, rv = rk[ro], rv[ro]

        union_k = np.concatenate([x["keys"] for x in res])
        union_v = np.concatenate([x["values"] for x in res])
        o = np.argsort(union_k)
        assert np.array_equal(union_k[o], rk)
        assert np.array_equal(union_v[o], rv)
        for r, x in enumerate(res):
            assert int(x["check"][0]) >= 0
            own = owner_of(torch.from_numpy(x["keys"].view(np.int64)), world)
            assert bool((own == r).all())
            q = query_batch(r)
            ov, of = ref.search_batch(q)
            assert np.array_equal(x["vals"].view(U64), ov)
            assert np.array_equal(x["found"], of)
            # routed scans: per scan the unsharded tree's values (as a multiset:
            # slots inside a leaf are unsorted, and leaf boundaries differ)
            slo, shi = scan_batch(r, world)
            key_of = dict(zip(rv.tolist(), rk.tolist()))  # values are unique
            off = np.concatenate([[0], np.cumsum(x["scounts"])])
            assert off[-1] == x["svals"].size
            for i in range(slo.size):
                want, _ = ref.range_query(int(slo[i]), int(shi[i]))
                got = x["svals"][off[i]:off[i + 1]].view(U64)
                assert np.array_equal(np.sort(got), np.sort(want)), i
                # pieces come back in shard order (key order across shards)
                ks = np.array([key_of[v] for v in got.tolist()], dtype=U64)
                own = owner_of(torch.from_numpy(ks.view(np.int64)), world)
                assert bool((own[1:] >= own[:-1]).all()), i
        ref.close()
