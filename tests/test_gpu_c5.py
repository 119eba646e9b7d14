"""Config C5 (BASELINE.json configs[4]) on the HIP path: the write-heavy
stream on real GPU shards against ONE unsharded CPU oracle.

  * preload: key(i) = to_key(i) -> 2i for i in 1..2^20 (test/benchmark.cpp:
    269-274 without the modulus), each rank inserting its own range shard;
  * batches of 2^16 ops per rank: key = to_key(1 + zipf(0.99) over TWICE the
    preloaded ids) (mehcached zipf, test/zipf.h, oracle restatement), so about
    half of the inserts are new keys and leaves split; op = range scan iff
    rand_r % 100 < 5 (test/benchmark.cpp:173 with kReadRatio = 5), else an
    insert of value (global op index + 1);
  * scans [k, k + span], span ~ 100 stored keys, run before the batch's
    inserts (SURVEY §8a batch semantics): every rank's scans see the state
    after the previous batch, then the inserts of all ranks apply in
    rank-major order (routed inserts, sherman_amd/shard.py);
  * world 1 over RCCL ("nccl") and world 2 over gloo with two trees sharing
    the GPU (RCCL refuses two ranks on one device; the driver's 8-GPU run
    covers RCCL at world > 1), and world 1 through the C-ABI shard
    (sherman_amd.CShard: routed inserts and range scans in C++, shm_shard_*).

Checked: per scan the oracle's values (a multiset: slot order inside a leaf
and leaf boundaries after batched splits may differ), the final key->value
contents, the structural invariants of every shard, and that leaves split.
"""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_multi_rank import free_port

pytestmark = pytest.mark.gpu

U64 = np.uint64
N_PRE = 1 << 20
BATCH = 1 << 16
ROUNDS = 4
SCAN_PCT = 5


def c5_batch(rank, b, world):
    """(is_scan, ids) of rank's batch b (host arrays; keys are hashed on the
    device and on the oracle side identically)."""
    from oracle.pyoracle import op_mix, zipf_fill
    seed = 0x5EED0000 + 97 * rank + b
    ids = zipf_fill(2 * N_PRE * world, 0.99, seed, BATCH) + U64(1)
    is_scan = op_mix(1 + 31 * rank + b, SCAN_PCT, BATCH).astype(bool)
    return is_scan, ids


def span(world):
    return (1 << 64) // (N_PRE * world) * 100


def scan_bounds(keys, world):
    lo = keys.astype(U64)
    hi = lo + U64(span(world))
    hi[hi < lo] = U64((1 << 64) - 2)  # saturate
    hi[hi == U64((1 << 64) - 1)] = U64((1 << 64) - 2)
    return lo, hi


def op_values(rank, b, n):
    return (np.arange(n, dtype=U64) + U64((rank * ROUNDS + b) * BATCH + 1))


def gpu_worker(rank, world, port, outdir, backend, cabi=False):
    import sherman_amd as shm
    from oracle.pyoracle import to_key  # noqa: F401  (same generator family)
    from sherman_amd.shard import ShardRouter, owner_of, shard_range

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    kw = {"device_id": dev} if backend == "nccl" else {}
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}",
                            rank=rank, world_size=world, **kw)
    lo, bits = shard_range(rank, world)
    tree = shm.Tree(arena_bytes=512 << 20, max_batch=1 << 17, device=0, node_id=rank,
                    key_lo=lo, key_bits=bits)
    cs = shm.CShard(tree, world, rank, dist) if cabi else None
    router = ShardRouter(tree, world, dist, cshard=cs)
    # routed scans through the C shard: one piece-matrix width on every rank
    n_cap = max(int(c5_batch(r, b, world)[0].sum()) for r in range(world) for b in range(ROUNDS))
    # preload this rank's shard of key(1 .. N_PRE * world)
    total = N_PRE * world
    keys = torch.empty(total, dtype=torch.int64, device=dev)
    tree.gen_keys(1, total, keys)
    ids = torch.arange(1, total + 1, dtype=torch.int64, device=dev)
    mine = owner_of(keys, world) == rank
    pk, pv = keys[mine].contiguous(), (ids[mine] * 2).contiguous()
    for c in range(0, pk.numel(), 1 << 17):
        tree.insert_batch(pk[c:c + (1 << 17)], pv[c:c + (1 << 17)])
    pages0 = tree.stats()["pages_used"]
    out = {}
    for b in range(ROUNDS):
        is_scan, bid = c5_batch(rank, b, world)
        k = torch.empty(BATCH, dtype=torch.int64, device=dev)
        tree.hash_keys(torch.from_numpy(bid.view(np.int64)).to(dev), k)
        kh = k.cpu().numpy().view(U64)
        slo, shi = scan_bounds(kh[is_scan], world)
        counts, svals = router.range_query(torch.from_numpy(slo.view(np.int64)).to(dev),
                                           torch.from_numpy(shi.view(np.int64)).to(dev), n_cap)
        ik = torch.from_numpy(kh[~is_scan].view(np.int64)).to(dev)
        iv = torch.from_numpy(op_values(rank, b, int((~is_scan).sum())).view(np.int64)).to(dev)
        router.insert(ik, iv)
        out[f"scounts{b}"] = counts.cpu().numpy()
        out[f"svals{b}"] = svals.cpu().numpy()
        out[f"keys{b}"] = kh
    router.synchronize()
    st = tree.check()  # raises on a broken invariant
    from test_gpu_shard import tree_contents
    ck, cv = tree_contents(tree)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), ck=ck, cv=cv,
             grew=np.array([tree.stats()["pages_used"] - pages0, st["keys"]]), **out)
    if cs is not None:
        cs.close()
    tree.close()
    dist.barrier()
    dist.destroy_process_group()


def verify(d, world):
    from oracle.pyoracle import OracleTree, to_key
    res = [np.load(os.path.join(d, f"rank{r}.npz")) for r in range(world)]
    total = N_PRE * world
    ref = OracleTree(2 << 30)
    pre = np.array([to_key(i) for i in range(1, total + 1)], dtype=U64)
    ref.apply_batch(pre, np.arange(1, total + 1, dtype=U64) * U64(2))
    for b in range(ROUNDS):
        # every rank's scans see the state after batch b - 1 ...
        for r, x in enumerate(res):
            is_scan, _ = c5_batch(r, b, world)
            kh = x[f"keys{b}"]
            slo, shi = scan_bounds(kh[is_scan], world)
            oc, ov = ref.range_query_batch(slo, shi)
            gc = x[f"scounts{b}"]
            assert np.array_equal(oc.astype(np.int64), gc), (r, b)
            goff = np.concatenate([[0], np.cumsum(gc)])
            ooff = np.concatenate([[0], np.cumsum(oc)]).astype(np.int64)
            gv = x[f"svals{b}"].view(U64)
            for i in range(slo.size):
                assert np.array_equal(np.sort(gv[goff[i]:goff[i + 1]]),
                                      np.sort(ov[ooff[i]:ooff[i + 1]])), (r, b, i)
        # ... then the inserts of all ranks, rank-major
        for r, x in enumerate(res):
            is_scan, _ = c5_batch(r, b, world)
            kh = x[f"keys{b}"][~is_scan]
            ref.apply_batch(kh, op_values(r, b, kh.size))
    rk, rv = ref.dump()
    o = np.argsort(rk)
    uk = np.concatenate([x["ck"] for x in res])
    uv = np.concatenate([x["cv"] for x in res])
    u = np.argsort(uk)
    assert np.array_equal(uk[u], rk[o])
    assert np.array_equal(uv[u], rv[o])
    assert sum(int(x["grew"][0]) for x in res) > 0, "no leaf split in the C5 stream"
    assert sum(int(x["grew"][1]) for x in res) == rk.size
    ref.close()


@pytest.mark.parametrize("backend,world,cabi", [("nccl", 1, False), ("gloo", 2, False),
                                                ("nccl", 1, True)])
def test_c5_stream_on_gpu_shards_matches_unsharded_oracle(backend, world, cabi):
    assert torch.cuda.is_available(), "GPU test without a GPU"
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(gpu_worker, args=(world, free_port(), d, backend, cabi), nprocs=world,
                 join=True)
        verify(d, world)
