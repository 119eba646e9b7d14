"""N > 1 path with real GPU shards: sherman_amd.shard.ShardRouter over
sherman_amd.Tree (HIP, through the C-ABI) on cuda:0, checked against ONE
unsharded CPU oracle tree exactly as tests/test_multi_rank.py checks the
oracle-backed shards (routed inserts with cross-rank conflicts and deletes,
routed gets with misses, routed range scans across shard boundaries).

  * world 1 over the "nccl" backend (RCCL on ROCm): the exchange calls bench.py
    makes at N > 1 (all_to_all_single with split lists, int64 payloads) run
    through RCCL on the box's one GPU;
  * world 2 over "gloo" with CUDA tensors: two ranks, two trees sharing the
    GPU, each built with its shard's key-range hint, a real two-way exchange;
  * world 1 through the C-ABI shard (sherman_amd.CShard, shm_shard_* in
    csrc/shard.cpp): at world 1 its get and insert take the local path (no
    exchange; a one-shard batch is all the rank's own) and its range scan the
    1-rank exchange; two batches in flight (begin, begin, end, end);
  * the same with the routed path forced (shm__shard_force_route, "routed"):
    slot placement, the key / value / count exchange through grouped
    ncclSend / ncclRecv (each run sent by the rank to itself), the local
    batch, the results back and the gather -- every RCCL step of a world > 1
    get and insert, on the box's one GPU.

One GPU is all a gpurun box has, and RCCL refuses two ranks on one device, so
the RCCL exchange at world > 1 is covered by the driver's 8-GPU run; its
logic is the gloo one.
"""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_multi_rank import (free_port, query_batch, rank_batches, scan_batch,
                             verify_against_unsharded)

pytestmark = pytest.mark.gpu

U64 = np.uint64


def gpu_worker(rank, world, port, outdir, backend, cabi=False):
    routed = cabi == "routed"
    import sherman_amd as shm
    from sherman_amd.shard import ShardRouter, shard_range

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    kw = {"device_id": dev} if backend == "nccl" else {}
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}",
                            rank=rank, world_size=world, **kw)
    lo, bits = shard_range(rank, world)
    tree = shm.Tree(arena_bytes=64 << 20, max_batch=1 << 14, device=0, node_id=rank,
                    key_lo=lo, key_bits=bits)
    cs = shm.CShard(tree, world, rank, dist) if cabi else None
    if routed:
        cs.force_route(True)
    router = ShardRouter(tree, world, dist, cshard=cs)

    def d(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)

    for rnd in range(3):
        k, v = rank_batches(rank)[rnd]
        router.insert(d(k), d(v))
    q = query_batch(rank)
    vals = torch.empty(q.size, dtype=torch.int64, device=dev)
    found = torch.empty(q.size, dtype=torch.uint8, device=dev)
    router.search(d(q), vals, found)
    if cabi:
        # two batches in flight on two streams (the C shard's two slots)
        q1, q2 = d(q), d(q[::-1].copy())
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        s1.wait_stream(torch.cuda.current_stream())
        s2.wait_stream(torch.cuda.current_stream())
        v1, f1 = torch.empty_like(vals), torch.empty_like(found)
        v2, f2 = torch.empty_like(vals), torch.empty_like(found)
        with torch.cuda.stream(s1):
            p1 = router.search_begin(q1)
        with torch.cuda.stream(s2):
            p2 = router.search_begin(q2)
        router.search_end(p1, v1, f1)
        router.search_end(p2, v2, f2)
        torch.cuda.synchronize()
        assert torch.equal(v1, vals) and torch.equal(f1, found)
        assert torch.equal(v2, vals.flip(0)) and torch.equal(f2, found.flip(0))
    slo, shi = scan_batch(rank, world)
    counts, svals = router.range_query(d(slo), d(shi))
    if cabi:
        # the same scans with no host read-back (fixed runs per peer over the
        # transport: RCCL here), equal to the synchronous form
        ac, _, av, st = cs.range_query_async(d(slo), d(shi), vals_cap=1 << 18, peer_cap=1 << 17)
        torch.cuda.synchronize()
        tot, flags = (int(x) for x in st.cpu().tolist())
        assert flags == 0 and tot == svals.numel(), (tot, flags, svals.numel())
        assert torch.equal(ac, counts) and torch.equal(av[:tot], svals)
    torch.cuda.synchronize()
    rc = tree.check()["keys"]  # raises on a broken invariant
    keys, values = tree_contents(tree)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), keys=keys, values=values,
             vals=vals.cpu().numpy(), found=found.cpu().numpy(), check=np.array([rc]),
             scounts=counts.cpu().numpy(), svals=svals.cpu().numpy())
    if cs is not None:
        cs.close()
    tree.close()
    dist.barrier()
    dist.destroy_process_group()


def tree_contents(tree):
    """(keys, values) of every valid slot, read through the oracle over the
    tree's own page image (test infrastructure as the checker)."""
    from oracle.pyoracle import OracleTree
    img, root = tree.dump_image()
    orc = OracleTree(image=img, root_ptr=root, node_id=tree.node_id)
    k, v = orc.dump()
    orc.close()
    return k, v


@pytest.mark.parametrize("backend,world,cabi", [("nccl", 1, False), ("gloo", 2, False),
                                                ("nccl", 1, True), ("nccl", 1, "routed")])
def test_routed_gpu_shards_match_unsharded_oracle(backend, world, cabi):
    assert torch.cuda.is_available(), "GPU test without a GPU"
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(gpu_worker, args=(world, free_port(), d, backend, cabi), nprocs=world,
                 join=True)
        verify_against_unsharded(d, world)


def test_slot_padding_once_per_capacity():
    """The shard's placement pads its runs with kKeyMax only when a slot's
    capacity changes (shm__route_slots_ex fill); later batches leave earlier
    keys in the runs' tails.  Those must be keys of the run's own owner (so
    the owner's walk never sees a key outside its range), the counts each
    batch publishes must be its own (the claim words return to zero after
    every launch), and the gathered results must equal a plain search."""
    import ctypes

    import sherman_amd as shm
    from sherman_amd.shard import owner_of

    L = shm.lib()
    L.shm__route_slots_ex.restype = ctypes.c_int
    L.shm__route_slots_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                      ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    L.shm__route_gather.restype = ctypes.c_int
    L.shm__route_gather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    P = 8
    rng = np.random.default_rng(77)
    keys = np.unique(rng.integers(1, (1 << 64) - 2, 60000, dtype=np.uint64))
    t = shm.Tree(arena_bytes=64 << 20, max_batch=1 << 16)
    kd = torch.from_numpy(keys.view(np.int64)).to(dev)
    t.insert_batch(kd, kd ^ 0x77)
    cursor = torch.zeros(P + 1, dtype=torch.int32, device=dev)
    ovk = torch.zeros(1 << 15, dtype=torch.int64, device=dev)
    ovi = torch.zeros(1 << 15, dtype=torch.int32, device=dev)
    filled = None
    for rnd, n in enumerate([20000, 20000, 12000, 20000, 20000]):
        cap = n // P + 6 * int(np.sqrt(n // P)) + 256
        if filled is None or filled[0] != cap:
            slots = torch.empty(P * cap, dtype=torch.int64, device=dev)
            fill = 1
        else:
            slots, fill = filled[1], 0
        filled = (cap, slots)
        q = np.concatenate([keys[rng.integers(0, keys.size, n - 500)],
                            rng.integers(1, (1 << 64) - 2, 500, dtype=np.uint64)])
        qd = torch.from_numpy(q.view(np.int64)).to(dev)
        spos = torch.empty(n, dtype=torch.int32, device=dev)
        assert L.shm__route_slots_ex(t.h, qd.data_ptr(), n, P, cap, cursor.data_ptr(),
                                     slots.data_ptr(), spos.data_ptr(), ovk.data_ptr(),
                                     ovi.data_ptr(), fill, None) == 0
        res = torch.empty_like(slots)
        t.search_batch(slots, res)
        out = torch.empty(n, dtype=torch.int64, device=dev)
        fnd = torch.empty(n, dtype=torch.uint8, device=dev)
        assert L.shm__route_gather(res.data_ptr(), spos.data_ptr(), n, out.data_ptr(),
                                   fnd.data_ptr(), None) == 0
        v, f = torch.empty_like(qd), torch.empty(n, dtype=torch.uint8, device=dev)
        t.search_batch(qd, v, f)
        torch.cuda.synchronize()
        assert torch.equal(out, v) and torch.equal(fnd, f), rnd
        cur = cursor.cpu().numpy()
        qo = owner_of(qd.cpu(), P).numpy()
        assert np.array_equal(cur[:P], np.bincount(qo, minlength=P)), rnd  # this batch's own
        assert cur[P] == 0
        sl = slots.cpu().numpy().view(np.uint64).reshape(P, cap)
        so = owner_of(torch.from_numpy(sl.reshape(-1).view(np.int64)), P).numpy().reshape(P, cap)
        pad = sl == np.uint64((1 << 64) - 1)
        # every slot: kKeyMax padding or a key of the run's owner
        assert bool(np.all(pad | (so == np.arange(P)[:, None]))), rnd
    t.close()


@pytest.mark.parametrize("P", [2, 3, 8])
def test_slot_routed_get_p_shards_on_one_gpu(P):
    """The C-ABI shard's get placement for P > 1 without P ranks: P trees on
    cuda:0 (each with its shard's key-range hint), one batch of queries
    (hits, misses, a duplicate, key 0) placed into P runs of fixed-capacity
    slots (shm__route_slots), run p searched by tree p -- what the
    ncclAllToAll hands each rank -- and the results gathered back
    (shm__route_gather).  Every key lands in its owner's run, the runs'
    tails are kKeyMax, and the gathered values equal the unsharded dict.  A
    too-small capacity puts the overflowing keys on the overflow list (key
    and input position: what shm_shard_search_end's second round answers,
    test_local_group_p8_routed_paths); without a list they find nothing and
    kErrOverflow is reported."""
    import ctypes

    import sherman_amd as shm
    from sherman_amd.shard import owner_of, shard_range

    L = shm.lib()
    L.shm__route_slots.restype = ctypes.c_int
    L.shm__route_slots.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                   ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p]
    L.shm__route_gather.restype = ctypes.c_int
    L.shm__route_gather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    rng = np.random.default_rng(100 + P)
    keys = np.unique(rng.integers(1, (1 << 64) - 2, 30000, dtype=np.uint64))
    vals = keys ^ U64(0x5555)
    trees = []
    own = owner_of(torch.from_numpy(keys.view(np.int64)), P).numpy()
    for p in range(P):
        lo, bits = shard_range(p, P)
        t = shm.Tree(arena_bytes=32 << 20, max_batch=1 << 15, node_id=p, key_lo=lo,
                     key_bits=bits)
        kp = keys[own == p]
        t.insert_batch(torch.from_numpy(kp.view(np.int64)).to(dev),
                       torch.from_numpy(vals[own == p].view(np.int64)).to(dev))
        trees.append(t)
    q = np.concatenate([keys[rng.integers(0, keys.size, 20000)],
                        rng.integers(1, (1 << 64) - 2, 5000, dtype=np.uint64),  # misses
                        keys[:1], keys[:1], np.array([0], dtype=U64)])
    rng.shuffle(q)
    n = q.size
    qd = torch.from_numpy(q.view(np.int64)).to(dev)
    want = dict(zip(keys.tolist(), vals.tolist()))
    exp = np.array([want.get(int(x), 0) for x in q], dtype=U64)

    for cap, overflow, listed in (((n + n // 4) // P + 256, False, True),
                                  (n // (2 * P), True, True), (n // (2 * P), True, False)):
        cursor = torch.zeros(P + 1, dtype=torch.int32, device=dev)
        slots = torch.empty(P * cap, dtype=torch.int64, device=dev)
        spos = torch.empty(n, dtype=torch.int32, device=dev)
        ovk = torch.zeros(n, dtype=torch.int64, device=dev)
        ovi = torch.zeros(n, dtype=torch.int32, device=dev)
        rc = L.shm__route_slots(trees[0].h, qd.data_ptr(), n, P, cap, cursor.data_ptr(),
                                slots.data_ptr(), spos.data_ptr(),
                                ovk.data_ptr() if listed else None,
                                ovi.data_ptr() if listed else None, None)
        assert rc == 0
        res = torch.empty_like(slots)
        for p in range(P):
            fp = torch.empty(cap, dtype=torch.uint8, device=dev)
            trees[p].search_batch(slots[p * cap:(p + 1) * cap], res[p * cap:(p + 1) * cap], fp)
        out = torch.empty(n, dtype=torch.int64, device=dev)
        fnd = torch.empty(n, dtype=torch.uint8, device=dev)
        assert L.shm__route_gather(res.data_ptr(), spos.data_ptr(), n, out.data_ptr(),
                                   fnd.data_ptr(), None) == 0
        torch.cuda.synchronize()
        sl = slots.cpu().numpy().view(U64).reshape(P, cap)
        sp = spos.cpu().numpy().view(np.uint32)
        qo = owner_of(qd.cpu(), P).numpy()
        o = out.cpu().numpy().view(U64)
        f = fnd.cpu().numpy()
        placed = sp != 0xFFFFFFFF
        assert bool(placed.all()) != overflow
        # every placed key sits in its owner's run at the recorded slot
        assert np.array_equal(sl.reshape(-1)[sp[placed]], q[placed])
        assert np.array_equal(sp[placed] // cap, qo[placed])
        for p in range(P):
            c = int((placed & (qo == p)).sum())
            assert np.all(sl[p, c:] == U64((1 << 64) - 1))  # kKeyMax padding
        assert np.array_equal(o[placed], exp[placed])
        assert np.all(o[~placed] == 0) and np.array_equal(f, (o != 0).astype(np.uint8))
        cur = cursor.cpu().numpy()
        assert np.array_equal(cur[:P], np.bincount(qo, minlength=P))  # routed per peer
        if listed:
            # the overflow list: exactly the cut inputs, each with its key
            m = int(cur[P])
            assert m == int((~placed).sum())
            oi = ovi.cpu().numpy().view(np.uint32)[:m]
            assert np.array_equal(np.sort(oi), np.flatnonzero(~placed).astype(np.uint32))
            assert np.array_equal(ovk.cpu().numpy().view(U64)[:m], q[oi])
            trees[0].synchronize()  # nothing reported: the second round answers them
        elif overflow:
            with pytest.raises(shm.ShermanError):
                trees[0].synchronize()  # kErrOverflow reported by the next sync
    for t in trees:
        t.close()
