"""The C-ABI shard's whole routed path at P = 8 on the one GPU of a test box.

RCCL refuses two ranks on one device, so the 8-GPU exchange itself is the
driver's.  Everything around it — csrc/shard.cpp's slot placement, the
overflow rounds of gets and inserts, the padded insert slots, the range
pieces, the one read-back per scan batch, the gathers — runs here unchanged
at P = 8: eight shm_tree shards on cuda:0, eight host threads (one per rank,
ctypes releases the GIL), and the library's in-process transport, whose
collectives are device copies between the ranks' buffers (the shard's
transport interface; shm__shard_create_local).  All ranks queue on one
stream, as the trees' persistent kernels must not share the device.

Checked against ONE unsharded CPU oracle tree (test infrastructure):
  * three rounds of routed inserts with cross-rank conflicts, in-batch
    duplicates and deletes, then a round whose every key belongs to shard 0
    (each rank's run passes its slot of max_batch / P: the tails go in the
    second round, applied before anything else; a rank re-writes some of its
    keys inside the batch, head and tail): contents = the rank-major
    application of every rank's batches;
  * a round in which rank 3's batch holds kKeyMax: that batch is rejected
    whole on the sending rank (nothing of it reaches any shard, SHM_EINVAL at
    rank 3's next synchronising call) while the other ranks' batches apply,
    as a local insert rejects the chunk holding kKeyMax;
  * routed gets of a uniform batch, of a zipf(0.99) batch (the hot key's
    shard passes its slot of n / P + 6 sqrt(n / P) + 256) and of a batch whose every key
    belongs to shard 0 (7/8 of it overflows): every value returned, no key
    dropped; two batches in flight (begin, begin, end, end);
  * routed range scans across shard boundaries (whole key space, empty,
    single key): per scan the unsharded tree's values in key order across
    shards.
"""
import threading

import numpy as np
import pytest
import torch

from test_multi_rank import query_batch, rank_batches, scan_batch

pytestmark = pytest.mark.gpu

U64 = np.uint64
P = 8
MAX_BATCH = 8192


def skew_batch(rank, n=2000):
    """Keys all owned by shard 0 (top 3 bits 0), distinct across ranks; the
    first 300 are written again at the end of the batch (head, then tail)."""
    k = np.arange(n, dtype=U64) + U64(1 + 100000 * rank)
    k[n - 300:] = k[:300]
    v = np.arange(n, dtype=U64) + U64(5 * 10 ** 8 + 10 ** 6 * rank)
    return k, v


KM_RANK = 3


def keymax_batch(rank):
    """Five keys per rank spread over the shards; rank KM_RANK's batch also
    holds kKeyMax (rejected whole)."""
    k = (np.arange(5, dtype=U64) * U64(0x3333333333333333)) + U64(777 + rank)
    v = np.arange(5, dtype=U64) + U64(9 * 10 ** 8 + 10 ** 3 * rank)
    if rank == KM_RANK:
        k = np.concatenate([k[:2], np.array([(1 << 64) - 1], dtype=U64), k[2:]])
        v = np.concatenate([v[:2], np.array([1], dtype=U64), v[2:]])
    return k, v


def zipf_ids(rank, n, items=4000, theta=0.99):
    rng = np.random.default_rng(4242 + rank)
    p = 1.0 / np.arange(1, items + 1) ** theta
    return rng.choice(np.arange(1, items + 1), size=n, p=p / p.sum())


def rank_queries(rank):
    from oracle.pyoracle import to_key
    zq = np.array([to_key(int(i)) for i in zipf_ids(rank, 8000)], dtype=U64)
    sq = np.arange(8000, dtype=U64) + U64(1 + 100000 * rank)  # shard 0 only, hits
    return {"uniform": query_batch(rank), "zipf": zq, "shard0": sq}


def narrow_scans(rank, n=40):
    from oracle.pyoracle import to_key
    rng = np.random.default_rng(31 + rank)
    lo = np.array([to_key(int(i)) for i in rng.integers(1, 4001, n)], dtype=U64)
    hi = lo + U64(1 << 54)
    hi[hi < lo] = U64((1 << 64) - 2)
    return lo, hi


def run_rank(r, trees, group, stream, out, errs):
    import sherman_amd as shm
    try:
        dev = torch.device("cuda:0")

        def d(a):
            return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)

        with torch.cuda.stream(stream):
            cs = shm.CShard.local(trees[r], group, r)
            for rnd in range(3):
                k, v = rank_batches(r)[rnd]
                cs.insert(d(k), d(v), stream=stream)
            k, v = skew_batch(r)
            cs.insert(d(k), d(v), stream=stream)
            k, v = keymax_batch(r)
            cs.insert(d(k), d(v), stream=stream)
            km = None
            if r == KM_RANK:
                try:
                    cs.synchronize()
                except shm.ShermanError as e:
                    km = e.rc
            res = {}
            for name, q in rank_queries(r).items():
                vals = torch.empty(q.size, dtype=torch.int64, device=dev)
                found = torch.empty(q.size, dtype=torch.uint8, device=dev)
                cs.search(d(q), vals, found, stream=stream)
                res[name] = (vals, found)
            # two batches in flight through the two search slots
            q1, q2 = d(rank_queries(r)["zipf"]), d(rank_queries(r)["shard0"])
            v1, f1 = torch.empty_like(q1), torch.empty(q1.numel(), dtype=torch.uint8, device=dev)
            v2, f2 = torch.empty_like(q2), torch.empty(q2.numel(), dtype=torch.uint8, device=dev)
            t1 = cs.search_begin(q1, stream=stream)
            t2 = cs.search_begin(q2, stream=stream)
            cs.search_end(t1, v1, f1)
            cs.search_end(t2, v2, f2)
            res["inflight_zipf"], res["inflight_shard0"] = (v1, f1), (v2, f2)
            scans = {}
            for name, (lo, hi) in (("wide", scan_batch(r, P)), ("narrow", narrow_scans(r))):
                c, sv = cs.range_query(d(lo), d(hi), n_cap=64, stream=stream)
                scans[name] = (c, sv)
            # the same scans with no host read-back (fixed runs per peer), and
            # once with runs too short for them (flagged, not silently cut)
            asy = {}
            for name, (lo, hi) in (("wide", scan_batch(r, P)), ("narrow", narrow_scans(r))):
                ac, _, av, st = cs.range_query_async(d(lo), d(hi), vals_cap=1 << 19,
                                                     peer_cap=1 << 18, n_cap=64, stream=stream)
                asy[name] = (ac, av, st)
            lo, hi = scan_batch(r, P)
            _, _, _, st_short = cs.range_query_async(d(lo), d(hi), vals_cap=1 << 16, peer_cap=1,
                                                     n_cap=64, stream=stream)
            cs.synchronize()
            stream.synchronize()
            out[r] = ({k: (a.cpu().numpy().view(U64), b.cpu().numpy()) for k, (a, b) in res.items()},
                      {k: (a.cpu().numpy(), b.cpu().numpy().view(U64)) for k, (a, b) in scans.items()},
                      km,
                      {k: (a.cpu().numpy(), b.cpu().numpy().view(U64), c.cpu().numpy())
                       for k, (a, b, c) in asy.items()},
                      st_short.cpu().numpy())
            cs.close()
    except BaseException as e:  # noqa: BLE001 - reported by the main thread
        errs.append((r, repr(e)))


def test_local_group_p8_routed_paths():
    import sherman_amd as shm
    from oracle.pyoracle import OracleTree
    from sherman_amd.shard import owner_of, shard_range
    from test_gpu_shard import tree_contents

    assert torch.cuda.is_available(), "GPU test without a GPU"
    torch.cuda.set_device(0)
    trees = []
    for r in range(P):
        lo, bits = shard_range(r, P)
        trees.append(shm.Tree(arena_bytes=32 << 20, max_batch=MAX_BATCH, device=0, node_id=r,
                              key_lo=lo, key_bits=bits))
    group = shm.LocalGroup(P)
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    out, errs = [None] * P, []
    th = [threading.Thread(target=run_rank, args=(r, trees, group, stream, out, errs))
          for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank thread hung"
    assert not errs, errs
    torch.cuda.synchronize()

    # expected: one tree, the rounds rank-major, then the shard-0 round
    ref = OracleTree(64 << 20)
    for rnd in range(3):
        for r in range(P):
            ref.apply_batch(*rank_batches(r)[rnd])
    for r in range(P):
        ref.apply_batch(*skew_batch(r))
    for r in range(P):
        if r != KM_RANK:
            ref.apply_batch(*keymax_batch(r))
    assert out[KM_RANK][2] == shm.SHM_EINVAL, out[KM_RANK][2]
    rk, rv = ref.dump()
    o = np.argsort(rk)
    rk, rv = rk[o], rv[o]
    ks, vs = [], []
    for r, t in enumerate(trees):
        assert t.check()["keys"] >= 0
        k, v = tree_contents(t)
        own = owner_of(torch.from_numpy(k.view(np.int64)), P)
        assert bool((own == r).all())
        ks.append(k)
        vs.append(v)
    uk, uv = np.concatenate(ks), np.concatenate(vs)
    o = np.argsort(uk)
    assert np.array_equal(uk[o], rk)
    assert np.array_equal(uv[o], rv)
    key_of = dict(zip(rv.tolist(), rk.tolist()))
    for r in range(P):
        res, scans, _, asy, st_short = out[r]
        for name, (c, sv) in scans.items():
            ac, av, st = asy[name]
            assert st[1] == 0 and st[0] == sv.size, (r, name, st)
            assert np.array_equal(ac, c) and np.array_equal(av[:sv.size], sv), (r, name)
        assert st_short[1] & 1, (r, st_short)  # runs past peer_cap are flagged
        qs = rank_queries(r)
        for name, q in list(qs.items()) + [("inflight_zipf", qs["zipf"]),
                                            ("inflight_shard0", qs["shard0"])]:
            ov, of = ref.search_batch(q)
            gv, gf = res[name]
            assert np.array_equal(gv, ov), (r, name, int((gv != ov).sum()))
            assert np.array_equal(gf, of), (r, name)
        for name, (lo, hi) in (("wide", scan_batch(r, P)), ("narrow", narrow_scans(r))):
            c, sv = scans[name]
            off = np.concatenate([[0], np.cumsum(c)])
            assert off[-1] == sv.size
            for i in range(lo.size):
                want, _ = ref.range_query(int(lo[i]), int(hi[i]))
                got = sv[off[i]:off[i + 1]]
                assert np.array_equal(np.sort(got), np.sort(want)), (r, name, i)
                kk = np.array([key_of[x] for x in got.tolist()], dtype=U64)
                own = owner_of(torch.from_numpy(kk.view(np.int64)), P)
                assert bool((own[1:] >= own[:-1]).all()), (r, name, i)
    ref.close()
    group.close()
    for t in trees:
        t.close()


FZ_P = 4
FZ_ROUNDS = 12


def fuzz_round_batches(rank, rnd, pool):
    """Rank rank's round-rnd batch: keys drawn from a shared pool (so ranks
    collide), a skewed slice owned by one shard, deletes (value 0)."""
    rng = np.random.default_rng(1000 * rnd + rank)
    n = int(rng.integers(200, 3000))
    k = pool[rng.integers(0, pool.size, n)]
    hot = np.uint64(rng.integers(0, FZ_P)) << np.uint64(62)  # one shard's range
    k[: n // 5] = hot | (k[: n // 5] & np.uint64((1 << 62) - 1))
    v = rng.integers(1, 1 << 40, n, dtype=np.uint64)
    v[rng.random(n) < 0.1] = 0
    return k, v


def fuzz_rank(r, trees, group, stream, pool, out, errs):
    import sherman_amd as shm
    try:
        dev = torch.device("cuda:0")

        def d(a):
            return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)

        res = []
        with torch.cuda.stream(stream):
            cs = shm.CShard.local(trees[r], group, r)
            for rnd in range(FZ_ROUNDS):
                k, v = fuzz_round_batches(r, rnd, pool)
                cs.insert(d(k), d(v), stream=stream)
                # every rank passes the same get batch size (the slots' size
                # derives from it: include/sherman_amd.h), different keys
                nq = int(np.random.default_rng(7000 + rnd).integers(100, 4000))
                rng = np.random.default_rng(5000 + 100 * rnd + r)
                q = pool[rng.integers(0, pool.size, nq)]
                vals = torch.empty(q.size, dtype=torch.int64, device=dev)
                found = torch.empty(q.size, dtype=torch.uint8, device=dev)
                cs.search(d(q), vals, found, stream=stream)
                scan = None
                if rnd % 3 == 2:
                    lo = np.sort(pool[rng.integers(0, pool.size, 16)])
                    hi = lo + np.uint64(1 << 58)
                    hi[hi < lo] = np.uint64((1 << 64) - 2)
                    ac, _, av, st = cs.range_query_async(d(lo), d(hi), vals_cap=1 << 16,
                                                         peer_cap=1 << 15, n_cap=64, stream=stream)
                    scan = (lo, hi, ac, av, st)
                cs.synchronize()
                stream.synchronize()
                res.append((q, vals.cpu().numpy().view(U64), found.cpu().numpy(),
                            None if scan is None else
                            (scan[0], scan[1], scan[2].cpu().numpy().view(U64),
                             scan[3].cpu().numpy().view(U64), scan[4].cpu().numpy())))
            cs.close()
        out[r] = res
    except BaseException as e:  # noqa: BLE001 - reported by the main thread
        errs.append((r, repr(e)))


def test_local_group_random_rounds_vs_oracle():
    """Twelve rounds at P = 4 on the in-process transport: every rank inserts
    a random batch (keys from one shared pool, so ranks collide; a fifth of
    each batch forced into one shard's range, which overflows its slot; 10 %
    deletes), then gets a random batch, and every third round scans with the
    no-read-back form.  After each round every rank's gets and scans equal
    one unsharded oracle that applied the round's batches rank-major."""
    import sherman_amd as shm
    from oracle.pyoracle import OracleTree
    from sherman_amd.shard import shard_range

    assert torch.cuda.is_available(), "GPU test without a GPU"
    torch.cuda.set_device(0)
    rng = np.random.default_rng(99)
    pool = np.unique(rng.integers(1, (1 << 64) - 2, 20000, dtype=np.uint64))
    trees = []
    for r in range(FZ_P):
        lo, bits = shard_range(r, FZ_P)
        trees.append(shm.Tree(arena_bytes=32 << 20, max_batch=MAX_BATCH, device=0, node_id=r,
                              key_lo=lo, key_bits=bits))
    group = shm.LocalGroup(FZ_P)
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    out, errs = [None] * FZ_P, []
    th = [threading.Thread(target=fuzz_rank, args=(r, trees, group, stream, pool, out, errs))
          for r in range(FZ_P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank thread hung"
    assert not errs, errs
    ref = OracleTree(64 << 20)
    for rnd in range(FZ_ROUNDS):
        for r in range(FZ_P):
            ref.apply_batch(*fuzz_round_batches(r, rnd, pool))
        for r in range(FZ_P):
            q, gv, gf, scan = out[r][rnd]
            ov, of = ref.search_batch(q)
            assert np.array_equal(gv, ov) and np.array_equal(gf, of), (rnd, r)
            if scan is not None:
                lo, hi, c, v, st = scan
                assert st[1] == 0, (rnd, r, st)
                oc, ovv = ref.range_query_batch(lo, hi)
                assert np.array_equal(c, oc), (rnd, r)
                assert int(st[0]) == ovv.size, (rnd, r)
                # per scan the same values (the sharded trees' leaves hold
                # them in another slot order than the one oracle tree's)
                off = np.concatenate([[0], np.cumsum(oc)]).astype(np.int64)
                for i in range(lo.size):
                    a_, b_ = off[i], off[i + 1]
                    assert np.array_equal(np.sort(v[a_:b_]), np.sort(ovv[a_:b_])), (rnd, r, i)
    ref.close()
    group.close()
    for t in trees:
        assert t.check()["keys"] >= 0
        t.close()
