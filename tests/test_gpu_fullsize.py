"""GPU parity at the benchmark's own sizes.

C2 at full scale: 2^26 keys key(i) -> 2i and a 2^20-query uniform batch with
~9 % misses, checked against the key stream (the values that were written,
test/benchmark.cpp:43-46 and :165-188), not against the tree's own image.
C3 at 2^22 keys: zipf(0.99) 50 % get / 50 % insert batches of 2^20 ops
through shm_mixed_batch, every get and the final contents against the
oracle's Tree::search / Tree::insert over the GPU's own page image.

All GPU work runs in this one process.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import sherman_amd as shm  # noqa: E402
from oracle.pyoracle import OracleTree, op_mix, zipf_fill  # noqa: E402

U64 = np.uint64


def host(t):
    return t.cpu().numpy().view(U64)


@pytest.fixture(scope="module")
def lib_ok():
    assert torch.cuda.is_available(), "GPU test without a GPU"
    shm.lib()
    return True


def build_stream(t, n, chunk=1 << 20):
    """key(i) -> 2i for i = 1..n, inserted in key-stream order in chunks."""
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    t.gen_keys(1, n, keys)
    vals = torch.arange(1, n + 1, device="cuda", dtype=torch.int64) * 2
    for c in range(0, n, chunk):
        t.insert_batch(keys[c:c + chunk], vals[c:c + chunk])
    return keys, vals


def test_c2_full_size_get_parity(lib_ok):
    """Config C2 as the bench runs it: 2^26 keys, a 2^20-query uniform batch
    (queries key(1 + u), u uniform over the key count) whose every get must
    return 2i, and the same batch with ~9 % of its queries replaced by
    never-stored keys (ids past 2^26), each of which must miss with value 0
    (Tree.cpp:445-448); the stored key count and the B-link invariants
    (shm_check) hold."""
    n, b = 1 << 26, 1 << 20
    t = shm.Tree(arena_bytes=4 << 30, max_batch=1 << 20)
    keys, _ = build_stream(t, n)
    st = t.check()
    assert st["keys"] == n, st
    g = torch.Generator(device="cuda")
    g.manual_seed(26)
    qi = torch.randint(0, n, (b,), device="cuda", generator=g, dtype=torch.int64)
    q = keys[qi]
    v = torch.empty_like(q)
    f = torch.empty(b, dtype=torch.uint8, device="cuda")
    # the form the bench's timed steps walk: the read phase's pair-form
    # directory (four searches without an insert, tree.cpp kReadPhase)
    for _ in range(4):
        t.search_batch(q, v, f)
    t.profile(False, index_stats=True)
    t.search_batch(q, v, f)
    t.synchronize()
    idx = t.index_stats()
    t.profile(False)
    d = t.dir_stats()
    assert d["form"] == "pairs" and d["entries"] == 1 << 25, d
    assert idx["gets"] == b and idx["dir_fp_hits"] == b, idx  # every get from its entry
    want = (qi + 1) * 2
    assert bool(f.all()), int((f == 0).sum())
    assert torch.equal(v, want), int((v != want).sum())
    miss = torch.rand(b, device="cuda", generator=g) < 0.09
    m = int(miss.sum())
    mk = torch.empty(m, dtype=torch.int64, device="cuda")
    t.gen_keys(n + 1, m, mk)
    assert not bool(torch.isin(mk, keys).any())  # the key stream has no collision here
    q2 = q.clone()
    q2[miss] = mk
    t.search_batch(q2, v, f)
    t.synchronize()
    want2 = torch.where(miss, torch.zeros_like(want), want)
    assert torch.equal(v, want2), int((v != want2).sum())
    assert torch.equal(f.bool(), ~miss)
    # split-heavy chunks of new keys at full size (key(i) for ids past 2^26,
    # value 2i), a get batch after each (the gets that make the chunks keep
    # the directory: tree.cpp insert_apply's policy), then gets before any
    # rebuild: the chunks kept the pair-form entries (dir_upkeep.h), so every
    # stored key is still answered exactly -- old, new and their moved slots
    # -- with no rebuild
    builds = d["builds"]
    pages = t.stats()["pages_used"]
    nk = torch.empty(4 << 20, dtype=torch.int64, device="cuda")
    t.gen_keys(n + 1, nk.numel(), nk)
    nv = torch.arange(n + 1, n + 1 + nk.numel(), device="cuda", dtype=torch.int64) * 2
    for c in range(0, nk.numel(), 1 << 20):
        t.insert_batch(nk[c:c + (1 << 20)], nv[c:c + (1 << 20)])
        t.search_batch(nk[c:c + (1 << 20)], v, f)
        t.synchronize()
        assert torch.equal(v, nv[c:c + (1 << 20)]) and bool(f.all())
    assert t.stats()["pages_used"] > pages + 10000  # leaves split
    t.profile(False, index_stats=True)
    t.search_batch(q, v, f)  # the old keys
    t.synchronize()
    assert torch.equal(v, want) and bool(f.all())
    sel = torch.randint(0, nk.numel(), (b,), device="cuda", generator=g)
    t.search_batch(nk[sel], v, f)  # the new ones
    t.synchronize()
    idx = t.index_stats()
    t.profile(False)
    assert torch.equal(v, nv[sel]) and bool(f.all())
    d2 = t.dir_stats()
    assert d2["builds"] == builds and d2["form"] == "pairs" and d2["exact"], d2
    assert idx["dir_fp_hits"] >= 0.95 * idx["gets"], idx
    t.close()


def test_c3_2p22_mixed_vs_oracle_on_gpu_image(lib_ok):
    """Config C3's mix at 2^22 keys: the GPU tree is built from the key
    stream and its page image loaded into the oracle, then three zipf(0.99)
    batches of 2^20 ops (get iff rand_r % 100 < 50, insert value = op index
    + 1) run through shm_mixed_batch.  Each batch's gets must equal the
    oracle's Tree::search before the batch's inserts; the inserts apply in
    batch order (last writer wins); the final contents equal the oracle's."""
    n, b = 1 << 22, 1 << 20
    t = shm.Tree(arena_bytes=1 << 30, max_batch=1 << 20)
    build_stream(t, n)
    t.synchronize()
    img, root = t.dump_image()
    orc = OracleTree(image=img, root_ptr=root, node_id=t.node_id, spare_bytes=64 << 20)
    del img
    for r in range(3):
        ids = zipf_fill(n, 0.99, 0x5EED0000 + r, b) + U64(1)
        dids = torch.from_numpy(ids.view(np.int64)).cuda()
        dkeys = torch.empty_like(dids)
        t.hash_keys(dids, dkeys)  # device CityHash = oracle to_key (test_device_cityhash_...)
        keys = host(dkeys)
        is_get = op_mix(r + 1, 50, b).astype(bool)
        op_val = np.arange(r * b, (r + 1) * b, dtype=U64) + U64(1)
        dg = torch.from_numpy(is_get).cuda()
        gk, pk = dkeys[dg], dkeys[~dg]
        pv = torch.from_numpy(op_val[~is_get].view(np.int64)).cuda()
        gv = torch.empty_like(gk)
        gf = torch.empty(gk.numel(), dtype=torch.uint8, device="cuda")
        t.mixed_batch(gk, gv, gf, pk, pv)
        t.synchronize()
        ov, of = orc.search_batch(keys[is_get])
        hv, hf = host(gv), gf.cpu().numpy()
        bad = np.nonzero((hv != ov) | (hf != of))[0]
        assert bad.size == 0, f"batch {r}: {bad.size} gets differ"
        orc.apply_batch(keys[~is_get], op_val[~is_get])
    ok, ov = orc.dump()
    dk = torch.from_numpy(ok.view(np.int64)).cuda()
    v = torch.empty_like(dk)
    f = torch.empty(dk.numel(), dtype=torch.uint8, device="cuda")
    t.search_batch(dk, v, f)
    t.synchronize()
    assert bool(f.all())
    assert np.array_equal(host(v), ov)
    assert t.check()["keys"] == ok.size
    orc.close()
    t.close()
