"""The leaf directory kept current by the insert chunks' leaf writers
(sherman_amd/csrc/dir_upkeep.h; VERDICT r5 #3 / ADVICE r5).

The directory plays the reference's IndexCache (include/IndexCache.h:59-259):
an index a search starts from, kept current by the writers.  Results never
depend on it (a get that does not find its key through its entry walks the
summary path), so every test checks exact results against the oracle's
Tree::search / Tree::insert AND that the upkeep did its job: no rebuild
after splitting chunks, and the gets still answered from their entries.

All GPU work runs in this one process.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import sherman_amd as shm  # noqa: E402
from oracle.pyoracle import OracleTree  # noqa: E402

U64 = np.uint64


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()


def host(t):
    return t.cpu().numpy().view(U64)


def gen_keys(t, first, n):
    """key(i) = CityHash64(i) + 1 for i = first .. first + n - 1 (the
    device generator; test_device_cityhash_matches_oracle pins it)."""
    k = torch.empty(n, dtype=torch.int64, device="cuda")
    t.gen_keys(first, n, k)
    torch.cuda.synchronize()
    return host(k).copy()


def gpu_search(t, keys, stats=False):
    k = dev(keys)
    v = torch.empty_like(k)
    f = torch.empty(k.numel(), dtype=torch.uint8, device="cuda")
    if stats:
        t.profile(False, index_stats=True)
    t.search_batch(k, v, f)
    t.synchronize()
    st = None
    if stats:
        st = t.index_stats()
        t.profile(False)
    return host(v), f.cpu().numpy(), st


def assert_same(probe, ov, of, gv, gf):
    bad = np.nonzero((of != gf) | (ov != gv))[0]
    if bad.size:
        lines = [f"key={int(probe[i]):#x} oracle=({of[i]},{int(ov[i])}) gpu=({gf[i]},{int(gv[i])})"
                 for i in bad[:8]]
        raise AssertionError(f"{bad.size} mismatches:\n" + "\n".join(lines))


@pytest.fixture(scope="module")
def lib_ok():
    assert torch.cuda.is_available(), "GPU test without a GPU"
    shm.lib()
    return True


def loaded(n0, maint="always", arena=512 << 20, max_batch=1 << 18):
    t = shm.Tree(arena_bytes=arena, max_batch=max_batch)
    t.dir_config(maint=maint)
    orc = OracleTree(arena)
    base = gen_keys(t, 1, n0)
    bv = np.arange(1, n0 + 1, dtype=U64) * U64(2)
    for c in range(0, n0, max_batch):
        t.insert_batch(dev(base[c:c + max_batch]), dev(bv[c:c + max_batch]))
    orc.apply_batch(base, bv)
    return t, orc, base


def assert_dir_exact(t):
    """Every directory entry the walks trust names exactly what the tree
    holds (shm__dir_verify): leaf lists and split points, every key's pair,
    every valid slot's fingerprint."""
    v = t.dir_verify()
    assert v["bad_lists"] == 0 and v["bad_pairs"] == 0 and v["bad_fps"] == 0, v
    return v


def next_pow2(x):
    return 1 << max(0, int(x - 1).bit_length())


@pytest.mark.parametrize("form", ["fingerprints", "pairs"])
def test_splitting_chunks_keep_the_directory_current(lib_ok, form):
    """Both directory forms: after the load (fingerprint form) or a read
    phase (pair form), chunks go in with the upkeep on: runs of 30 new keys
    next to stored ones (each splits its leaf), new keys spread over the
    tree (each into an empty slot of its leaf), in-place updates and
    deletes.  Every later get equals the oracle, the directory is NOT
    rebuilt (the tree stays below the next power of two of pages, which
    would call for a denser one), and the share of gets answered from their
    directory entry stays within a few percent of what it was before the
    chunks (the one or two prefixes per split page shared with a neighbour
    go to the summary walk)."""
    n0 = 1 << 18
    t, orc, base = loaded(n0)
    rng = np.random.default_rng(7)
    probe = base[rng.integers(0, n0, 1 << 15)]
    reads = 5 if form == "pairs" else 1  # four searches without an insert: the read phase
    for _ in range(reads):
        gv, gf, _ = gpu_search(t, probe)
    gv, gf, st0 = gpu_search(t, probe, stats=True)
    assert_same(probe, *orc.search_batch(probe), gv, gf)
    d0 = t.dir_stats()
    assert d0["form"] == form and d0["maintained"], d0
    assert assert_dir_exact(t)["checked"] > 0  # the build itself
    frac0 = st0["dir_fp_hits"] / st0["gets"]
    if form == "pairs":
        assert st0["dir_fp_hits"] == st0["gets"], st0  # every get from its entry
    pages0 = t.stats()["pages_used"]
    nid = n0 + 1
    for r in range(2):
        anchors = base[rng.integers(0, n0, 100)]
        runs = np.unique((anchors[:, None] + np.arange(1, 31, dtype=U64)[None, :]).ravel())
        runs = runs[~np.isin(runs, base)]
        spread = gen_keys(t, nid, 1 << 14)
        nid += spread.size
        upd = base[rng.integers(0, n0, 4000)]
        dele = base[rng.integers(0, n0, 2000)]
        k = np.concatenate([runs, spread, upd, dele])
        v = np.concatenate([runs ^ U64(0x77), np.arange(1, spread.size + 1, dtype=U64) * U64(3),
                            upd ^ U64(0x5A5A + r), np.zeros(dele.size, dtype=U64)])
        t.insert_batch(dev(k), dev(v))
        orc.apply_batch(k, v)
        assert_dir_exact(t)
    pages1 = t.stats()["pages_used"]
    assert pages1 > pages0 + 150, (pages0, pages1)  # leaves split
    assert next_pow2(pages1 + 1) == next_pow2(pages0 + 1), (pages0, pages1)  # same density
    stored, _ = orc.dump()
    probe2 = np.concatenate([stored[rng.integers(0, stored.size, 1 << 15)],
                             gen_keys(t, nid, 4096)])  # + never stored
    gv, gf, st1 = gpu_search(t, probe2, stats=True)
    assert_same(probe2, *orc.search_batch(probe2), gv, gf)
    d1 = t.dir_stats()
    assert d1["builds"] == d0["builds"], (d0, d1)  # no rebuild: the chunks kept it
    assert d1["form"] == form
    frac1 = st1["dir_fp_hits"] / max(st1["hits"], 1)
    if form == "pairs":
        # as good as a fresh build: the runs of 30 keys leave ~200 prefixes
        # with more than 16 keys, which no pair entry can list (k_dir_pairs
        # leaves them unusable as well); rebuild (round 5's rules, upkeep
        # off) and compare on the same probe
        t.dir_config(maint=False)
        for _ in range(4):
            gpu_search(t, probe2)
        gv, gf, st2 = gpu_search(t, probe2, stats=True)
        assert t.dir_stats()["builds"] > d1["builds"]
        frac2 = st2["dir_fp_hits"] / max(st2["hits"], 1)
        assert frac1 >= frac2 - 0.002, (frac1, frac2, st1, st2)
    else:
        assert frac1 >= frac0 - 0.02, (frac0, frac1, st1)  # the repairs after each chunk
    rc, oc = orc.check()
    assert rc == 0 and t.check()["keys"] == oc["keys"]
    orc.close()
    t.close()


def test_without_upkeep_the_same_chunks_stay_exact(lib_ok):
    """SHM_DIR_MAINT=0's rules (the round-5 directory: stale entries between
    rebuilds) on the same chunks: results stay exact; the stale pairs only
    cost the summary walk, which the index statistics show."""
    n0 = 1 << 18
    t, orc, base = loaded(n0, maint=False)
    rng = np.random.default_rng(8)
    probe = base[rng.integers(0, n0, 1 << 15)]
    for _ in range(5):
        gpu_search(t, probe)
    assert t.dir_stats()["form"] == "pairs" and not t.dir_stats()["maintained"]
    new = gen_keys(t, n0 + 1, 1 << 16)
    nv = np.arange(n0 + 1, n0 + 1 + new.size, dtype=U64) * U64(2)
    t.insert_batch(dev(new), dev(nv))
    orc.apply_batch(new, nv)
    probe2 = np.concatenate([probe, new[:8192]])
    gv, gf, st = gpu_search(t, probe2, stats=True)  # the first search after: stale pairs
    assert_same(probe2, *orc.search_batch(probe2), gv, gf)
    assert st["dir_fp_hits"] < st["hits"], st  # new keys and moved slots missed the pairs
    orc.close()
    t.close()


def test_directory_allocation_failure_keeps_the_tree_working(lib_ok):
    """a read phase wants a larger directory; when that
    allocation fails the tree keeps the one it has (same bits) instead of
    freeing it first, and does not retry the failed size on every call.
    With a cap below even the smallest directory, the gets walk from the
    root.  Results equal the oracle throughout."""
    n0 = 1 << 17
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 17)
    orc = OracleTree(256 << 20)
    base = gen_keys(t, 1, n0)
    bv = np.arange(1, n0 + 1, dtype=U64) * U64(2)
    t.insert_batch(dev(base), dev(bv))
    orc.apply_batch(base, bv)
    rng = np.random.default_rng(9)
    probe = np.concatenate([base[rng.integers(0, n0, 1 << 14)], gen_keys(t, n0 + 1, 1024)])
    want = orc.search_batch(probe)
    gv, gf, _ = gpu_search(t, probe)  # the write phase's fingerprint directory, sized
    assert_same(probe, *want, gv, gf)
    d = t.dir_stats()
    assert d["form"] == "fingerprints", d
    # a cap that admits this directory (2^(ceil(log2 pages) + 3) entries of
    # 72 B with the hints) but not the read phase's twice as large one
    t.dir_config(mem_limit=d["bytes"])
    builds = []
    for _ in range(10):  # into the read phase and on
        gv, gf, _ = gpu_search(t, probe)
        assert_same(probe, *want, gv, gf)
        builds.append(t.dir_stats()["builds"])
    d1 = t.dir_stats()
    assert d1["bytes"] == d["bytes"] and d1["entries"] == d["entries"], (d, d1)
    assert d1["form"] == "pairs"  # rebuilt once in the read phase's form, same size
    assert builds[-1] - d["builds"] <= 1 and builds[-1] == builds[4], builds
    t.close()
    # no room for any directory: walks from the root
    t2 = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 17)
    t2.dir_config(mem_limit=4096)
    t2.insert_batch(dev(base), dev(bv))
    for _ in range(5):
        gv, gf, _ = gpu_search(t2, probe)
        assert_same(probe, *want, gv, gf)
    assert t2.dir_stats()["form"] == "none"
    t2.close()
    orc.close()


def test_insert_every_cycles_build_once(lib_ok):
    """bench.py --insert-every's cycle at 2^20 keys: a chunk of 2^16 new keys
    after every 8 get batches.  With the upkeep the directory is built for
    the read phase once and then kept by the chunks -- no rebuild per cycle
    (round 5's rules rebuilt it in every cycle, 2.9 ms of k_dir_pairs at
    C2), at most one when the tree passes a power of two of pages (a read
    phase then wants the denser directory) -- and every get and every new
    key equal the oracle."""
    n0 = 1 << 20
    t, orc, base = loaded(n0, maint=True, arena=1 << 30, max_batch=1 << 20)
    rng = np.random.default_rng(10)
    qs = [base[rng.integers(0, n0, 1 << 16)] for _ in range(4)]
    for _ in range(5):
        gpu_search(t, qs[0])
    b0 = t.dir_stats()["builds"]
    pages0 = t.stats()["pages_used"]
    nid = n0 + 1
    for c in range(4):
        new = gen_keys(t, nid, 1 << 16)
        nv = np.arange(nid, nid + new.size, dtype=U64) * U64(2)
        nid += new.size
        t.insert_batch(dev(new), dev(nv))
        orc.apply_batch(new, nv)
        assert_dir_exact(t)
        for j in range(8):
            q = np.concatenate([qs[j % 4], new[j::8]])
            gv, gf, _ = gpu_search(t, q)
            if j in (0, 7):
                assert_same(q, *orc.search_batch(q), gv, gf)
    d = t.dir_stats()
    crossed = next_pow2(t.stats()["pages_used"] + 1) != next_pow2(pages0 + 1)
    assert d["builds"] - b0 <= (1 if crossed else 0), (d, crossed)
    assert d["form"] == "pairs" and d["last_build_ms"] > 0, d
    orc.close()
    t.close()


def test_upkeep_policy_idle_and_write_only_streams(lib_ok):
    """The default policy (tree.cpp insert_apply): a chunk keeps the
    directory only when gets read it since the last chunk and recent upkeeps
    found work.  Update-only chunks between searches (C3's mix) stop the
    upkeep after kIdleUpkeeps idle ones; a chunk with no search before it
    (C5's stream) stops it at once.  Either way the directory is then no
    longer exact, the exact shortcuts stay off, and every get still equals
    the oracle; a chunk that adds keys while searched keeps it exact."""
    n0 = 1 << 17
    t, orc, base = loaded(n0, maint=True, arena=256 << 20, max_batch=1 << 17)
    rng = np.random.default_rng(13)
    probe = np.concatenate([base[rng.integers(0, n0, 1 << 14)], gen_keys(t, 10**9, 1000)])
    for _ in range(5):
        gpu_search(t, probe)
    assert t.dir_stats()["exact"] == 1
    # a searched chunk of new keys: kept exact
    nid = n0 + 1
    new = gen_keys(t, nid, 5000)
    nid += new.size
    t.insert_batch(dev(new), dev(new ^ U64(1)))
    orc.apply_batch(new, new ^ U64(1))
    t.synchronize()
    assert t.dir_stats()["exact"] == 1
    assert_dir_exact(t)
    # update-only chunks, searched between: idle upkeeps stop the upkeep
    for r in range(5):
        gv, gf, _ = gpu_search(t, probe)
        assert_same(probe, *orc.search_batch(probe), gv, gf)
        upd = base[rng.integers(0, n0, 4000)]
        t.insert_batch(dev(upd), dev(upd ^ U64(100 + r)))
        orc.apply_batch(upd, upd ^ U64(100 + r))
        t.synchronize()
    assert t.dir_stats()["exact"] == 0
    gv, gf, _ = gpu_search(t, probe)
    assert_same(probe, *orc.search_batch(probe), gv, gf)
    # a fresh build makes it exact again; a chunk with no search before it
    # (the second one) stops the upkeep at once
    t.dir_config(maint=True)
    more = gen_keys(t, nid, 40000)
    nid += more.size
    t.insert_batch(dev(more), dev(more ^ U64(2)))
    orc.apply_batch(more, more ^ U64(2))
    for _ in range(5):
        gpu_search(t, probe)
    assert t.dir_stats()["exact"] == 1
    for c in range(2):
        new = gen_keys(t, nid, 3000)
        nid += new.size
        t.insert_batch(dev(new), dev(new ^ U64(3)))
        orc.apply_batch(new, new ^ U64(3))
        t.synchronize()
    assert t.dir_stats()["exact"] == 0
    ok_, ov = orc.dump()
    gv, gf, _ = gpu_search(t, ok_)
    assert bool(gf.all()) and np.array_equal(gv, ov)
    miss = gen_keys(t, 10**9 + 7, 2000)
    gv, gf, _ = gpu_search(t, miss)
    assert_same(miss, *orc.search_batch(miss), gv, gf)
    orc.close()
    t.close()


@pytest.mark.parametrize("reads", [1, 5])
def test_exact_directory_places_new_keys_through_many_chunks(lib_ok, reads):
    """With the upkeep on the directory is exact, so k_locate places a key an
    entry does not name straight in the entry's leaf and k_get_sum answers a
    miss from the entry (no summary walk).  Twelve rounds of chunks that
    split clustered runs and spread new keys, delete, update and re-insert
    deleted keys -- searched between them once (fingerprint form) or five
    times (the read phase's pair form) -- must leave every get, the contents
    and the B-link invariants equal to the oracle's (a key placed in a leaf
    whose fences do not hold it would fail the upsert's fence check)."""
    n0 = 1 << 16
    t, orc, base = loaded(n0, arena=256 << 20, max_batch=1 << 16)
    rng = np.random.default_rng(11 + reads)
    nid = n0 + 1
    deleted = np.zeros(0, dtype=U64)
    for r in range(12):
        stored, _ = orc.dump()
        anchors = stored[rng.integers(0, stored.size, 60)]
        runs = np.unique((anchors[:, None] + np.arange(1, 41, dtype=U64)[None, :]).ravel())
        spread = gen_keys(t, nid, 2000)
        nid += spread.size
        dele = stored[rng.integers(0, stored.size, 500)]
        back = deleted[:300]  # re-inserted
        upd = stored[rng.integers(0, stored.size, 500)]
        k = np.concatenate([runs, spread, dele, back, upd])
        v = np.concatenate([runs ^ U64(r + 1), spread ^ U64(7), np.zeros(dele.size, dtype=U64),
                            back ^ U64(3), upd ^ U64(0xABC + r)])
        t.insert_batch(dev(k), dev(v))
        orc.apply_batch(k, v)
        assert_dir_exact(t)
        deleted = np.unique(np.concatenate([deleted[300:], dele]))
        probe = np.concatenate([k, stored[rng.integers(0, stored.size, 4000)],
                                gen_keys(t, nid + 10**7, 500)])
        for _ in range(reads):
            gv, gf, _ = gpu_search(t, probe)
        assert_same(probe, *orc.search_batch(probe), gv, gf)
    d = t.dir_stats()
    assert d["maintained"] and d["form"] == ("pairs" if reads == 5 else "fingerprints"), d
    rc, oc = orc.check()
    assert rc == 0 and t.check()["keys"] == oc["keys"]
    ok_, ov = orc.dump()
    gv, gf, _ = gpu_search(t, ok_)
    assert bool(gf.all()) and np.array_equal(gv, ov)
    orc.close()
    t.close()


def test_page_check_flag_on_the_fast_path(lib_ok):
    """SHM_FLAG_PAGE_CHECK: every page a get takes a value from also has its
    front / rear versions compared (Tree.h:241-261); with gets and writers
    ordered by the call rule no page is ever torn under a get, so the
    checked walk reports nothing and equals the oracle, in both directory
    forms and through the summary path (misses, a stale phase)."""
    n0 = 1 << 17
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 17, page_check=True)
    orc = OracleTree(256 << 20)
    base = gen_keys(t, 1, n0)
    bv = np.arange(1, n0 + 1, dtype=U64) * U64(2)
    t.insert_batch(dev(base), dev(bv))
    orc.apply_batch(base, bv)
    rng = np.random.default_rng(12)
    for r in range(3):
        probe = np.concatenate([base[rng.integers(0, n0, 1 << 14)], gen_keys(t, 10**9 + r, 2000)])
        for _ in range(5 if r == 1 else 1):
            gv, gf, _ = gpu_search(t, probe)
            assert_same(probe, *orc.search_batch(probe), gv, gf)
        new = gen_keys(t, n0 + 1 + r * 20000, 20000)
        nv = new ^ U64(5)
        t.insert_batch(dev(new), dev(nv))
        orc.apply_batch(new, nv)
    t.synchronize()
    assert t.last_error()["bits"] == 0
    orc.close()
    t.close()


@pytest.mark.parametrize("seed", [2024, 7])
def test_random_phases_against_the_oracle(lib_ok, seed):
    """A randomised stream under the default policy: chunks of new keys,
    updates, deletes and re-inserts, clustered runs that split, with 0 to 6
    get batches between them (so the chunks are kept, idle or unkept and the
    directory turns exact and back, changes form and density), the odd range
    batch and update-only chunk.  Every get, every scan and the final
    contents equal the oracle's, and whenever the library reports the
    directory exact, every entry it trusts is (shm__dir_verify)."""
    n0 = 1 << 16
    t, orc, base = loaded(n0, maint=True, arena=256 << 20, max_batch=1 << 16)
    rng = np.random.default_rng(seed)
    nid = n0 + 1
    deleted = np.zeros(0, dtype=U64)
    exact_seen = 0
    for r in range(50):
        stored, _ = orc.dump()
        kind = rng.integers(0, 4)
        if kind == 0:  # updates only
            k = stored[rng.integers(0, stored.size, 3000)]
            v = k ^ U64(r + 11)
        else:
            anchors = stored[rng.integers(0, stored.size, int(rng.integers(5, 60)))]
            runs = np.unique((anchors[:, None] +
                              np.arange(1, int(rng.integers(2, 50)), dtype=U64)[None, :]).ravel())
            spread = gen_keys(t, nid, int(rng.integers(0, 4000)))
            nid += spread.size
            dele = stored[rng.integers(0, stored.size, int(rng.integers(0, 800)))]
            back = deleted[:int(rng.integers(0, 300))]
            k = np.concatenate([runs, spread, dele, back])
            v = np.concatenate([runs ^ U64(r + 1), spread ^ U64(5), np.zeros(dele.size, dtype=U64),
                                back ^ U64(9)])
            deleted = np.unique(np.concatenate([deleted[back.size:], dele]))
        if k.size:
            t.insert_batch(dev(k), dev(v))
            orc.apply_batch(k, v)
        if t.dir_stats()["exact"]:
            assert_dir_exact(t)
            exact_seen += 1
        stored, _ = orc.dump()
        probe = np.concatenate([k[:2000], stored[rng.integers(0, stored.size, 3000)],
                                gen_keys(t, 10**9 + 1000 * r, 300)])
        for _ in range(int(rng.integers(0, 7))):
            gv, gf, _ = gpu_search(t, probe)
            assert_same(probe, *orc.search_batch(probe), gv, gf)
        if r % 7 == 3:
            lo = stored[rng.integers(0, stored.size, 64)]
            hi = lo + U64(1 << 50)
            hi[hi < lo] = U64((1 << 64) - 2)
            c, sv = t.range_query_batch(dev(lo), dev(hi))
            oc, ov = orc.range_query_batch(lo, hi)
            assert np.array_equal(c.cpu().numpy().view(U64), oc)
            assert np.array_equal(np.sort(sv.cpu().numpy().view(U64)), np.sort(ov))
    assert exact_seen > 0  # the stream did pass through exact phases
    rc, oc = orc.check()
    assert rc == 0 and t.check()["keys"] == oc["keys"]
    ok_, ov = orc.dump()
    gv, gf, _ = gpu_search(t, ok_)
    assert bool(gf.all()) and np.array_equal(gv, ov)
    orc.close()
    t.close()
