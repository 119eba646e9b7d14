"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bit-exact bar: every batched get returns the oracle's (found, value); after
every insert batch the GPU tree's key->value contents equal the oracle's
(last writer in batch order, value 0 = delete); both trees satisfy the
B-link invariants; and each side's page image is searchable by the other
(byte-layout conformance with include/Tree.h:130-336).

All GPU work runs in this one process.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import sherman_amd as shm  # noqa: E402
from oracle.pyoracle import OracleTree, op_mix, to_key, zipf_fill  # noqa: E402

U64 = np.uint64


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=U64).view(np.int64)).cuda()


def host(t):
    return t.cpu().numpy().view(U64)


def gpu_search(tree, keys):
    k = dev(keys)
    v = torch.empty_like(k)
    f = torch.empty(k.numel(), dtype=torch.uint8, device=k.device)
    tree.search_batch(k, v, f)
    tree.synchronize()
    return host(v), f.cpu().numpy()


def gpu_insert(tree, keys, vals):
    tree.insert_batch(dev(keys), dev(vals))


def hashed_keys(lo, hi):
    i = np.arange(lo, hi, dtype=U64)
    # CityHash64 restatement on device vs oracle is checked separately; here
    # use the oracle's generator so both sides see identical streams
    return np.array([to_key(int(x)) for x in i], dtype=U64)


@pytest.fixture(scope="module")
def lib_ok():
    assert torch.cuda.is_available(), "GPU test without a GPU"
    shm.lib()
    return True


def assert_same(probe, ov, of, gv, gf):
    bad = np.nonzero((of != gf) | (ov != gv))[0]
    if bad.size:
        lines = [f"key={int(probe[i]):#x} oracle=({of[i]},{int(ov[i])}) gpu=({gf[i]},{int(gv[i])})"
                 for i in bad[:8]]
        raise AssertionError(f"{bad.size} mismatches:\n" + "\n".join(lines))


def compare_contents(tree, orc):
    ok, ov = orc.dump()
    order = np.argsort(ok)
    ok, ov = ok[order], ov[order]
    v, f = gpu_search(tree, ok)
    assert f.all(), f"{int((f == 0).sum())} oracle keys missing on GPU"
    assert np.array_equal(v, ov)
    st = tree.check()
    assert st["keys"] == ok.size, (st, ok.size)
    return st


def test_tree_test_kat(lib_ok):
    """test/tree_test.cpp:31-68 through the single-op API (batch of 1)."""
    t = shm.Tree(arena_bytes=64 << 20, max_batch=1 << 14)
    N = 10240
    for i in range(1, N):
        t.insert(i, i * 2)
    for i in range(N - 1, 0, -1):
        t.insert(i, i * 3)
    ks = np.arange(1, N, dtype=U64)
    v, f = gpu_search(t, ks)
    assert f.all() and np.array_equal(v, ks * U64(3))
    for i in range(1, N):
        t.del_(i)
    v, f = gpu_search(t, ks)
    assert not f.any()
    for i in range(N - 1, 0, -1):
        t.insert(i, i * 3)
    v, f = gpu_search(t, ks)
    assert f.all() and np.array_equal(v, ks * U64(3))
    for k in (1, 77, N - 1):
        assert t.search(k) == (True, k * 3)
    assert t.search(N + 5) == (False, 0)
    t.check()
    t.close()


def test_tree_test_kat_batched(lib_ok):
    """Same KAT with each phase as one batch (descending overwrite order)."""
    t = shm.Tree(arena_bytes=64 << 20, max_batch=1 << 16)
    N = 10240
    ks = np.arange(1, N, dtype=U64)
    gpu_insert(t, ks, ks * U64(2))
    rk = ks[::-1].copy()
    gpu_insert(t, rk, rk * U64(3))
    v, f = gpu_search(t, ks)
    assert f.all() and np.array_equal(v, ks * U64(3))
    t.del_batch(dev(ks))
    v, f = gpu_search(t, ks)
    assert not f.any()
    gpu_insert(t, rk, rk * U64(3))
    v, f = gpu_search(t, ks)
    assert f.all() and np.array_equal(v, ks * U64(3))
    t.close()


@pytest.mark.parametrize("batch", [1, 37, 1000, 65536])
def test_random_batches_vs_oracle(lib_ok, batch):
    """Random upserts/deletes with in-batch duplicates, batch by batch."""
    rng = np.random.default_rng(1234 + batch)
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 17)
    orc = OracleTree(256 << 20)
    universe = hashed_keys(1, 20001)
    total = 60000 if batch >= 1000 else 3000
    done = 0
    while done < total:
        b = min(batch, total - done)
        ks = universe[rng.integers(0, universe.size, b)]
        vs = rng.integers(1, 1 << 62, b).astype(U64)
        vs[rng.random(b) < 0.1] = 0  # deletes
        gpu_insert(t, ks, vs)
        orc.apply_batch(ks, vs)
        done += b
        if batch >= 1000 or done >= total:
            compare_contents(t, orc)
    # absent keys
    probe = np.concatenate([universe, hashed_keys(30001, 31001)])
    ov, of = orc.search_batch(probe)
    gv, gf = gpu_search(t, probe)
    assert_same(probe, ov, of, gv, gf)
    assert orc.check()[0] == 0
    t.close()


def test_insert_order_apply_pipeline_vs_oracle(lib_ok):
    """shm_insert_order / shm_insert_apply: batch i + 1 ordered on a second
    stream while batch i applies (the ordering outputs alternate between two
    buffer parities).  Upserts with in-batch duplicates, deletes and new keys
    that split leaves; gets queued between the applies see exactly the
    batches applied before them; contents and invariants equal the oracle's
    after every batch; the API's refusals (third ticket, out-of-order apply,
    other inserts while a ticket is outstanding, a chunk over max_batch) and
    a kKeyMax chunk rejected at the next synchronising call."""
    rng = np.random.default_rng(77)
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 14)
    orc = OracleTree(256 << 20)
    universe = hashed_keys(1, 40001)
    pre = universe[:10000]
    gpu_insert(t, pre, pre + U64(1))
    orc.apply_batch(pre, pre + U64(1))
    s_ord, s_main = torch.cuda.Stream(), torch.cuda.Stream()
    s_ord.wait_stream(torch.cuda.current_stream())
    s_main.wait_stream(torch.cuda.current_stream())
    batches = []
    for _ in range(8):
        b = int(rng.integers(3000, 1 << 14))
        ks = universe[rng.integers(0, universe.size, b)]  # updates, new keys, duplicates
        vs = rng.integers(1, 1 << 62, b).astype(U64)
        vs[rng.random(b) < 0.08] = 0  # deletes
        batches.append((dev(ks), dev(vs), ks, vs))
    probe = np.concatenate([universe, hashed_keys(50001, 51001)])
    dprobe = dev(probe)
    outs = []
    tickets = [t.insert_order(batches[0][0], batches[0][1], stream=s_ord)]
    for i in range(len(batches)):
        if i + 1 < len(batches):
            tickets.append(t.insert_order(batches[i + 1][0], batches[i + 1][1], stream=s_ord))
            if i == 0:
                # two tickets outstanding: a third is refused, and so is the
                # newer one applied first, and any other insert
                with pytest.raises(shm.ShermanError):
                    t.insert_order(batches[0][0], batches[0][1], stream=s_ord)
                with pytest.raises(shm.ShermanError):
                    t.insert_apply(tickets[1], stream=s_main)
                with pytest.raises(shm.ShermanError):
                    t.insert_batch_async(batches[0][0], batches[0][1])
        t.insert_apply(tickets[i], stream=s_main)
        v = torch.empty_like(dprobe)
        f = torch.empty(dprobe.numel(), dtype=torch.uint8, device="cuda")
        t.search_batch(dprobe, v, f, stream=s_main)  # sees batches 0..i
        outs.append((v, f))
    t.synchronize()
    for i, (_, _, ks, vs) in enumerate(batches):
        orc.apply_batch(ks, vs)
        ov, of = orc.search_batch(probe)
        assert_same(probe, ov, of, host(outs[i][0]), outs[i][1].cpu().numpy())
    compare_contents(t, orc)
    assert orc.check()[0] == 0
    # a chunk over max_batch is refused; a kKeyMax chunk is rejected whole
    big = torch.ones((1 << 14) + 1, dtype=torch.int64, device="cuda")
    with pytest.raises(shm.ShermanError):
        t.insert_order(big, big)
    bad = batches[0][2].copy()
    bad[7] = U64((1 << 64) - 1)
    dbad = dev(bad)
    tk = t.insert_order(dbad, batches[0][1])
    t.insert_apply(tk)
    with pytest.raises(shm.ShermanError) as ei:
        t.synchronize()
    assert ei.value.rc == shm.SHM_EINVAL
    compare_contents(t, orc)  # nothing of the rejected chunk applied
    t.close()


def test_bulk_sorted_and_reverse(lib_ok):
    """One huge batch into an empty tree (k-way splits up to a new root)."""
    t = shm.Tree(arena_bytes=512 << 20, max_batch=1 << 20)
    ks = np.arange(1, 400001, dtype=U64) * U64(7919)
    gpu_insert(t, ks, ks + U64(1))
    st = t.check()
    assert st["keys"] == ks.size
    v, f = gpu_search(t, ks)
    assert f.all() and np.array_equal(v, ks + U64(1))
    # overwrite in reverse batch order with different values
    rk = ks[::-1].copy()
    gpu_insert(t, rk, rk + U64(2))
    v, f = gpu_search(t, ks)
    assert f.all() and np.array_equal(v, ks + U64(2))
    assert t.stats()["height"] >= 3
    t.close()


def test_image_conformance_oracle_to_gpu(lib_ok):
    """Oracle-built pages (reference split rules) are walked by the GPU."""
    orc = OracleTree(256 << 20)
    ks = hashed_keys(1, 150001)
    orc.apply_batch(ks, ks ^ U64(0x5555))
    img = orc.image()
    t = shm.Tree(arena_bytes=512 << 20, max_batch=1 << 18)
    t.load_image(img, orc.root_ptr)
    probe = np.concatenate([ks, hashed_keys(200001, 210001)])
    ov, of = orc.search_batch(probe)
    gv, gf = gpu_search(t, probe)
    assert_same(probe, ov, of, gv, gf)
    # and the GPU can keep inserting into the reference-built tree
    more = hashed_keys(150001, 170001)
    gpu_insert(t, more, more)
    orc.apply_batch(more, more)
    compare_contents(t, orc)
    t.close()


def test_image_conformance_gpu_to_oracle(lib_ok):
    """GPU-built pages are walked by the oracle (reference search code)."""
    t = shm.Tree(arena_bytes=512 << 20, max_batch=1 << 18)
    ks = hashed_keys(1, 120001)
    for c in range(0, ks.size, 40000):
        gpu_insert(t, ks[c:c + 40000], ks[c:c + 40000] + U64(5))
    img, root = t.dump_image()
    orc = OracleTree(image=img, root_ptr=root)
    rc, shape = orc.check()
    assert rc == 0, rc
    assert shape["keys"] == ks.size
    probe = np.concatenate([ks, hashed_keys(900001, 905001)])
    ov, of = orc.search_batch(probe)
    gv, gf = gpu_search(t, probe)
    assert_same(probe, ov, of, gv, gf)
    # and both equal what was written, independently of the image
    want = np.concatenate([ks + U64(5), np.zeros(5000, dtype=U64)])
    assert np.array_equal(ov, want) and np.array_equal(of, (want != 0).astype(np.uint8))
    t.close()


def test_overwrites_write_the_reference_entry_bytes(lib_ok):
    """Overwrite-only leaves are written entry by entry at the slot k_locate
    found, without staging the page (upsert.hip); leaves that also get a new
    key are staged.  Either way every byte of the page image equals the
    oracle's after the same batch: the value, f_version + 1 and r_version =
    f_version per overwritten entry (Tree.cpp:878-912), nothing else moved."""
    rng = np.random.default_rng(4242)
    orc = OracleTree(256 << 20)
    ks = hashed_keys(1, 150001)
    orc.apply_batch(ks, ks ^ U64(0x77))
    t = shm.Tree(arena_bytes=512 << 20, max_batch=1 << 18)
    t.load_image(orc.image(), orc.root_ptr)

    def same_image():
        img, root = t.dump_image()
        ref = orc.image()
        assert root == orc.root_ptr
        assert img.size == ref.size, (img.size, ref.size)
        diff = np.nonzero(img[1024:] != ref[1024:])[0]
        assert diff.size == 0, f"{diff.size} bytes differ, first at {1024 + int(diff[0])}"

    for r in range(3):  # overwrite-only: every leaf written in place
        up = rng.choice(ks, 60000, replace=False)
        vs = rng.integers(1, 1 << 62, up.size).astype(U64)
        gpu_insert(t, up, vs)
        orc.apply_batch(up, vs)
        same_image()
    # overwrites plus a few new keys (those leaves staged, no split)
    up = rng.choice(ks, 40000, replace=False)
    new = hashed_keys(500001, 500301)
    both = np.concatenate([up, new])
    vs = rng.integers(1, 1 << 62, both.size).astype(U64)
    gpu_insert(t, both, vs)
    orc.apply_batch(both, vs)
    if t.stats()["splits"] == 0:
        same_image()
    compare_contents(t, orc)
    t.close()


def test_range_query_async_long_scans_match_sync(lib_ok):
    """The async scans' one-pass placement (launch_range_place): thousands of
    scans over many placement blocks, with scans longer than their staging
    (> 160 values: walked again from the overflow list) mixed with short and
    empty ones; counts, offsets and values equal the synchronous call's."""
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 14)
    ks = hashed_keys(1, 60001)
    gpu_insert(t, ks, ks + U64(5))
    rng = np.random.default_rng(23)
    n = 3000
    lo = rng.integers(0, 1 << 63, n, dtype=np.uint64) * U64(2)
    # ~0-60 keys per scan, every 97th scan ~ 200-600 keys, a few whole-space
    span = (U64(1) << U64(52)) * rng.integers(0, 16, n).astype(U64)
    span[::97] = (U64(1) << U64(57)) * rng.integers(1, 4, span[::97].size).astype(U64)
    hi = lo + span
    hi[hi < lo] = U64((1 << 64) - 1)
    lo[5], hi[5] = U64(0), U64((1 << 64) - 1)
    lo[6], hi[6] = U64(9), U64(8)  # empty
    sc, sv = t.range_query_batch(dev(lo), dev(hi))
    scn = sc.cpu().numpy()
    assert (scn > 160).sum() >= 20 and scn[5] == ks.size
    pend = t.range_query_batch_async(dev(lo), dev(hi))
    assert pend.tot is not None
    ac, av = pend.result()
    assert np.array_equal(ac.cpu().numpy(), scn)
    assert np.array_equal(host(av), host(sv))
    t.check()
    t.close()


@pytest.mark.parametrize("max_batch,cap,leaf_dir", [(1 << 17, None, True),
                                                    (128, 16, True),
                                                    (1 << 17, None, False)])
def test_range_query_vs_oracle(lib_ok, max_batch, cap, leaf_dir):
    """Batched scans vs the oracle; (128, 16): scans in chunks of max_batch
    and a values buffer too small at first (SHM_ENOSPC, then the fill)."""
    t = shm.Tree(arena_bytes=256 << 20, max_batch=max_batch, leaf_dir=leaf_dir)
    if cap is not None:
        t._rq_cap = cap
    orc = OracleTree(256 << 20)
    ks = hashed_keys(1, 50001)
    gpu_insert(t, ks, ks + U64(9))
    orc.apply_batch(ks, ks + U64(9))
    rng = np.random.default_rng(7)
    lo = rng.integers(0, 1 << 63, 300, dtype=np.uint64) * U64(2)
    span = (U64(1) << U64(50)) * rng.integers(0, 64, 300).astype(U64)
    hi = lo + span
    hi[hi < lo] = U64((1 << 64) - 1)
    lo[0], hi[0] = U64(0), U64((1 << 64) - 1)  # whole key space
    lo[1], hi[1] = U64(5), U64(4)              # empty (from > to)
    counts, vals = t.range_query_batch(dev(lo), dev(hi))
    counts = counts.cpu().numpy()
    vals = host(vals)
    # exact order (leaf order, then slot order) is a property of the page
    # image: check it with the reference scan over the GPU's own pages
    img, root = t.dump_image()
    same_pages = OracleTree(image=img, root_ptr=root)
    off = 0
    for i in range(lo.size):
        ref, n = orc.range_query(int(lo[i]), int(hi[i]), cap=60000)
        assert counts[i] == n
        assert np.array_equal(np.sort(vals[off:off + n]), np.sort(ref))
        ref_img, n_img = same_pages.range_query(int(lo[i]), int(hi[i]), cap=60000)
        assert n_img == n and np.array_equal(vals[off:off + n], ref_img)
        off += n
    t.close()


def test_range_scan_plan_edges(lib_ok):
    """Range scans whose start meets each leaf-directory entry form: spread
    keys (one-leaf fingerprint entries and entries of two to four leaves)
    next to a dense run of consecutive keys (prefixes of more than four
    leaves: the entry names an internal page, so the scan descends from it
    before it walks the sibling chain); scans that end at
    the key space's top (past the directory's last prefix), scans inside one
    leaf, scans of exactly one key, and scans from below the smallest key.
    Counts and values against the oracle, exact leaf / slot order against
    the reference scan over the GPU's own pages."""
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 17)
    orc = OracleTree(256 << 20)
    spread = hashed_keys(1, 60001)
    c0 = U64(0x7123456789A00000)
    dense = c0 + np.arange(20000, dtype=U64) * U64(3)
    ks = np.unique(np.concatenate([spread, dense]))
    vs = ks ^ U64(0x5A5A)
    vs[vs == 0] = U64(1)
    gpu_insert(t, ks, vs)
    orc.apply_batch(ks, vs)
    rng = np.random.default_rng(23)
    probe = ks[rng.integers(0, ks.size, 4096)]
    assert_same(probe, *orc.search_batch(probe), *gpu_search(t, probe))  # builds the directory
    pick = ks[rng.integers(0, ks.size, 300)]
    lo = np.concatenate([
        c0 - (U64(1) << U64(50)) * rng.integers(1, 8, 40).astype(U64),  # into the dense run
        dense[rng.integers(0, dense.size, 40)],                          # inside it
        pick,                                                            # anywhere
        pick[:40],                                                       # one key
        np.array([0, 5, int(ks[-1]), int(ks[0])], dtype=U64)])
    hi = np.concatenate([
        c0 + U64(3 * 500) * rng.integers(1, 8, 40).astype(U64),
        lo[40:80] + U64(3 * 300),
        pick + (U64(1) << U64(44)) * rng.integers(0, 512, 300).astype(U64),
        pick[:40],
        np.array([(1 << 64) - 1, 4, (1 << 64) - 1, int(ks[0])], dtype=U64)])
    hi[hi < lo] = U64((1 << 64) - 1)
    hi[-3] = U64(4)  # from > to: empty
    counts, vals = t.range_query_batch(dev(lo), dev(hi))
    counts = counts.cpu().numpy()
    vals = host(vals)
    img, root = t.dump_image()
    same_pages = OracleTree(image=img, root_ptr=root)
    off = 0
    for i in range(lo.size):
        ref, n = orc.range_query(int(lo[i]), int(hi[i]), cap=120000)
        assert counts[i] == n, i
        ref_img, n_img = same_pages.range_query(int(lo[i]), int(hi[i]), cap=120000)
        assert n_img == n and np.array_equal(vals[off:off + n], ref_img), i
        assert np.array_equal(np.sort(vals[off:off + n]), np.sort(ref)), i
        off += n
    same_pages.close()
    orc.close()
    t.close()


def test_range_query_slots_vs_oracle(lib_ok):
    """shm_range_query_slots (a buffer per scan, Tree::range_query(from, to,
    buffer) batched): every scan's count and its values in the reference's
    leaf / slot order over the same pages, against the oracle's contents;
    scans longer than slot_cap keep their first slot_cap values, report the
    full count and are counted in the status; more scans than max_batch in
    one call; an empty batch; the buffers past each scan's values untouched."""
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 10)
    orc = OracleTree(256 << 20)
    ks = hashed_keys(1, 50001)
    gpu_insert(t, ks, ks + U64(9))
    orc.apply_batch(ks, ks + U64(9))
    rng = np.random.default_rng(29)
    n = 3000  # > max_batch: any n in one call
    lo = rng.integers(0, 1 << 63, n, dtype=np.uint64) * U64(2)
    span = (U64(1) << U64(50)) * rng.integers(0, 64, n).astype(U64)
    span[::101] = U64(1) << U64(58)  # ~780 keys: past the slot
    hi = lo + span
    hi[hi < lo] = U64((1 << 64) - 1)
    lo[1], hi[1] = U64(5), U64(4)  # empty (from > to)
    lo[2], hi[2] = U64(0), U64((1 << 64) - 1)  # whole key space
    cap = 200
    vals = torch.full((n, cap), 0x5A5A, dtype=torch.int64, device="cuda")
    status = torch.zeros(2, dtype=torch.int64, device="cuda")
    pend = t.range_query_slots(dev(lo), dev(hi), cap, vals=vals, status=status)
    ovf = pend.check()
    assert int(status[1].item()) == 0 and int(status[0].item()) == ovf
    counts = pend.counts.cpu().numpy()
    hv = vals.cpu().numpy().view(np.uint64)
    img, root = t.dump_image()
    same_pages = OracleTree(image=img, root_ptr=root)
    n_over = 0
    for i in range(n):
        ref, c = orc.range_query(int(lo[i]), int(hi[i]), cap=60000)
        assert counts[i] == c, i
        m = min(c, cap)
        ref_img, c_img = same_pages.range_query(int(lo[i]), int(hi[i]), cap=60000)
        assert c_img == c and np.array_equal(hv[i, :m], ref_img[:m]), i
        if c <= cap:
            assert np.array_equal(np.sort(hv[i, :m]), np.sort(ref)), i
        assert (hv[i, m:] == U64(0x5A5A)).all(), i  # nothing past the scan's values
        n_over += c > cap
    assert n_over >= 20 and ovf == n_over and counts[2] == ks.size and counts[1] == 0
    with pytest.raises(shm.ShermanError):
        pend.result()  # SHM_ENOSPC: some scans passed the slot
    # the compact form of a batch that fits
    sel = counts <= cap
    p2 = t.range_query_slots(dev(lo[sel]), dev(hi[sel]), cap)
    c2, v2 = p2.packed()
    sc, sv = t.range_query_batch(dev(lo[sel]), dev(hi[sel]))
    assert np.array_equal(c2.cpu().numpy(), sc.cpu().numpy())
    assert np.array_equal(host(v2), host(sv))
    # the status accumulates over calls; an empty batch adds nothing
    e = torch.empty(0, dtype=torch.int64, device="cuda")
    c0, v0 = t.range_query_slots(e, e, cap, status=status).result()
    assert c0.numel() == 0
    t.range_query_slots(dev(lo[:5]), dev(hi[:5]), cap, status=status).check()
    assert int(status[0].item()) == ovf + int((counts[:5] > cap).sum())
    t.check()
    t.close()


def test_range_query_async_matches_sync_and_reports_overflow(lib_ok):
    """shm_range_query_batch_async: the scans queued before an insert see the
    pre-insert tree and equal the synchronous call's (counts and values in the
    same order); a buffer smaller than the total drops the values past it
    (nothing is written out of bounds) and .result() raises SHM_ENOSPC."""
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 14)
    ks = hashed_keys(1, 40001)
    gpu_insert(t, ks, ks + U64(3))
    rng = np.random.default_rng(11)
    lo = rng.integers(0, 1 << 63, 500, dtype=np.uint64) * U64(2)
    hi = lo + (U64(1) << U64(52)) * rng.integers(0, 8, 500).astype(U64)
    hi[hi < lo] = U64((1 << 64) - 1)
    lo[1], hi[1] = U64(5), U64(4)  # empty (from > to)
    sc, sv = t.range_query_batch(dev(lo), dev(hi))
    alo, ahi = dev(lo), dev(hi)
    pend = t.range_query_batch_async(alo, ahi)
    assert pend.tot is not None  # the handle knows a buffer size: really async
    # an insert queued behind the scans (new keys inside their ranges)
    newk = lo[2:200] + U64(1)
    gpu_insert(t, newk, newk + U64(3))
    ac, av = pend.result()
    assert np.array_equal(ac.cpu().numpy(), sc.cpu().numpy())
    assert np.array_equal(host(av), host(sv))
    total = int(sc.sum().item())
    assert total > 64
    # overflow: a 64-value buffer inside a larger allocation, guard words intact
    t._rq_cap = 64
    n = lo.size
    guard = torch.full((total + 64,), 0x5A5A, dtype=torch.int64, device="cuda")
    counts = torch.empty(n, dtype=torch.int64, device="cuda")
    offs = torch.empty(n, dtype=torch.int64, device="cuda")
    tot = torch.empty(2, dtype=torch.int64, device="cuda")
    dlo, dhi = dev(lo), dev(hi)  # kept alive while the scans run
    rc = shm.lib().shm_range_query_batch_async(t.h, dlo.data_ptr(), dhi.data_ptr(), n,
                                               counts.data_ptr(), offs.data_ptr(),
                                               guard.data_ptr(), 64, tot.data_ptr(), None)
    assert rc == 0
    torch.cuda.synchronize()
    assert int(tot[1].item()) == 0 and int(tot[0].item()) >= total
    assert bool((guard[64:] == 0x5A5A).all().item())
    pend = shm.PendingRange(t, counts, guard[:64], tot)
    with pytest.raises(shm.ShermanError):
        pend.result()
    # more scans than one chunk is refused
    big = torch.zeros((1 << 14) + 1, dtype=torch.int64, device="cuda")
    rc = shm.lib().shm_range_query_batch_async(t.h, big.data_ptr(), big.data_ptr(), big.numel(),
                                               big.data_ptr(), big.data_ptr(), None, 0,
                                               tot.data_ptr(), None)
    assert rc == shm.SHM_EINVAL
    t.check()
    t.close()


def test_read_words_zero_copy(lib_ok):
    """shm_read_words (the router's count read-back) returns what the stream
    wrote before it, on the default and on a side stream; bad sizes are
    refused."""
    t = shm.Tree(arena_bytes=32 << 20, max_batch=4096)
    for it in range(3):
        x = torch.arange(32, dtype=torch.int64, device="cuda") * (it + 7) - (1 << 40)
        assert t.read_i64(x) == x.cpu().tolist()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        y = torch.full((5,), -3, dtype=torch.int64, device="cuda")
        y += 1
        assert t.read_i64(y) == [-2] * 5
    buf = (ctypes.c_int64 * 64)()
    assert shm.lib().shm_read_words(t.h, x.data_ptr(), 1028, buf, None) == shm.SHM_EINVAL
    assert shm.lib().shm_read_words(t.h, x.data_ptr(), 6, buf, None) == shm.SHM_EINVAL
    t.close()


def test_edge_cases(lib_ok):
    t = shm.Tree(arena_bytes=32 << 20, max_batch=4096)
    # empty batches
    e = torch.empty(0, dtype=torch.int64, device="cuda")
    t.insert_batch(e, e)
    t.search_batch(e, e)
    # kKeyMax is rejected and nothing is applied
    bad = np.array([5, (1 << 64) - 1], dtype=U64)
    with pytest.raises(shm.ShermanError) as ei:
        gpu_insert(t, bad, np.array([1, 2], dtype=U64))
    assert ei.value.rc == shm.SHM_EINVAL
    assert t.search(5) == (False, 0)
    v, f = gpu_search(t, np.array([(1 << 64) - 1], dtype=U64))
    assert not f.any()
    # key 0 (kKeyMin) is a valid key; value 0 means delete
    gpu_insert(t, np.array([0, 1], dtype=U64), np.array([10, 11], dtype=U64))
    assert t.search(0) == (True, 10)
    gpu_insert(t, np.array([0], dtype=U64), np.array([0], dtype=U64))
    assert t.search(0) == (False, 0)
    # duplicates inside one batch: last writer wins, delete-then-insert too
    gpu_insert(t, np.array([3, 3, 3, 4, 4], dtype=U64), np.array([1, 2, 3, 7, 0], dtype=U64))
    assert t.search(3) == (True, 3)
    assert t.search(4) == (False, 0)
    # batch larger than max_batch is chunked in order
    ks = np.arange(100, 100 + 10000, dtype=U64)
    gpu_insert(t, np.concatenate([ks, ks]), np.concatenate([ks, ks + U64(1)]))
    v, f = gpu_search(t, ks)
    assert f.all() and np.array_equal(v, ks + U64(1))
    # the largest storable key (kKeyMax - 1) and its neighbours, in every
    # directory form: the write phase's, then the read phase's pairs (five
    # searches), then after a chunk that touches them
    top = np.array([(1 << 64) - 2, (1 << 64) - 3, 1 << 63], dtype=U64)
    gpu_insert(t, top, np.array([21, 22, 23], dtype=U64))
    probe = np.concatenate([top, np.array([(1 << 64) - 4, (1 << 63) + 1], dtype=U64)])
    want_v = np.array([21, 22, 23, 0, 0], dtype=U64)
    for _ in range(6):
        v, f = gpu_search(t, probe)
        assert np.array_equal(v, want_v) and np.array_equal(f, (want_v != 0).astype(np.uint8))
    gpu_insert(t, top[:1], np.array([0], dtype=U64))  # delete kKeyMax - 1
    gpu_insert(t, np.array([(1 << 64) - 4], dtype=U64), np.array([24], dtype=U64))
    v, f = gpu_search(t, probe)
    assert np.array_equal(v, np.array([0, 22, 23, 24, 0], dtype=U64))
    t.check()
    t.close()


def test_device_cityhash_matches_oracle(lib_ok):
    t = shm.Tree(arena_bytes=8 << 20, max_batch=1024)
    out = torch.empty(5000, dtype=torch.int64, device="cuda")
    t.gen_keys(1, 5000, out)
    t.synchronize()
    assert np.array_equal(host(out), hashed_keys(1, 5001))
    t.gen_keys(1, 5000, out, keyspace=64 << 20)
    t.synchronize()
    ref = np.array([to_key(i, 64 << 20) for i in range(1, 5001)], dtype=U64)
    assert np.array_equal(host(out), ref)
    t.close()


def test_route_bucket_roundtrip(lib_ok):
    """Stable bucketing by owner (the permutation equals a stable argsort of
    the owners), companion permute, and the reverse permutation."""
    t = shm.Tree(arena_bytes=8 << 20, max_batch=1 << 17)
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 1 << 63, 100000, dtype=np.uint64) * U64(2) + U64(1)
    for shards in (1, 2, 3, 8):
        k = dev(keys)
        ko = torch.empty_like(k)
        perm = torch.empty(k.numel(), dtype=torch.int32, device="cuda")
        cnt = torch.empty(shards, dtype=torch.int64, device="cuda")
        t.route_bucket(k, shards, ko, perm, cnt)
        t.synchronize()
        c = cnt.cpu().numpy()
        kh = host(ko)
        owner = ((keys.astype(object) * shards) >> 64).astype(np.int64)
        assert np.array_equal(c, np.bincount(owner, minlength=shards))
        off = np.concatenate([[0], np.cumsum(c)])
        for s in range(shards):
            seg = kh[off[s]:off[s + 1]]
            assert np.array_equal(np.sort(seg), np.sort(keys[owner == s]))
        order = np.argsort(owner, kind="stable")
        assert np.array_equal(perm.cpu().numpy().astype(np.int64), order)
        assert np.array_equal(kh, keys[order])
        vals = dev(np.arange(keys.size, dtype=U64) * U64(3))
        vo = torch.empty_like(vals)
        t.route_permute(vals, perm, vo)
        t.synchronize()
        assert np.array_equal(host(vo), order.astype(U64) * U64(3))
        back = torch.empty_like(k)
        t.route_unpermute(ko, perm, back)
        t.synchronize()
        assert np.array_equal(host(back), keys)
    t.close()


# get start modes: (sort_gets, leaf_dir); the default is unordered from the
# leaf directory
START_MODES = [(False, True), (True, True), (True, False), (False, False)]


@pytest.mark.parametrize("sort_gets,leaf_dir", START_MODES[:2])
def test_uniform_get_large_vs_oracle(lib_ok, sort_gets, leaf_dir):
    """2^21 keys key(i) -> 2i (the bench's C2 stream at 1/32 scale), checked
    against the values that were written, not against the tree's own image:
    every stored key returns 2i (so no key was dropped or mis-stored), a 2^20
    uniform batch with ~11 % misses returns 2i or not-found, and its first
    200 K queries equal the oracle's Tree::search over an independently
    built tree of the same stream (device CityHash = oracle to_key is
    test_device_cityhash_matches_oracle)."""
    n = 1 << 21
    t = shm.Tree(arena_bytes=1 << 30, max_batch=1 << 20, sort_gets=sort_gets,
                 leaf_dir=leaf_dir)
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    t.gen_keys(1, n, keys)
    vals = (torch.arange(1, n + 1, device="cuda", dtype=torch.int64) * 2)
    for c in range(0, n, 1 << 20):
        t.insert_batch(keys[c:c + (1 << 20)], vals[c:c + (1 << 20)])
    st = t.check()
    assert st["keys"] == n
    # every stored key: value 2i
    for c in range(0, n, 1 << 20):
        v = torch.empty(1 << 20, dtype=torch.int64, device="cuda")
        f = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
        t.search_batch(keys[c:c + (1 << 20)], v, f)
        t.synchronize()
        assert bool(f.all()) and torch.equal(v, vals[c:c + (1 << 20)])
    # a uniform batch over 1.125 n ids: hits return 2i, ids > n miss
    rng = np.random.default_rng(11)
    idx = rng.integers(1, n + (n >> 3), 1 << 20)
    ids = torch.from_numpy(idx.astype(np.int64)).cuda()
    q = torch.empty_like(ids)
    t.hash_keys(ids, q)
    v = torch.empty_like(q)
    f = torch.empty(q.numel(), dtype=torch.uint8, device="cuda")
    t.search_batch(q, v, f)
    t.synchronize()
    want = np.where(idx <= n, idx * 2, 0).astype(U64)
    gv, gf = host(v), f.cpu().numpy()
    assert np.array_equal(gv, want), int((gv != want).sum())
    assert np.array_equal(gf, (want != 0).astype(np.uint8))
    # the reference's search over an independently built tree, on a sample
    m = 200000
    orc = OracleTree(1 << 30)
    orc.apply_batch(np.array([to_key(int(i)) for i in range(1, n + 1)], dtype=U64),
                    np.arange(1, n + 1, dtype=U64) * U64(2))
    probe = host(q)[:m]
    ov, of = orc.search_batch(probe)
    assert_same(probe, ov, of, gv[:m], gf[:m])
    orc.close()
    t.close()


@pytest.mark.parametrize("sort_gets,leaf_dir", START_MODES)
def test_sorted_get_skewed_and_ragged(lib_ok, sort_gets, leaf_dir):
    """Gets under skew: one 16-bit bucket far larger than a fine-pass chunk of
    the sorted-get partition, next to uniform keys, with a ragged batch
    length, in every start mode."""
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 18, sort_gets=sort_gets,
                 leaf_dir=leaf_dir)
    orc = OracleTree(256 << 20)
    dense = np.arange(1, 60001, dtype=U64) * U64(3)           # all in bucket 0
    spread = hashed_keys(1, 40001)
    keys = np.concatenate([dense, spread])
    vals = np.arange(1, keys.size + 1, dtype=U64) * U64(5)
    gpu_insert(t, keys, vals)
    orc.apply_batch(keys, vals)
    rng = np.random.default_rng(5)
    probe = np.concatenate([dense[rng.integers(0, dense.size, 70001)],
                            spread[rng.integers(0, spread.size, 30000)],
                            rng.integers(1, 1 << 63, 1234, dtype=np.int64).astype(U64)])
    rng.shuffle(probe)
    ov, of = orc.search_batch(probe)
    gv, gf = gpu_search(t, probe)
    assert_same(probe, ov, of, gv, gf)
    t.close()


@pytest.mark.parametrize("sort_gets", [False, True])
def test_mixed_zipf_batches_vs_oracle(lib_ok, sort_gets):
    """Config C3 at small scale: zipf(0.99) key stream, 50 % get / 50 % insert
    (oracle generators = the reference's zipf.h / rand_r restatement), batch
    semantics of SURVEY §8a: each batch's gets see the previous batch's state,
    then its inserts apply in batch order.  Every get result and the final
    contents must equal the oracle's."""
    n_items, batch = 1 << 16, 1 << 14
    t = shm.Tree(arena_bytes=128 << 20, max_batch=1 << 15, sort_gets=sort_gets)
    orc = OracleTree(128 << 20)
    pre = hashed_keys(1, n_items + 1)
    pv = np.arange(1, n_items + 1, dtype=U64) * U64(2)
    gpu_insert(t, pre, pv)
    orc.apply_batch(pre, pv)
    for b in range(4):
        ids = zipf_fill(n_items, 0.99, 0x5EED0000 + b, batch) + U64(1)
        keys = np.array([to_key(int(i)) for i in ids], dtype=U64)
        is_get = op_mix(b + 1, 50, batch).astype(bool)
        op_val = np.arange(b * batch, (b + 1) * batch, dtype=U64) + U64(1)
        gk, pk, pval = keys[is_get], keys[~is_get], op_val[~is_get]
        ov, of = orc.search_batch(gk)
        gv, gf = gpu_search(t, gk)
        assert_same(gk, ov, of, gv, gf)
        gpu_insert(t, pk, pval)
        orc.apply_batch(pk, pval)
    compare_contents(t, orc)
    t.close()


@pytest.mark.parametrize("sort_gets", [False, True])
def test_mixed_batch_gets_see_state_before_its_inserts(lib_ok, sort_gets):
    """shm_mixed_batch (the C3 step): every get returns the oracle's value
    BEFORE the batch's inserts, including keys the same batch overwrites,
    inserts, deletes or never had; the inserts (zipf duplicates, new keys
    that split leaves, value-0 deletes) then leave the oracle's contents."""
    n_items, batch = 1 << 16, 1 << 14
    t = shm.Tree(arena_bytes=128 << 20, max_batch=1 << 15, sort_gets=sort_gets)
    orc = OracleTree(128 << 20)
    pre = hashed_keys(1, n_items + 1)
    pv = np.arange(1, n_items + 1, dtype=U64) * U64(2)
    gpu_insert(t, pre, pv)
    orc.apply_batch(pre, pv)
    splits0 = t.stats()["splits"]
    for b in range(4):
        ids = zipf_fill(2 * n_items, 0.99, 0x5EED1000 + b, batch) + U64(1)
        keys = np.array([to_key(int(i)) for i in ids], dtype=U64)
        is_get = op_mix(b + 7, 50, batch).astype(bool)
        op_val = np.arange(b * batch, (b + 1) * batch, dtype=U64) + U64(1)
        op_val[::97] = 0  # deletes
        gk, pk, pval = keys[is_get], keys[~is_get], op_val[~is_get]
        gk = np.concatenate([gk, pk[:512]])  # keys this batch writes
        ov, of = orc.search_batch(gk)
        k = dev(gk)
        v = torch.empty_like(k)
        f = torch.empty(k.numel(), dtype=torch.uint8, device=k.device)
        t.mixed_batch(k, v, f, dev(pk), dev(pval))
        t.synchronize()
        assert_same(gk, ov, of, host(v), f.cpu().numpy())
        orc.apply_batch(pk, pval)
    assert t.stats()["splits"] > splits0, "no leaf split in the mixed stream"
    compare_contents(t, orc)
    t.close()


def test_leaf_dir_stale_after_splits(lib_ok):
    """The get path starts from the leaf directory (leafdir.hip), built at the
    first search and rebuilt only after the tree grew by 1/32.  Inserts that
    split leaves in between leave entries pointing at pages whose high fence
    moved left; those gets must still be exact (B-link right moves)."""
    n0 = 1 << 18
    t = shm.Tree(arena_bytes=512 << 20, max_batch=1 << 18)
    orc = OracleTree(512 << 20)
    base = hashed_keys(1, n0 + 1)
    bv = np.arange(1, n0 + 1, dtype=U64) * U64(2)
    gpu_insert(t, base, bv)
    orc.apply_batch(base, bv)
    rng = np.random.default_rng(17)
    probe = base[rng.integers(0, n0, 1 << 16)]
    assert_same(probe, *orc.search_batch(probe), *gpu_search(t, probe))  # builds the directory
    pages0 = t.stats()["pages_used"]
    nxt = n0 + 1
    for step in range(3):
        # 30 new keys right after each of 60 existing keys: those leaves
        # overflow and split (~1-2 % more pages, below the rebuild threshold
        # at least for the first step)
        anchors = base[rng.integers(0, n0, 60)]
        add = np.unique((anchors[:, None] + np.arange(1, 31, dtype=U64)[None, :]).ravel())
        add = add[~np.isin(add, base)]
        av = np.arange(nxt, nxt + add.size, dtype=U64) * U64(7)
        nxt += add.size
        gpu_insert(t, add, av)
        orc.apply_batch(add, av)
        probe = np.concatenate([add, add + U64(1 << 20), base[rng.integers(0, n0, 30000)]])
        assert_same(probe, *orc.search_batch(probe), *gpu_search(t, probe))
        # range scans over the split leaves: the stale directory still names
        # the pre-split leaves, so a scan's start may lie left of its key and
        # the walk must take the new pages from the sibling pointers
        slo = np.concatenate([anchors - np.minimum(anchors, U64(5)),
                              base[rng.integers(0, n0, 200)]])
        span = np.concatenate([np.full(60, 200, dtype=U64),
                               (U64(1) << U64(52)) * rng.integers(1, 8, 200).astype(U64)])
        shi = slo + span
        shi[shi < slo] = U64((1 << 64) - 1)
        counts, vals = t.range_query_batch(dev(slo), dev(shi))
        counts = counts.cpu().numpy()
        vals = host(vals)
        off = 0
        for i in range(slo.size):
            ref, n = orc.range_query(int(slo[i]), int(shi[i]), cap=60000)
            assert counts[i] == n
            assert np.array_equal(np.sort(vals[off:off + n]), np.sort(ref))
            off += n
        if step == 0:
            assert pages0 < t.stats()["pages_used"] <= pages0 + pages0 // 32
    assert t.stats()["pages_used"] > pages0
    compare_contents(t, orc)
    t.close()


def test_shard_key_range_hint(lib_ok):
    """A range shard (shm_config key_lo / key_bits, here shard 5 of 8) orders
    gets and builds its leaf directory over its own slice; keys outside the
    slice are still stored and found exactly."""
    from sherman_amd.shard import owner_of, shard_range
    lo, bits = shard_range(5, 8)
    t = shm.Tree(arena_bytes=512 << 20, max_batch=1 << 18, key_lo=lo, key_bits=bits)
    orc = OracleTree(512 << 20)
    allk = hashed_keys(1, 1 << 20)
    own = owner_of(torch.from_numpy(allk.view(np.int64)), 8).numpy()
    mine = allk[own == 5]                                   # ~131 K keys in the slice
    stray = allk[own != 5][:3000]                           # outside the hint
    keys = np.concatenate([mine, stray])
    vals = np.arange(1, keys.size + 1, dtype=U64) * U64(3)
    for c in range(0, keys.size, 1 << 17):
        gpu_insert(t, keys[c:c + (1 << 17)], vals[c:c + (1 << 17)])
        orc.apply_batch(keys[c:c + (1 << 17)], vals[c:c + (1 << 17)])
    rng = np.random.default_rng(23)
    probe = np.concatenate([mine[rng.integers(0, mine.size, 1 << 17)], stray,
                            allk[own != 5][3000:6000]])      # strays and misses
    rng.shuffle(probe)
    assert_same(probe, *orc.search_batch(probe), *gpu_search(t, probe))
    compare_contents(t, orc)
    t.close()


def test_insert_with_colliding_lock_words(lib_ok):
    """Three lock words for the whole arena: every wave of the in-place
    upsert (four leaves per wave) collides on its lock words with itself and
    with other waves, so the ordered one-at-a-time acquisition path runs.
    Contents must still equal the oracle's after updates, new keys and
    splits."""
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 16, num_locks=3)
    orc = OracleTree(256 << 20)
    base = hashed_keys(1, 60001)
    bv = np.arange(1, base.size + 1, dtype=U64)
    gpu_insert(t, base, bv)
    orc.apply_batch(base, bv)
    rng = np.random.default_rng(29)
    for r in range(3):
        upd = base[rng.integers(0, base.size, 30000)]             # updates + duplicates
        new = hashed_keys(100000 + 20000 * r, 100000 + 20000 * r + 8000)
        keys = np.concatenate([upd, new])
        rng.shuffle(keys)
        vals = np.arange(1, keys.size + 1, dtype=U64) + U64(10 ** 7 * (r + 1))
        gpu_insert(t, keys, vals)
        orc.apply_batch(keys, vals)
    compare_contents(t, orc)
    t.close()


def test_searches_on_two_streams_with_an_insert_between(lib_ok):
    """Cross-stream ordering (tree.cpp Order): ordered searches alternate over
    two streams and two get workspaces; an insert issued on a third stream is
    seen by every search issued after it (host order), on either stream."""
    n = 1 << 16
    keys = hashed_keys(1, n + 1)
    vals = np.arange(1, n + 1, dtype=U64) * U64(2)
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 16)
    orc = OracleTree(256 << 20)
    gpu_insert(t, keys, vals)
    orc.apply_batch(keys, vals)
    t.synchronize()
    rng = np.random.default_rng(5)
    s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    new_k = hashed_keys(n + 1, n + 20001)
    new_v = np.arange(1, new_k.size + 1, dtype=U64) * U64(7)
    pool = np.concatenate([keys, new_k])
    plan = []
    for i in range(8):
        q = pool[rng.integers(0, pool.size, 1 << 15)]
        plan.append(("get", q))
        if i == 3:
            plan.append(("put", None))
    outs, want = [], []
    for j, (kind, q) in enumerate(plan):
        if kind == "put":
            t.insert_batch(dev(new_k), dev(new_v), stream=s3)
            orc.apply_batch(new_k, new_v)
            continue
        st = s1 if j % 2 else s2
        with torch.cuda.stream(st):
            k = dev(q)
            v = torch.empty_like(k)
            f = torch.empty(k.numel(), dtype=torch.uint8, device=k.device)
        t.search_batch(k, v, f, stream=st)
        outs.append((q, v, f, k))
        want.append(orc.search_batch(q))
    torch.cuda.synchronize()
    for (q, v, f, _), (ov, of) in zip(outs, want):
        assert_same(q, ov, of, host(v), f.cpu().numpy())
    t.check()
    t.close()
    orc.close()


def test_async_interleaved_searches_and_split_inserts(lib_ok):
    """The ordering that replaces the get fast path's page-level
    check_consistent (Tree.h:241-261; the summary walk checks only entry
    versions): nothing but the library's cross-stream events (device-scope,
    hipEventDisableSystemFence) orders these calls.  Twelve rounds, no host
    wait anywhere: a search batch on stream A or B, then an async insert on
    stream C that splits leaves (new keys next to stored ones), updates and
    deletes.  Every search must equal the oracle's state at its point in
    host call order: a search that overlapped an insert on the device would
    read torn pages or a half-applied batch."""
    n = 1 << 16
    keys = hashed_keys(1, n + 1)
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 16)
    orc = OracleTree(256 << 20)
    gpu_insert(t, keys, keys + U64(1))
    orc.apply_batch(keys, keys + U64(1))
    t.synchronize()
    rng = np.random.default_rng(2024)
    sa, sb, sc = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    nxt = n + 1
    outs, want, keep = [], [], []
    for r in range(12):
        st = sa if r % 2 else sb
        q = np.concatenate([keys[rng.integers(0, keys.size, 20000)],
                            hashed_keys(nxt - 3000, nxt + 1000)])
        with torch.cuda.stream(st):
            k = dev(q)
            v = torch.empty_like(k)
            f = torch.empty(k.numel(), dtype=torch.uint8, device=k.device)
        t.search_batch(k, v, f, stream=st)
        outs.append((q, v, f))
        want.append(orc.search_batch(q))
        keep.append(k)
        add = hashed_keys(nxt, nxt + 6000)
        nxt += 6000
        upd = keys[rng.integers(0, keys.size, 3000)]
        dels = keys[rng.integers(0, keys.size, 500)]
        ik = np.concatenate([add, upd, dels])
        iv = np.concatenate([add ^ U64(r + 5), upd + U64(r + 9), np.zeros(dels.size, dtype=U64)])
        with torch.cuda.stream(sc):
            dk, dv = dev(ik), dev(iv)
        t.insert_batch_async(dk, dv, stream=sc)
        orc.apply_batch(ik, iv)
        keep += [dk, dv]
    t.synchronize()
    torch.cuda.synchronize()
    for (q, v, f), (ov, of) in zip(outs, want):
        assert_same(q, ov, of, host(v), f.cpu().numpy())
    assert t.stats()["splits"] > 0
    compare_contents(t, orc)
    t.close()
    orc.close()


def test_insert_bin_overflow_reorders(lib_ok):
    """Clustered keys put > 6144 ops into one ordering bin: k_bin_unique sorts
    that bin on the device with its global-scratch LSD radix path
    (isort.hip big_bin_unique) with the same result; a bin of <= 6144
    clustered keys takes the LDS bitonic fallback inside the bin."""
    t = shm.Tree(arena_bytes=64 << 20, max_batch=1 << 14)
    orc = OracleTree(64 << 20)
    rng = np.random.default_rng(11)
    for n in (12000, 5000, 16000):
        ks = (np.arange(1, n + 1, dtype=U64) * U64(3))[rng.permutation(n)]
        ks = np.concatenate([ks, ks[: n // 10]])                 # duplicates
        vs = np.arange(1, ks.size + 1, dtype=U64) + U64(n << 20)
        vs[rng.random(ks.size) < 0.03] = 0                         # deletes
        gpu_insert(t, ks, vs)
        orc.apply_batch(ks, vs)
        probe = np.arange(0, 3 * n + 10, dtype=U64)
        ov, of = orc.search_batch(probe)
        gv, gf = gpu_search(t, probe)
        assert_same(probe, ov, of, gv, gf)
    t.check()
    t.close()
    orc.close()


@pytest.mark.parametrize("from_image", [False, True])
def test_leaf_occupancy_bound_with_holes(lib_ok, from_image):
    """Gets read a leaf only up to its occupancy bound (leaf_hw, layout.h):
    leaves with deleted slots below and above the last valid one, slots
    reused by later inserts, pages rewritten by splits, and pages of a loaded
    image (bound unknown until first rewritten) all answer as the oracle."""
    rng = np.random.default_rng(77 + int(from_image))
    universe = hashed_keys(1, 40001)
    orc = OracleTree(256 << 20)
    orc.apply_batch(universe, universe + U64(3))
    dels = universe[rng.random(universe.size) < 0.5]
    orc.apply_batch(dels, np.zeros(dels.size, dtype=U64))
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 16)
    if from_image:
        t.load_image(orc.image(), orc.root_ptr)
    else:
        gpu_insert(t, universe, universe + U64(3))
        gpu_insert(t, dels, np.zeros(dels.size, dtype=U64))
    probe = np.concatenate([universe, hashed_keys(50001, 52001)])
    for r in range(6):
        ov, of = orc.search_batch(probe)
        gv, gf = gpu_search(t, probe)
        assert_same(probe, ov, of, gv, gf)
        # re-insert deleted keys (hole reuse), add new keys (slots past the
        # old bound, splits), delete the highest-slot keys of some leaves
        ks = np.concatenate([dels[rng.integers(0, dels.size, 3000)],
                             hashed_keys(60001 + 4000 * r, 62001 + 4000 * r),
                             universe[rng.integers(0, universe.size, 2000)]])
        vs = rng.integers(1, 1 << 62, ks.size).astype(U64)
        vs[-2000:][rng.random(2000) < 0.5] = 0
        gpu_insert(t, ks, vs)
        orc.apply_batch(ks, vs)
    compare_contents(t, orc)
    t.close()


def test_async_inserts_grow_from_empty_tree(lib_ok):
    """shm_insert_batch_async: batches queued without any host wait, from an
    empty tree (the root leaf splits, the root page is relocated and grows
    several levels inside one batch, k_upper) through small batches, in-batch
    duplicates and deletes; searches queued between the batches see exactly
    the state after the batches before them; one synchronize at the end."""
    rng = np.random.default_rng(4242)
    t = shm.Tree(arena_bytes=512 << 20, max_batch=1 << 18)
    orc = OracleTree(512 << 20)
    universe = hashed_keys(1, 400001)
    plan = [300000, 1, 37, 4096, 50000, 200000, 120000]
    pend = []
    keep = []
    for i, b in enumerate(plan):
        ks = universe[rng.integers(0, universe.size if i else 300000, b)]
        vs = rng.integers(1, 1 << 62, b).astype(U64)
        if i >= 3:
            vs[rng.random(b) < 0.05] = 0
        dk, dv = dev(ks), dev(vs)
        t.insert_batch_async(dk, dv)
        orc.apply_batch(ks, vs)
        probe = universe[rng.integers(0, universe.size, 20000)]
        pk = dev(probe)
        pv = torch.empty_like(pk)
        pf = torch.empty(pk.numel(), dtype=torch.uint8, device=pk.device)
        t.search_batch(pk, pv, pf)
        pend.append((probe, pv, pf) + orc.search_batch(probe))
        keep += [dk, dv, pk]
    t.synchronize()
    for probe, pv, pf, ov, of in pend:
        assert_same(probe, ov, of, host(pv), pf.cpu().numpy())
    st = compare_contents(t, orc)
    assert t.stats()["height"] >= 3, st
    t.close()
    orc.close()


def test_async_batch_with_kkeymax_is_rejected_and_reported(lib_ok):
    """A queued batch holding kKeyMax is dropped whole on the device and the
    error surfaces at the next synchronising call -- here a range scan, not
    an insert -- naming the chunk that failed (shm_last_error), not the call
    that read it; batches after it apply."""
    t = shm.Tree(arena_bytes=32 << 20, max_batch=4096)
    bad_k = dev(np.array([5, (1 << 64) - 1, 6], dtype=U64))
    bad_v = dev(np.array([1, 2, 3], dtype=U64))
    ok_k, ok_v = dev(np.array([7], dtype=U64)), dev(np.array([70], dtype=U64))
    t.insert_batch_async(ok_k, ok_v)
    t.insert_batch_async(bad_k, bad_v)
    bad_chunk = t.last_chunk()
    t.insert_batch_async(ok_k, ok_v)
    assert t.last_chunk() == bad_chunk + 1
    with pytest.raises(shm.ShermanError) as ei:
        t.range_query_batch(dev(np.array([0], dtype=U64)), dev(np.array([100], dtype=U64)))
    assert ei.value.rc == shm.SHM_EINVAL
    e = t.last_error()
    assert e["chunk"] == bad_chunk and e["bits"] & (1 << 31) and e["status"] == shm.SHM_EINVAL, e
    assert t.search(5) == (False, 0) and t.search(6) == (False, 0)
    assert t.search(7) == (True, 70)
    t.synchronize()  # reported once
    t.check()
    t.close()


def test_kkeymax_on_two_streams_both_reported(lib_ok):
    """the error word is cleared by the atomic exchange that reads
    it, not by a memset on the reading call's stream, so a rejected chunk on
    a second stream right after a synchronised one is still reported."""
    t = shm.Tree(arena_bytes=32 << 20, max_batch=4096)
    bad_k = dev(np.array([5, (1 << 64) - 1], dtype=U64))
    bad_v = dev(np.array([1, 2], dtype=U64))
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for s in (s1, s2, s1):
        with torch.cuda.stream(s):
            with pytest.raises(shm.ShermanError) as ei:
                t.insert_batch(bad_k, bad_v, stream=s)
            assert ei.value.rc == shm.SHM_EINVAL
            assert t.last_error()["chunk"] == t.last_chunk()
    t.synchronize()
    assert t.search(5) == (False, 0)
    t.close()


def _right_moves(t, probe):
    t.profile(False, index_stats=True)
    gpu_search(t, probe)
    st = t.index_stats()
    t.profile(False)
    return st["right_moves"]


@pytest.mark.parametrize("lists", [False, True])
def test_forced_handoff_abort_resumes(lib_ok, lists):
    """k_upper's blocks giving up at their first phase hand-off (forced by the
    diagnostic shm__upper_force; in a real run a timed-out wait).  The
    chunk's leaf splits are linked by sibling pointers when they stop; the
    launch's last block then runs the parent levels and the deletes again
    alone (Tree.cpp:973-988 always completes the parent insert), so nothing
    is dropped: the call returns SHM_OK, shm_last_error shows the hand-off
    bit, the chunk id and one completed chunk, the contents (deletes
    included) equal the oracle, and the right moves per get equal those of
    a tree that never gave up.  lists: the chunk propagates through the
    level lists (the bulk-load path) instead of the direct path."""
    H = shm._hooks()
    rng = np.random.default_rng(77)
    trees = [shm.Tree(arena_bytes=256 << 20, max_batch=1 << 16) for _ in range(2)]
    orc = OracleTree(256 << 20)
    ks = hashed_keys(1, 60001)
    for t in trees:
        gpu_insert(t, ks, ks ^ U64(0x33))
    orc.apply_batch(ks, ks ^ U64(0x33))
    new = hashed_keys(100001, 130001)
    dels = rng.choice(ks, 3000, replace=False)
    k = np.concatenate([new, dels])
    v = np.concatenate([np.arange(1, new.size + 1, dtype=U64) * U64(7),
                        np.zeros(dels.size, dtype=U64)])
    for i, t in enumerate(trees):
        flags = (1 if i == 0 else 0) | (2 if lists else 0)
        assert H.shm__upper_force(t.h, flags) == 0
        gpu_insert(t, k, v)  # SHM_OK: completed inside the launch
    orc.apply_batch(k, v)
    e = trees[0].last_error()
    assert e["bits"] & 0x100 and e["chunk"] == trees[0].last_chunk(), e
    assert e["resumed"] == 1 and e["status"] == shm.SHM_OK, e
    assert trees[1].last_error()["resumed"] == 0
    for t in trees:
        compare_contents(t, orc)
    probe = np.concatenate([ks, new, hashed_keys(900001, 901001)])
    rm = [_right_moves(t, probe) for t in trees]
    assert rm[0] <= rm[1] + probe.size // 100 + 16, rm
    # later chunks (splits, root growth, deletes) run normally
    for r in range(2):
        add = hashed_keys(200001 + 20000 * r, 220001 + 20000 * r)
        d2 = rng.choice(ks, 2000, replace=False)
        kk = np.concatenate([add, d2])
        vv = np.concatenate([add ^ U64(r + 1), np.zeros(d2.size, dtype=U64)])
        gpu_insert(trees[0], kk, vv)
        orc.apply_batch(kk, vv)
    compare_contents(trees[0], orc)
    ov, of = orc.search_batch(probe)
    gv, gf = gpu_search(trees[0], probe)
    assert_same(probe, ov, of, gv, gf)
    orc.close()
    for t in trees:
        t.close()


def test_async_forced_abort_completed_before_next_call(lib_ok):
    """An async chunk whose blocks give up at their hand-off is completed by
    the launch's last block, before the next call on the handle (a range scan
    here) reads the tree: the scan sees the chunk's inserts and deletes, and
    shm_last_error, read by that scan, names the chunk."""
    H = shm._hooks()
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 16)
    orc = OracleTree(256 << 20)
    ks = hashed_keys(1, 40001)
    gpu_insert(t, ks, ks + U64(1))
    orc.apply_batch(ks, ks + U64(1))
    new = hashed_keys(50001, 70001)
    dels = ks[::7].copy()
    k = np.concatenate([new, dels])
    v = np.concatenate([new + U64(5), np.zeros(dels.size, dtype=U64)])
    assert H.shm__upper_force(t.h, 1) == 0
    dk, dv = dev(k), dev(v)
    t.insert_batch_async(dk, dv)
    chunk = t.last_chunk()
    orc.apply_batch(k, v)
    lo = np.array([0], dtype=U64)
    hi = np.array([(1 << 64) - 2], dtype=U64)
    counts, vals = t.range_query_batch(dev(lo), dev(hi))
    ok, ov = orc.dump()
    assert int(counts.cpu().numpy()[0]) == ok.size
    e = t.last_error()
    assert e["chunk"] == chunk and e["bits"] & 0x100 and e["resumed"] == 1, e
    compare_contents(t, orc)
    orc.close()
    t.close()


# A second process that holds 240 of the GPU's 256 CUs: each block of
# shm__hog declares a whole CU's LDS and spins on the wall clock.  A separate
# process, so its kernel is on a hardware queue of its own (two streams of
# one process may share a queue and then run in order).
HOG_SRC = r"""
import ctypes, sys, time
L = ctypes.CDLL(sys.argv[1])
L.shm__hog.restype = ctypes.c_int
L.shm__hog.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p]
hip = ctypes.CDLL("libamdhip64.so")
hip.hipDeviceSynchronize()  # runtime up before the clock starts
assert L.shm__hog(240, int(sys.argv[2]), None) == 0
time.sleep(0.5)  # the blocks are dispatched
print("started", flush=True)
assert hip.hipDeviceSynchronize() == 0
print("done", flush=True)
"""


@pytest.mark.parametrize("lists", [False, True])
def test_split_insert_beside_cu_hog(lib_ok, lists):
    """Forward progress of the split propagation: another
    process holds 240 of the 256 CUs for 4 s while a split-heavy insert
    with deletes runs on the rest.  k_upper's phases hand work out by ticket
    and never wait for a block that is not running, so the insert returns
    SHM_OK with oracle-equal contents while the hog still holds its CUs (a
    grid barrier over 256 blocks would have waited for the hog, or timed
    out).  lists: through the level lists and their hand-offs."""
    import subprocess
    import sys
    import time
    H = shm._hooks()
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 17)
    orc = OracleTree(256 << 20)
    ks = hashed_keys(1, 50001)
    gpu_insert(t, ks, ks + U64(3))
    orc.apply_batch(ks, ks + U64(3))
    new = hashed_keys(60001, 160001)  # 2x the tree: splits everywhere
    dels = ks[::5].copy()
    k = np.concatenate([new, dels])
    v = np.concatenate([new ^ U64(9), np.zeros(dels.size, dtype=U64)])
    dk, dv = dev(k), dev(v)
    gpu_search(t, ks[:1000])  # the leaf directory is current: no reallocation
    torch.cuda.synchronize()
    if lists:
        assert H.shm__upper_force(t.h, 2) == 0
    proc = subprocess.Popen([sys.executable, "-c", HOG_SRC, shm.LIB_PATH, str(400_000_000)],
                            stdout=subprocess.PIPE, text=True)
    try:
        assert proc.stdout.readline().strip() == "started"
        t0 = time.time()
        t.insert_batch(dk, dv)
        took = time.time() - t0
        assert proc.poll() is None, f"the insert ({took:.2f} s) outlasted the CU hog"
    finally:
        proc.wait(timeout=60)
    assert proc.returncode == 0
    orc.apply_batch(k, v)
    assert t.last_error()["bits"] == 0
    compare_contents(t, orc)
    orc.close()
    t.close()


def test_lookback_kernels_of_two_trees_side_by_side(lib_ok):
    """The decoupled look-backs (k_bin_unique's bin prefix, k_seg_fill,
    k_scan_u64) of two trees queued side by side on two streams: each
    ordering's 256 bin blocks want a CU each, so the two launches share the
    card.  The bin prefix and the scans take their block index by ticket
    (lookback_index, device_common.h; k_seg_fill keeps blockIdx by default,
    tree.cpp lb_ctr) and wait only on running blocks: every chunk ends with
    no error bit (kErrBinSpin / kErrSegSpin / kErrScanSpin among them) and
    both trees hold the oracle's contents and scan counts."""
    rng = np.random.default_rng(777)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    trees = [shm.Tree(arena_bytes=256 << 20, max_batch=1 << 16) for _ in range(2)]
    orcs = [OracleTree(256 << 20) for _ in range(2)]
    keep = []  # the queued batches' tensors stay alive until the end
    for r in range(6):
        batches = []
        keep.append(batches)
        for i in range(2):
            k = rng.integers(1, 1 << 62, size=1 << 16, dtype=np.int64).astype(U64)
            v = k ^ U64(0x55)
            batches.append((dev(k), dev(v)))
            orcs[i].apply_batch(k, v)
        torch.cuda.synchronize()
        for i in range(2):
            trees[i].insert_batch_async(*batches[i], stream=streams[i])
    lo = np.sort(rng.integers(1, 1 << 62, size=1 << 14, dtype=np.int64).astype(U64))
    hi = lo + U64(1 << 52)
    pend = [trees[i].range_query_batch_async(dev(lo), dev(hi), stream=streams[i])
            for i in range(2)]
    for i in range(2):
        counts, _ = pend[i].result()
        trees[i].synchronize()
        ok, _ = orcs[i].dump()
        ok = np.sort(ok)
        want = np.searchsorted(ok, hi, side="right") - np.searchsorted(ok, lo, side="left")
        assert np.array_equal(host(counts).astype(np.int64), want.astype(np.int64))
        assert trees[i].last_error()["bits"] == 0
        compare_contents(trees[i], orcs[i])
    for i in range(2):
        orcs[i].close()
        trees[i].close()


def early_pages(t):
    x = ctypes.c_uint64()
    assert shm._hooks().shm__early_pages(t.h, ctypes.byref(x)) == 0
    return x.value


def test_early_splits_match_k_upper_splits(lib_ok):
    """Small splits built by the upsert kernel itself (early, upsert.hip) and
    the same chunks with every split left to k_upper (shm__upper_force bit 2)
    both give the oracle's contents and B-link invariants after every chunk;
    early chunks took pages of their own, forced ones none."""
    rng = np.random.default_rng(4242)
    H = shm._hooks()
    trees = {m: shm.Tree(arena_bytes=256 << 20, max_batch=1 << 16) for m in ("early", "late")}
    orc = OracleTree(256 << 20)
    universe = hashed_keys(1, 120001)
    pre = universe[:20000]
    for t in trees.values():
        gpu_insert(t, pre, pre + U64(5))
    orc.apply_batch(pre, pre + U64(5))
    took = []
    for _ in range(6):
        b = int(rng.integers(8000, 1 << 16))
        ks = universe[rng.integers(0, universe.size, b)]
        vs = rng.integers(1, 1 << 62, b).astype(U64)
        vs[rng.random(b) < 0.05] = 0  # deletes
        for mode, t in trees.items():
            if mode == "late":
                assert H.shm__upper_force(t.h, 4) == 0
            gpu_insert(t, ks, vs)
            ep = early_pages(t)
            if mode == "late":
                assert ep == 0
            else:
                took.append(ep)
        orc.apply_batch(ks, vs)
        for t in trees.values():
            compare_contents(t, orc)
    assert orc.check()[0] == 0
    assert sum(took) > 0, took
    for t in trees.values():
        t.close()


def test_early_split_block_list_overflow(lib_ok):
    """Every leaf of a 3M-key tree splits in one chunk: a block of the upsert
    kernel finds more small splits than its early list holds (64), so the
    chunk has early splits and k_upper splits side by side.  Every key reads
    back with its value and the tree keeps its invariants (size-independent
    properties: the oracle would take minutes at this size)."""
    n = 3_000_000
    t = shm.Tree(arena_bytes=1 << 30, max_batch=1 << 22)
    ev = np.arange(1, n + 1, dtype=U64) * U64(2)
    gpu_insert(t, ev, ev + U64(1))  # a leaf root at first: all of it k_upper's
    od = ev + U64(1)  # every leaf gets as many new keys as it holds
    gpu_insert(t, od, od * U64(3))
    assert early_pages(t) > 0
    allk = np.concatenate([ev, od])
    v, f = gpu_search(t, allk)
    assert f.all(), int((f == 0).sum())
    assert np.array_equal(v, np.concatenate([ev + U64(1), od * U64(3)]))
    st = t.check()
    assert st["keys"] == 2 * n, st
    t.close()


def test_directory_ties_start_at_the_leaf(lib_ok):
    """A directory entry's split points are the top 32 bits of each leaf's
    lowest fence within the prefix, so a lookup of a leaf's FIRST key ties
    with its split point (round 4: 2.7 % of C2's gets did, and started one
    leaf to the left).  A tie now starts at the leaf itself and falls back to
    the safe start only when the key is not there: with a fresh directory,
    gets and in-place updates of every leaf's first key make no right move,
    and keys just below / above those fences (absent) still come back
    exactly as the oracle says."""
    t = shm.Tree(arena_bytes=512 << 20, max_batch=1 << 18)
    orc = OracleTree(512 << 20)
    ks = hashed_keys(1, 300001)
    for c in range(0, ks.size, 1 << 17):
        gpu_insert(t, ks[c:c + (1 << 17)], ks[c:c + (1 << 17)] ^ U64(0x55))
    orc.apply_batch(ks, ks ^ U64(0x55))
    img, _ = t.dump_image()
    pg = np.frombuffer(img, dtype=np.uint8)[1024:].reshape(-1, 1024)
    leftmost = pg[:, 9:17].copy().view(U64).ravel()
    lowest = pg[:, 28:36].copy().view(U64).ravel()
    seps = np.unique(lowest[(leftmost == 0) & (lowest != 0)])
    seps = seps[np.isin(seps, ks)]  # every leaf's first key (stored)
    assert seps.size > 1000
    for _ in range(6):  # a read phase: the directory is rebuilt exact
        gpu_search(t, ks[:4096])
    t.profile(False, index_stats=True)
    gv, gf = gpu_search(t, seps)
    st = t.index_stats()
    assert st["right_moves"] == 0, st
    assert_same(seps, *orc.search_batch(seps), gv, gf)
    near = np.concatenate([seps - U64(1), seps + U64(1)])
    gv, gf = gpu_search(t, near)
    t.profile(False)
    assert_same(near, *orc.search_batch(near), gv, gf)
    # in-place updates of the first keys, then new keys right below them
    # (they belong to the leaf on the left): contents equal the oracle
    upd_v = seps ^ U64(0xABC)
    gpu_insert(t, seps, upd_v)
    orc.apply_batch(seps, upd_v)
    below = seps[:2000] - U64(1)
    below = below[~np.isin(below, ks)]
    gpu_insert(t, below, below + U64(9))
    orc.apply_batch(below, below + U64(9))
    compare_contents(t, orc)
    orc.close()
    t.close()


@pytest.mark.parametrize("start", ["dir", "lds", "root"])
def test_get_start_modes_and_index_stats(lib_ok, start):
    """The summary walk from each start: the leaf directory, the LDS replica
    of the top levels (SHM_FLAG_TOP_LDS: every page of the deepest upper
    level that fits 4096 entries, binary-searched in LDS) and the root.
    Same answers as the oracle through growth (the replica and the directory
    go stale and are rebuilt); the index statistics count what each start
    costs: from the directory almost every get starts at its leaf, from the
    replica or the root every get starts at an internal page."""
    t = shm.Tree(arena_bytes=512 << 20, max_batch=1 << 18, leaf_dir=start == "dir",
                 top_lds=start == "lds")
    orc = OracleTree(512 << 20)
    rng = np.random.default_rng(99)
    for r in range(3):
        ks = hashed_keys(1 + 150000 * r, 1 + 150000 * (r + 1))
        gpu_insert(t, ks, ks ^ U64(r + 3))
        orc.apply_batch(ks, ks ^ U64(r + 3))
        ok, _ = orc.dump()
        probe = np.concatenate([ok[rng.integers(0, ok.size, 60000)],
                                rng.integers(1, 1 << 63, 5000, dtype=np.int64).astype(U64)])
        t.profile(False, index_stats=True)
        gv, gf = gpu_search(t, probe)
        st = t.index_stats()
        t.profile(False)
        ov, of = orc.search_batch(probe)
        assert_same(probe, ov, of, gv, gf)
        assert st["gets"] == probe.size and st["hits"] == int(of.sum())
        assert st["dir_fp_hits"] <= st["hits"], st
        if start == "dir":
            assert st["start_internal"] < probe.size // 100, st
            # most prefixes lie inside one leaf: their gets are answered from
            # the directory entry's fingerprints (the misses never are)
            assert st["dir_fp_hits"] > st["hits"] // 4, st
        else:
            assert st["dir_fp_hits"] == 0, st
            assert st["start_internal"] == probe.size, st
            assert st["page_hops"] >= probe.size * (1 if start == "lds" else 2), st
            # the replica's page is the one holding k (no walk along a level)
            hops = t.stats()["height"] - (2 if start == "lds" else 1)
            assert st["page_hops"] <= probe.size * hops, (st, hops)
        assert st["right_moves"] < probe.size // 10, st
    assert t.stats()["height"] >= 3
    orc.close()
    t.close()


def test_lock_bench_contended_words(lib_ok):
    """Tree::lock_bench (Tree.cpp:310-321) over the HBM lock table: 2^17 keys
    on 100 distinct lock words (lanes of one wave contend for one word)
    finish without a lock error, and every word is free afterwards (an
    insert that takes the words of its pages succeeds)."""
    t = shm.Tree(arena_bytes=64 << 20, max_batch=1 << 14)
    orc = OracleTree(64 << 20)
    ks = hashed_keys(1, 20001)
    gpu_insert(t, ks, ks + U64(1))
    orc.apply_batch(ks, ks + U64(1))
    rng = np.random.default_rng(3)
    t.lock_bench(dev(rng.integers(1, 101, 1 << 17).astype(U64)))
    t.synchronize()
    more = hashed_keys(30001, 40001)
    gpu_insert(t, more, more + U64(2))
    orc.apply_batch(more, more + U64(2))
    compare_contents(t, orc)
    orc.close()
    t.close()


def test_pending_range_waits_for_its_issue_stream(lib_ok):
    """range_query_batch_async issued on a side stream (stream=None there
    means that stream) and .result() called outside it: the result waits for
    the stream the scans were queued on, not the one current at .result()."""
    t = shm.Tree(arena_bytes=128 << 20, max_batch=1 << 14)
    ks = hashed_keys(1, 30001)
    gpu_insert(t, ks, ks + U64(7))
    rng = np.random.default_rng(12)
    lo = rng.integers(0, 1 << 63, 400, dtype=np.uint64) * U64(2)
    hi = lo + (U64(1) << U64(54))
    hi[hi < lo] = U64((1 << 64) - 2)
    sc, sv = t.range_query_batch(dev(lo), dev(hi))
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        dlo, dhi = dev(lo), dev(hi)
        pend = t.range_query_batch_async(dlo, dhi)
        # keep the side stream busy behind the scans
        junk = torch.randn(1 << 22, device="cuda")
        for _ in range(20):
            junk = junk * 1.0001
    ac, av = pend.result()
    assert np.array_equal(ac.cpu().numpy(), sc.cpu().numpy())
    assert np.array_equal(host(av), host(sv))
    t.close()


def test_pair_form_directory_reads_through_stale_pairs(lib_ok):
    """A read phase builds the pair-form directory (layout.h kDirPairs: each
    prefix lists its own keys' slots): every get of the current tree is then
    answered from its entry.  Inserts that split leaves, in-place updates and
    deletes follow without a rebuild (below the 1/32 growth rule), so the
    next searches read stale pairs -- moved keys, emptied and overwritten
    slots, keys the pairs never listed -- and must still equal the oracle
    (a pair is only a slot to read; a miss takes the summary walk).  The
    next read phase rebuilds the pairs, and the contents stay exact."""
    n0 = 1 << 18
    t = shm.Tree(arena_bytes=512 << 20, max_batch=1 << 18)
    orc = OracleTree(512 << 20)
    base = hashed_keys(1, n0 + 1)
    bv = np.arange(1, n0 + 1, dtype=U64) * U64(2)
    gpu_insert(t, base, bv)
    orc.apply_batch(base, bv)
    rng = np.random.default_rng(23)
    probe = base[rng.integers(0, n0, 1 << 15)]
    for _ in range(5):  # four searches without an insert: the read phase
        gv, gf = gpu_search(t, probe)
    assert_same(probe, *orc.search_batch(probe), gv, gf)
    t.profile(False, index_stats=True)
    gv, gf = gpu_search(t, probe)
    st = t.index_stats()
    t.profile(False)
    assert_same(probe, *orc.search_batch(probe), gv, gf)
    assert st["dir_fp_hits"] == st["gets"] == probe.size, st  # all from the entries
    # updates, deletes and splitting inserts, no rebuild in between
    upd = base[rng.integers(0, n0, 5000)]
    dele = base[rng.integers(0, n0, 3000)]
    anchors = base[rng.integers(0, n0, 40)]
    add = np.unique((anchors[:, None] + np.arange(1, 31, dtype=U64)[None, :]).ravel())
    add = add[~np.isin(add, base)]
    k = np.concatenate([upd, dele, add])
    v = np.concatenate([upd ^ U64(0x5A5A), np.zeros(dele.size, dtype=U64),
                        np.arange(1, add.size + 1, dtype=U64) * U64(11)])
    pages = t.stats()["pages_used"]
    gpu_insert(t, k, v)
    orc.apply_batch(k, v)
    assert t.stats()["pages_used"] > pages  # leaves split
    probe2 = np.concatenate([upd, dele, add, add + U64(1 << 20),
                             base[rng.integers(0, n0, 20000)]])
    for _ in range(6):  # stale pairs first, then the next read phase's rebuild
        gv, gf = gpu_search(t, probe2)
        assert_same(probe2, *orc.search_batch(probe2), gv, gf)
    rc, oc = orc.check()
    assert rc == 0 and t.check()["keys"] == oc["keys"]
    orc.close()
    t.close()
