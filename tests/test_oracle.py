"""CPU oracle checks (no GPU): the oracle is pinned by the reference's own
known-answer test (test/tree_test.cpp:31-68) and by structural invariants,
and its generators by committed golden fixtures (tests/golden/)."""
import json
import os

import numpy as np
import pytest

from oracle.pyoracle import (OracleTree, cityhash64_u64, op_mix, to_key,
                             zipf_fill)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
U64 = np.uint64


def test_tree_test_kat():
    """test/tree_test.cpp:31-68 verbatim (N = 10240), including the delete
    phase the reference only prints."""
    t = OracleTree(1 << 26)
    N = 10240
    for i in range(1, N):
        t.insert(i, i * 2)
    for i in range(N - 1, 0, -1):
        t.insert(i, i * 3)
    for i in range(1, N):
        assert t.search(i) == (True, i * 3)
    for i in range(1, N):
        t.delete(i)
    for i in range(1, N):
        assert t.search(i) == (False, 0)
    for i in range(N - 1, 0, -1):
        t.insert(i, i * 3)
    for i in range(1, N):
        assert t.search(i) == (True, i * 3)
    rc, shape = t.check()
    assert rc == 0
    assert shape["keys"] == N - 1


def test_write_test_shape():
    """test/write_test.cpp:66-70 shape: random hashed inserts; every page
    obeys the reference's occupancy / fence / ordering invariants."""
    t = OracleTree(1 << 28)
    rng = np.random.default_rng(1)
    n = 200000
    ids = 1 + rng.integers(0, n, n)
    keys = np.array([to_key(int(i)) for i in ids], dtype=U64)
    vals = np.arange(1, n + 1, dtype=U64) * U64(2)
    t.apply_batch(keys, vals)
    rc, shape = t.check()
    assert rc == 0
    uniq = {}
    for k, v in zip(keys.tolist(), vals.tolist()):
        uniq[k] = v
    assert shape["keys"] == len(uniq)
    ks, vs = t.dump()
    got = dict(zip(ks.tolist(), vs.tolist()))
    assert got == uniq
    # reference split rule: 54 -> 27/27, random fill ~ 69 %
    fill = shape["keys"] / shape["leaves"] / 54
    assert 0.6 < fill < 0.8


def test_root_growth_and_levels():
    t = OracleTree(1 << 28)
    for i in range(1, 200001):
        t.insert(i, i)
    rc, shape = t.check()
    assert rc == 0
    assert shape["height"] == t.root_level + 1 >= 3


def test_search_read_count_matches_height():
    """DSM.cpp:119-120 counters: one page read per level for a hit."""
    t = OracleTree(1 << 27)
    keys = np.array([to_key(i) for i in range(1, 50001)], dtype=U64)
    t.apply_batch(keys, keys)
    before = t.read_pages
    for k in keys[:1000].tolist():
        assert t.search(k) == (True, k)
    per = (t.read_pages - before) / 1000
    assert per == t.check()[1]["height"]


def test_range_query_intended_semantics():
    t = OracleTree(1 << 27)
    rng = np.random.default_rng(2)
    keys = np.unique(rng.integers(0, 1 << 40, 30000, dtype=np.uint64))
    t.apply_batch(keys, keys + U64(1))
    for _ in range(50):
        a, b = sorted(rng.integers(0, 1 << 40, 2).tolist())
        got, n = t.range_query(a, b)
        ref = keys[(keys >= a) & (keys <= b)] + U64(1)
        assert n == ref.size
        assert np.array_equal(np.sort(got), ref)
    got, n = t.range_query(10, 5)
    assert n == 0


def test_delete_then_reinsert_uses_first_empty_slot():
    """Tree.cpp:890-906: inserts take the first empty slot; deleted slots
    (value == kValueNull) are reusable."""
    t = OracleTree(1 << 22)
    for k in range(1, 11):
        t.insert(k, k)
    t.delete(3)
    t.insert(100, 7)
    img = t.image()
    root = t.root_ptr >> 16
    base = root + 44 + 18 * 2  # slot 2 held key 3
    assert int.from_bytes(img[base + 1:base + 9].tobytes(), "little") == 100
    assert int.from_bytes(img[base + 9:base + 17].tobytes(), "little") == 7
    # entry versions: insert, delete, insert -> f == r == 3 (4-bit)
    assert img[base] & 0xF == 3 and img[base + 17] & 0xF == 3


def test_kkeymax_rejected():
    t = OracleTree(1 << 22)
    assert t.insert((1 << 64) - 1, 5) == -1
    assert t.search((1 << 64) - 1) == (False, 0)


def _golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_golden_cityhash_and_to_key():
    g = _golden("generators.json")
    for i, h in g["cityhash64"]:
        assert cityhash64_u64(i) == h
    for i, ks, k in g["to_key"]:
        assert to_key(i, ks) == k


def test_golden_zipf_and_op_mix():
    g = _golden("generators.json")
    for case in g["zipf"]:
        got = zipf_fill(case["n"], case["theta"], case["seed"], len(case["draws"]))
        assert got.tolist() == case["draws"]
    for case in g["op_mix"]:
        got = op_mix(case["seed"], case["read_ratio"], len(case["ops"]))
        assert got.tolist() == case["ops"]


@pytest.mark.skipif(not os.path.isdir("/root/reference/test"),
                    reason="the reference checkout is not on this machine")
def test_golden_zipf_is_the_reference_generator():
    """The golden zipf draws equal the REFERENCE's own test/zipf.h, compiled
    by path (oracle/Makefile `ref`, tests/golden/make_zipf_ref.py), and so
    does the oracle's restatement on further (n, theta, seed) cases — among
    them C3's and C5's generators (theta 0.99 over 2^26 and 2^31 items)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rc = subprocess.run([sys.executable, os.path.join(root, "tests", "golden",
                                                      "make_zipf_ref.py")])
    assert rc.returncode == 0
    sys.path.insert(0, os.path.join(root, "tests", "golden"))
    from make_zipf_ref import reference_draws
    for n, theta, seed in [(64 << 20, 0.99, 0x5EED0007), (1 << 31, 0.99, 12345),
                           (4000, 0.99, 1), (1 << 20, 0.3, 99), (10, 0.0, 3)]:
        assert zipf_fill(n, theta, seed, 2000).tolist() == reference_draws(n, theta, seed, 2000)


def test_golden_tree_fixture():
    """Reference-rule tree built by the oracle: digest of the search answers
    for a fixed stream (regression pin for the restatement)."""
    g = _golden("tree_fixture.json")
    t = OracleTree(1 << 27)
    keys = np.array([to_key(i) for i in range(1, g["n_keys"] + 1)], dtype=U64)
    vals = np.arange(1, g["n_keys"] + 1, dtype=U64) * U64(2)
    t.apply_batch(keys, vals)
    rc, shape = t.check()
    assert rc == 0
    assert shape == g["shape"]
    probe = np.array([to_key(i) for i in range(1, g["n_probe"] + 1)], dtype=U64)
    v, f = t.search_batch(probe)
    assert int(f.sum()) == g["found"]
    assert int(np.bitwise_xor.reduce(v)) == g["xor_values"]


def test_mt_apply_and_range_match_serial():
    """The CPU baseline's multi-threaded legs (orc_apply_batch_mt partitioned
    by page lock word, orc_range_query_batch_mt) leave the same contents and
    return the same scans as the serial restatement."""
    import numpy as np
    from oracle.pyoracle import OracleTree, to_key
    rng = np.random.default_rng(99)
    universe = np.array([to_key(i) for i in range(1, 60001)], dtype=np.uint64)
    a, b = OracleTree(256 << 20), OracleTree(256 << 20)
    for r in range(6):
        n = 40000 if r else 50000
        ks = universe[rng.integers(0, universe.size, n)]
        vs = rng.integers(1, 1 << 62, n).astype(np.uint64)
        vs[rng.random(n) < 0.1] = 0
        a.apply_batch(ks, vs)
        b.apply_batch_mt(ks, vs, 7)
        ka, va = a.dump()
        kb, vb = b.dump()
        oa, ob = np.argsort(ka), np.argsort(kb)
        assert np.array_equal(ka[oa], kb[ob]) and np.array_equal(va[oa], vb[ob])
        assert b.check()[0] == 0
    lo = rng.integers(0, 1 << 63, 500, dtype=np.uint64) * np.uint64(2)
    hi = lo + (np.uint64(1) << np.uint64(56))
    hi[hi < lo] = np.uint64((1 << 64) - 1)
    ca, xa = b.range_query_batch(lo, hi)
    cb, xb, _ = b.range_query_batch_mt(lo, hi, 5)
    assert np.array_equal(ca, cb) and np.array_equal(xa, xb)
    w = b.c1_bench(2, 1 << 20, windows=2, window_s=0.2)
    assert w.size == 2 and (w > 0).all()
    a.close()
    b.close()
