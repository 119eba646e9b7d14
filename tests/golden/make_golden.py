"""Regenerates the golden fixtures from the CPU oracle (run from repo root:
`python tests/golden/make_golden.py`).  These pin the oracle's restated
generators (CityHash64 v1.1 len-8 path, test/benchmark.cpp:43-46 to_key,
test/zipf.h mehcached zipf, glibc rand_r op mix) and a reference-rule tree
against regressions.  The reference itself cannot run here,
so the hash values are a self-pin ("parity unpinned at the hash")."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle.pyoracle import (OracleTree, cityhash64_u64, op_mix, to_key,  # noqa
                             zipf_fill)

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ids = list(range(0, 64)) + [1 << 20, (1 << 26) + 7, (1 << 63) + 5, (1 << 64) - 1]
    gen = {
        "cityhash64": [[i, cityhash64_u64(i)] for i in ids],
        "to_key": [[i, ks, to_key(i, ks)] for i in ids[:40] for ks in (0, 64 << 20)],
        "zipf": [],
        "op_mix": [],
    }
    for n, theta, seed in [(64 << 20, 0.0, 0x5EED0000), (64 << 20, 0.99, 0x5EED0001),
                           (1000, 0.5, 7), (1 << 30, 0.0, 0x5EED0002)]:
        gen["zipf"].append({"n": n, "theta": theta, "seed": seed,
                            "draws": zipf_fill(n, theta, seed, 256).tolist()})
    for seed, rr in [(1, 50), (2, 95), (3, 5)]:
        gen["op_mix"].append({"seed": seed, "read_ratio": rr,
                              "ops": op_mix(seed, rr, 256).tolist()})
    with open(os.path.join(HERE, "generators.json"), "w") as f:
        json.dump(gen, f)

    n_keys, n_probe = 100000, 120000
    t = OracleTree(1 << 27)
    keys = np.array([to_key(i) for i in range(1, n_keys + 1)], dtype=np.uint64)
    t.apply_batch(keys, np.arange(1, n_keys + 1, dtype=np.uint64) * np.uint64(2))
    rc, shape = t.check()
    assert rc == 0
    probe = np.array([to_key(i) for i in range(1, n_probe + 1)], dtype=np.uint64)
    v, fnd = t.search_batch(probe)
    fix = {"n_keys": n_keys, "n_probe": n_probe, "shape": shape,
           "found": int(fnd.sum()), "xor_values": int(np.bitwise_xor.reduce(v))}
    with open(os.path.join(HERE, "tree_fixture.json"), "w") as f:
        json.dump(fix, f, indent=1)


if __name__ == "__main__":
    main()
