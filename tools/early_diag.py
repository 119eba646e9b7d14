"""Diagnostic for the early-split overflow case (tests/test_gpu_parity.py::
test_early_split_block_list_overflow): which keys go missing, and where.

    python tools/early_diag.py [n]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sherman_amd as shm  # noqa: E402

U64 = np.uint64


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=U64).view(np.int64)).cuda()


def search(t, keys):
    k = dev(keys)
    v = torch.empty_like(k)
    f = torch.empty(k.numel(), dtype=torch.uint8, device="cuda")
    t.search_batch(k, v, f)
    t.synchronize()
    return v.cpu().numpy().view(U64), f.cpu().numpy()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3_000_000
    t = shm.Tree(arena_bytes=1 << 30, max_batch=1 << 22)
    ev = np.arange(1, n + 1, dtype=U64) * U64(2)
    t.insert_batch(dev(ev), dev(ev + U64(1)))
    v, f = search(t, ev)
    print("after evens: missing", int((f == 0).sum()), "wrong", int((v != ev + U64(1)).sum()),
          t.check(), flush=True)
    od = ev + U64(1)
    t.insert_batch(dev(od), dev(od * U64(3)))
    t.synchronize()
    print("last_error", t.last_error(), flush=True)
    allk = np.concatenate([ev, od])
    want = np.concatenate([ev + U64(1), od * U64(3)])
    v, f = search(t, allk)
    bad = np.nonzero((f == 0) | (v != want))[0]
    print("after odds: bad", bad.size, t.check(), flush=True)
    for i in bad[:10]:
        k = allk[i]
        nb = np.array([k - U64(2), k - U64(1), k, k + U64(1), k + U64(2)], dtype=U64)
        nv, nf = search(t, nb)
        print(f"key {int(k)} idx {i} found {f[i]} val {int(v[i])} want {int(want[i])} "
              f"neighbours {list(zip(nb.tolist(), nf.tolist()))}", flush=True)
    # a range scan over the neighbourhood of the first bad key
    if bad.size:
        k = int(allk[bad[0]])
        lo = dev(np.array([k - 40], dtype=U64))
        hi = dev(np.array([k + 40], dtype=U64))
        try:
            c, vals = t.range_query_batch(lo, hi)
            print("range", int(c[0]), [int(x) for x in vals.cpu().numpy().view(U64)], flush=True)
        except Exception as e:  # noqa: BLE001
            print("range failed", e, flush=True)
    t.close()


if __name__ == "__main__":
    main()
