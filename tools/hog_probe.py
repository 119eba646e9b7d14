"""Diagnostic: does work on another stream run while shm__hog holds CUs?

    python tools/hog_probe.py

Prints the hog's own duration, then how long a torch op and a split-heavy
insert on a second non-blocking stream take while the hog runs, and whether
the hog was still running when each returned.
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sherman_amd as shm  # noqa: E402
from oracle.pyoracle import to_key  # noqa: E402

U64 = np.uint64


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=U64).view(np.int64)).cuda()


def main():
    H = shm._hooks()
    hog = torch.cuda.Stream()
    side = torch.cuda.Stream()
    print("streams", hog.cuda_stream, side.cuda_stream, flush=True)
    # 1. the hog alone
    torch.cuda.synchronize()
    t0 = time.time()
    assert H.shm__hog(240, 50_000_000, ctypes.c_void_p(hog.cuda_stream)) == 0
    ev = torch.cuda.Event()
    ev.record(hog)
    ev.synchronize()
    print(f"hog alone (0.5 s asked): {time.time() - t0:.3f} s", flush=True)
    # 2. a torch op on another stream while the hog runs
    x = torch.ones(1 << 20, device="cuda")
    torch.cuda.synchronize()
    t0 = time.time()
    assert H.shm__hog(240, 100_000_000, ctypes.c_void_p(hog.cuda_stream)) == 0
    ev.record(hog)
    with torch.cuda.stream(side):
        y = x * 2
    e2 = torch.cuda.Event()
    e2.record(side)
    e2.synchronize()
    print(f"torch op beside the hog: {time.time() - t0:.3f} s, hog done: {ev.query()}", flush=True)
    ev.synchronize()
    # 3. an insert beside the hog
    t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 17)
    ks = np.array([to_key(i) for i in range(1, 50001)], dtype=U64)
    t.insert_batch(dev(ks), dev(ks + U64(3)))
    new = np.array([to_key(i) for i in range(60001, 160001)], dtype=U64)
    dk, dv = dev(new), dev(new ^ U64(9))
    probe = dev(ks[:1000])
    pv = torch.empty_like(probe)
    t.search_batch(probe, pv)
    t.synchronize()
    torch.cuda.synchronize()
    for mode in ("search", "insert_async", "insert"):
        t0 = time.time()
        assert H.shm__hog(240, 100_000_000, ctypes.c_void_p(hog.cuda_stream)) == 0
        ev.record(hog)
        with torch.cuda.stream(side):
            if mode == "search":
                t.search_batch(probe, pv, stream=side)
            elif mode == "insert_async":
                t.insert_batch_async(dk, dv, stream=side)
            else:
                t.insert_batch(dk, dv, stream=side)
        t1 = time.time() - t0
        e2.record(side)
        e2.synchronize()
        print(f"{mode} beside the hog: call {t1:.3f} s, done {time.time() - t0:.3f} s, "
              f"hog done at return: {ev.query()}", flush=True)
        ev.synchronize()
    print("last_error", t.last_error(), flush=True)
    # 4. the hog in another process
    import subprocess
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "tests"))
    from test_gpu_parity import HOG_SRC
    for mode in ("search", "insert"):
        proc = subprocess.Popen([sys.executable, "-c", HOG_SRC, shm.LIB_PATH, str(200_000_000)],
                                stdout=subprocess.PIPE, text=True)
        line = proc.stdout.readline().strip()
        t0 = time.time()
        with torch.cuda.stream(side):
            if mode == "search":
                t.search_batch(probe, pv, stream=side)
                t.synchronize()
            else:
                t.insert_batch(dk, dv ^ 5, stream=side)
        took = time.time() - t0
        print(f"{mode} beside a hog process ({line}): {took:.3f} s, hog alive: {proc.poll() is None}",
              flush=True)
        proc.wait(timeout=60)
    t.close()


if __name__ == "__main__":
    main()
