"""k_upper phase clock (diagnostic; run on the GPU box):
    python tools/upper_stamps.py [keys_log2] [batches] [pipe]
Builds a tree of 2^keys_log2 keys, then applies C5-like insert batches
(1 Mi ops, key = to_key(1 + zipf(0.99) over twice the key set)) and C3-like
ones (zipf over the stored keys: updates only) and prints, per batch, the
microseconds between k_upper's phase stamps (block 0's view: prefix sums,
leaf builds, barrier, then I1 / barrier / I2 / I3 / barrier per internal
level, deletes, end)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sherman_amd as shm  # noqa: E402
from sherman_amd.workload import Zipf  # noqa: E402


def main():
    kl = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    pipe = len(sys.argv) > 3 and sys.argv[3] == "pipe"
    s_ord, s_app = torch.cuda.Stream(), torch.cuda.Stream()
    dev = torch.device("cuda:0")
    n = 1 << kl
    t = shm.Tree(arena_bytes=max(2 << 30, n * 1024 // 20), max_batch=1 << 20, device=0)
    keys = torch.empty(1 << 20, dtype=torch.int64, device=dev)
    for c in range(0, n, 1 << 20):
        m = min(1 << 20, n - c)
        t.gen_keys(1 + c, m, keys[:m])
        t.insert_batch(keys[:m], torch.arange(1 + c, 1 + c + m, dtype=torch.int64, device=dev) * 2)
    lib = shm.lib()
    fn = lib.shm__upper_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
    fn(t.h, 1, None)
    out = (ctypes.c_uint64 * (32 + 10 * 256 + 9 * 1024))()
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    for name, zn in (("c5", 2 * n), ("c3", n)):
        z = Zipf(zn, 0.99, dev)
        for b in range(nb):
            ids = z.sample(1 << 20, g) + 1
            k = torch.empty_like(ids)
            t.hash_keys(ids, k)
            v = torch.arange(1, (1 << 20) + 1, dtype=torch.int64, device=dev)
            if pipe and name == "c5":
                # bench's C5 shape: the next chunk's ordering on its own
                # stream beside this chunk's apply (the upsert rows are this
                # chunk's, the ordering rows the next chunk's)
                ids2 = z.sample(1 << 20, g) + 1
                k2 = torch.empty_like(ids2)
                t.hash_keys(ids2, k2)
                s_ord.wait_stream(torch.cuda.current_stream())
                s_app.wait_stream(torch.cuda.current_stream())
                t0_ = t.insert_order(k, v, stream=s_ord)
                t1_ = t.insert_order(k2, v, stream=s_ord)
                t.insert_apply(t0_, stream=s_app)
                torch.cuda.synchronize()
                fn(t.h, 2, out)
                t.insert_apply(t1_, stream=s_app)
                torch.cuda.synchronize()
            else:
                t.insert_batch(k, v)
                fn(t.h, 2, out)
            cnt = int(out[0])
            ts = [int(out[i]) for i in range(1, cnt)]
            d = [round((ts[i] - ts[i - 1]) / 100.0, 1) for i in range(1, len(ts))]  # 100 MHz
            print(name, b, "total %.1f us" % ((ts[-1] - ts[0]) / 100.0), d, flush=True)
            # k_bin_unique: per phase, mean / max over bins of the clock
            # since the earliest bin's start (phases a, b, c, d, prefix, end)
            bs = [[int(out[32 + p * 256 + x]) for x in range(256)] for p in range(7)]
            t0 = min(bs[0])
            row = []
            for p in range(7):
                v = [(x - t0) / 100.0 for x in bs[p] if x]
                row.append("%.1f/%.1f" % (sum(v) / max(len(v), 1), max(v) if v else 0))
            print("   bin_unique phases (mean/max us):", " ".join(row), flush=True)
            upsert_rows(out, ts[0])
            # k_upper per block: start and end clocks since block 0's first stamp
            st = [int(out[32 + 8 * 256 + x]) for x in range(256)]
            en = [int(out[32 + 9 * 256 + x]) for x in range(256)]
            pairs = [(a_, b_) for a_, b_ in zip(st, en) if a_ and b_ >= a_]
            if pairs:
                s0 = ts[0]
                ss = sorted((a_ - s0) / 100.0 for a_, _ in pairs)
                ee = sorted((b_ - s0) / 100.0 for _, b_ in pairs)
                q = lambda v, f: v[min(len(v) - 1, int(f * len(v)))]  # noqa: E731
                print("   k_upper blocks (us since block 0's start): start min/p50/max "
                      "%.1f/%.1f/%.1f, end min/p50/p90/max %.1f/%.1f/%.1f/%.1f" %
                      (ss[0], q(ss, 0.5), ss[-1], ee[0], q(ee, 0.5), q(ee, 0.9), ee[-1]),
                      flush=True)
    fn(t.h, 0, None)
    t.close()


def upsert_rows(out, s0):
    """The upsert kernel's per-block clocks (us since k_upper's block 0
    start of the same chunk is not comparable: relative to the earliest
    upsert block start) and early-split counts."""
    base = 32 + 10 * 256
    st = [int(out[base + x]) for x in range(1024)]
    mid = [int(out[base + 1024 + x]) for x in range(1024)]
    en = [int(out[base + 2048 + x]) for x in range(1024)]
    ne = [int(out[base + 3072 + x]) for x in range(1024)]
    blocks = [i for i in range(1024) if st[i] and en[i] >= st[i]]
    if not blocks:
        return
    t0 = min(st[i] for i in blocks)
    q = lambda v, f: v[min(len(v) - 1, int(f * len(v)))]  # noqa: E731
    ss = sorted((st[i] - t0) / 100.0 for i in blocks)
    mm = sorted((mid[i] - t0) / 100.0 for i in blocks if mid[i])
    ee = sorted((en[i] - t0) / 100.0 for i in blocks)
    sp = sorted((en[i] - mid[i]) / 100.0 for i in blocks if mid[i] and ne[i])
    hist = {}
    for i in blocks:
        hist[ne[i]] = hist.get(ne[i], 0) + 1
    print("   upsert blocks %d: start p50/max %.1f/%.1f, in-place done p50/p90/max %.1f/%.1f/%.1f, "
          "end p50/p90/max %.1f/%.1f/%.1f; split time (blocks with splits) p50/p90/max %s; "
          "early splits per block %s" %
          (len(blocks), q(ss, .5), ss[-1], q(mm, .5) if mm else 0, q(mm, .9) if mm else 0,
           mm[-1] if mm else 0, q(ee, .5), q(ee, .9), ee[-1],
           "%.1f/%.1f/%.1f" % (q(sp, .5), q(sp, .9), sp[-1]) if sp else "-",
           dict(sorted(hist.items()))), flush=True)
    # the first early split of each block: its phases (us)
    ph = [[int(out[base + (4 + r) * 1024 + x]) for x in range(1024)] for r in range(5)]
    rows = []
    held = 0
    for x in range(1024):
        v = [ph[r][x] & ((1 << 63) - 1) for r in range(5)]
        if all(v) and v[4] >= v[0] and v[0] >= t0:
            held += ph[3][x] >> 63
            rows.append([(v[r + 1] - v[r]) / 100.0 for r in range(4)])
    if rows:
        cols = list(zip(*rows))
        desc = " ".join("%s p50/max %.1f/%.1f" % (nm, sorted(c)[len(c) // 2], max(c))
                        for nm, c in zip(("load", "build", "lock", "propagate"), cols))
        print("   first early split per block (%d, parent word held at once %d): %s" %
              (len(rows), held, desc), flush=True)


if __name__ == "__main__":
    main()
