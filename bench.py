#!/usr/bin/env python3
"""Benchmark: batched get on the MI355X-native Sherman B+tree.

Workload (BASELINE.json configs[1], "C2"): 2^26 keys per GPU,
key(i) = CityHash64(i) + 1 (test/benchmark.cpp:43-46 without the modulus),
value(i) = 2i, inserted through the batched insert path in 1 Mi batches;
then uniform 100 % get batches of 1 Mi queries resident in HBM.  A "step" is
one batched get of 1 Mi queries (per GPU).

N > 1 (python -m torch.distributed.run ... bench.py --gpus N): the key space
is range-partitioned one shard per GPU (shard s owns [s*2^64/N, (s+1)*2^64/N)),
each rank holds 2^26 keys of a 2^26*N global key set and issues 1 Mi uniform
queries over the whole set per step; queries and replies are routed with
RCCL all-to-all (weak scaling).

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for every field).
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ALG_BYTES_PER_GET = 1040  # 1024 B leaf + 8 B key + 8 B value
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--keys-log2", type=int, default=26, help="keys per GPU = 2^k")
    p.add_argument("--batch-log2", type=int, default=20, help="queries per step per GPU")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=6.0)
    p.add_argument("--no-sort", action="store_true", help="walk gets in input order")
    p.add_argument("--profile-steps", type=int, default=10)
    return p.parse_args()


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    import numpy as np
    import torch

    import sherman_amd as shm
    from sherman_amd.shard import ShardRouter, owner_of

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE {world}"
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    n_keys = 1 << args.keys_log2          # per GPU
    batch = 1 << args.batch_log2          # queries per GPU per step
    total_keys = n_keys * world
    dev = torch.device(f"cuda:{local}")
    arena = max(2 << 30, n_keys * 48)
    tree = shm.Tree(arena_bytes=arena, max_batch=1 << 20, device=local,
                    node_id=rank, sort_gets=not args.no_sort)

    # ---- build the shard through the batched insert path (untimed) --------
    t0 = time.time()
    chunk = 1 << 22
    inserted = 0
    all_keys = []
    for first in range(1, total_keys + 1, chunk):
        m = min(chunk, total_keys + 1 - first)
        k = torch.empty(m, dtype=torch.int64, device=dev)
        tree.gen_keys(first, m, k)
        ids = torch.arange(first, first + m, dtype=torch.int64, device=dev)
        if world > 1:
            # owner = floor(key * world / 2^64), on unsigned bits
            mine = owner_of(k, world) == rank
            k, ids = k[mine], ids[mine]
        all_keys.append(k)
        for c in range(0, k.numel(), 1 << 20):
            kk = k[c:c + (1 << 20)]
            tree.insert_batch(kk, ids[c:c + (1 << 20)] * 2)
            inserted += kk.numel()
    torch.cuda.synchronize()
    build_s = time.time() - t0
    keys_local = torch.cat(all_keys)
    del all_keys
    st = tree.stats()
    log(f"[rank {rank}] built {inserted} keys in {build_s:.1f}s "
        f"({inserted / build_s / 1e6:.2f} M inserts/s), height {st['height']}, "
        f"pages {st['pages_used']}")

    # ---- query batches (uniform over the global key set), resident in HBM --
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0000 + rank)
    n_batches = 8
    if world == 1:
        qs = [keys_local[torch.randint(0, n_keys, (batch,), device=dev, generator=g)]
              for _ in range(n_batches)]
    else:
        qs = []
        for _ in range(n_batches):
            # uniform i over the GLOBAL key set, key(i) hashed on device with
            # the same CityHash64 as the build; owners are spread uniformly
            ids = torch.randint(1, total_keys + 1, (batch,), device=dev, generator=g)
            qs.append(hash_ids(tree, ids, dev))
    vals = torch.empty(batch, dtype=torch.int64, device=dev)
    found = torch.empty(batch, dtype=torch.uint8, device=dev)

    route = None
    if world > 1:
        route = ShardRouter(tree, world, dist)

    def step(i):
        q = qs[i % n_batches]
        if route is None:
            tree.search_batch(q, vals, found)
        else:
            route.search(q, vals, found)

    for i in range(args.warmup):
        step(i)
    barrier()
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(i)
    barrier()
    elapsed = time.perf_counter() - t_start
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    total_q = batch * args.steps * world
    mops = total_q / elapsed / 1e6

    # correctness on the last batch: every query hits (keys all present)
    torch.cuda.synchronize()
    hit_rate = float(found.float().mean().item())

    # ---- roofline: k_walk timed with HIP events on its launch stream -------
    tree.profile(True)
    for i in range(args.profile_steps):
        step(i)
    torch.cuda.synchronize()
    prof = tree.profile_read(reset=True)
    tree.profile(False)
    walk_ms = prof["walk_ms"] / max(prof["calls"], 1)
    order_ms = prof["order_ms"] / max(prof["calls"], 1)
    q_per_launch = prof["queries"] / max(prof["calls"], 1)
    achieved = q_per_launch * ALG_BYTES_PER_GET / (walk_ms * 1e-3) / 1e9 if walk_ms else 0.0
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_walk.json")
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            if pmc.get("batch") == batch and pmc.get("keys_log2") == args.keys_log2:
                traffic = pmc.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    # ---- CPU baseline (rank 0, N=1 only): reference algorithm on host cores
    cpu = None
    parity = None
    if world == 1 and not args.no_cpu_baseline:
        cpu, parity = cpu_baseline(tree, qs, vals, found, args, step)

    if rank == 0:
        out = {
            "metric": "batched get Mops/s (64M uint64 keys)",
            "value": round(mops, 2),
            "unit": "Mops/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic: key(i)=CityHash64(i)+1, value=2i; uniform queries",
            "config": {
                "workload": "C2: batched get, 2^%d uint64 keys/GPU, uniform 100%% read, "
                            "2^%d-query batches%s" % (args.keys_log2, args.batch_log2,
                                                        "" if world == 1 else
                                                        ", range shards + RCCL all-to-all"),
                "keys_per_gpu": n_keys,
                "batch_per_gpu": batch,
                "tree_height": st["height"],
                "pages": st["pages_used"],
                "sorted_gets": not args.no_sort,
                "build_inserts_per_s": round(inserted / build_s, 1),
                "hit_rate": round(hit_rate, 4),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": "k_walk<false>",
                "alg_bytes_per_get": ALG_BYTES_PER_GET,
                "walk_ms_per_launch": round(walk_ms, 4),
                "order_ms_per_launch": round(order_ms, 4),
                "queries_per_launch": int(q_per_launch),
            },
            "cpu_baseline": cpu,
            "parity_vs_oracle": parity,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    tree.close()


def hash_ids(tree, ids, dev):
    """key(i) = CityHash64(i) + 1 for an arbitrary id tensor (device)."""
    import torch
    # gen_keys hashes a contiguous range; hash ids chunk-wise via a sort-free
    # route: compute on device with torch integer ops (same arithmetic as
    # layout.h cityhash64_u64, 64-bit wrap-around).
    return cityhash64_torch(ids) + 1


def cityhash64_torch(x):
    import torch
    M = (1 << 64) - 1

    def c(v):  # signed int64 constant with the same bits
        v &= M
        return v - (1 << 64) if v >= (1 << 63) else v

    k2 = c(0x9ae16a3b2f90404f)
    mul = c(0x9ae16a3b2f90404f + 16)

    def rot(v, s):
        return ((v >> s) & ((1 << (64 - s)) - 1)) | (v << (64 - s))

    def lsr(v, s):
        return (v >> s) & ((1 << (64 - s)) - 1)

    a = x + k2
    b = x
    cc = rot(b, 37) * mul + a
    d = (rot(a, 25) + b) * mul
    h = (cc ^ d) * mul
    h = h ^ lsr(h, 47)
    g = (d ^ h) * mul
    g = g ^ lsr(g, 47)
    return g * mul


def cpu_baseline(tree, qs, vals, found, args, step):
    """Reference Tree::search restated in C (oracle/, "port"), run on this
    host's cores over the GPU's own page image (identical tree), on a bounded
    sample: repeated 1 Mi-query batches for ~args.cpu_seconds."""
    import numpy as np
    import torch

    from oracle.pyoracle import OracleTree

    img, root = tree.dump_image()
    orc = OracleTree(image=img, root_ptr=root, node_id=tree.node_id)
    ncpu = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = max(1, min(16, ncpu))
    q0 = qs[0].cpu().numpy().view(np.uint64)
    # parity on one full batch: same queries through the GPU path
    step(0)
    torch.cuda.synchronize()
    gv = vals.cpu().numpy().view(np.uint64)
    gf = found.cpu().numpy()
    done = 0
    secs = 0.0
    parity = None
    while secs < args.cpu_seconds or done == 0:
        ov, of, s = orc.search_batch_mt(q0, threads)
        if parity is None:
            parity = bool(np.array_equal(ov, gv) and np.array_equal(of, gf))
        secs += s
        done += q0.size
    orc.close()
    del img
    cpu = {
        "value": round(done / secs / 1e6, 3),
        "unit": "Mops/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{done} uniform gets ({done // q0.size} x 1 Mi batch) over the "
                  f"GPU-built tree image, oracle Tree::search restatement, "
                  f"{threads} pinned threads on {platform.processor() or platform.machine()}",
    }
    return cpu, parity


if __name__ == "__main__":
    main()
