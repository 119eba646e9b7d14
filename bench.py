#!/usr/bin/env python3
"""Benchmark: batched get (and mixed get/insert) on the MI355X-native Sherman
B+tree.

Default workload, C2 (BASELINE.json configs[1]) — the headline line:
  * 2^26 keys per GPU, key(i) = CityHash64(i) + 1 (test/benchmark.cpp:43-46
    without the modulus), value(i) = 2i.
  * The keys go in through the batched insert path in 1 Mi batches (untimed).
  * Then uniform 100 % get batches of 1 Mi queries, resident in HBM.
  * A "step" is one batched get of 1 Mi queries per GPU.

--workload c3 (BASELINE.json configs[2], N = 1):
  * The C2 tree, then batches of 1 Mi ops.
  * Key = to_key(1 + zipf(0.99) over 2^26).
  * An op is a get with probability 50 %, otherwise an insert of value
    (global op index + 1).
  * A step is one batch: its gets see the previous batch's state, then its
    inserts apply in batch order.

--workload c5 (BASELINE.json configs[4], N >= 1):
  * The C2 tree(s), then batches of 1 Mi ops per GPU.
  * Key = to_key(1 + zipf(0.99) over twice the global key set): the ids past
    the preload are new keys, so leaves split (within their shard).
  * 5 % of the ops are range scans [key, key + span] with span =
    --scan-keys * 2^64 / (global keys) (about that many stored keys per
    scan), the other 95 % inserts of value (global op index + 1).
  * A step is one batch: its scans see the previous batch's state, then its
    inserts apply.  N > 1: scans are cut at shard boundaries and routed, and
    inserts routed to their owners, with RCCL all-to-all.

N > 1 (python -m torch.distributed.run ... bench.py --gpus N, C4 / C5):
  * The key space is range-partitioned, one shard per GPU: shard s owns
    [s*2^64/N, (s+1)*2^64/N).
  * C4 (BASELINE.json configs[3]): 2^30 keys in all, 2^30 / N per rank
    (--keys-log2 overrides the per-rank size).
  * Each rank issues 1 Mi uniform queries over the whole set per step.
  * Queries and replies are routed with RCCL all-to-all (sherman_amd.shard),
    i.e. weak scaling in queries per GPU.

Prints ONE JSON line on rank 0 (DESIGN.md §Measurement explains every field).
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ALG_BYTES_PER_GET = 1040     # 1024 B leaf + 8 B key + 8 B value: the page walk
# the summary walk (default): three random reads, each served as a 128 B
# L2 line (directory entry, the 64 B leaf summary, the matching entry) + 8 B
# key + 8 B value
ALG_BYTES_PER_GET_SUM = 3 * 128 + 16
ALG_BYTES_PER_INSERT = 1074  # the reference's per-op leaf read (context only)
# A batched insert chunk's algorithmic bytes, per touched leaf rather than per
# op: the random 128 B lines and whole pages the
# sorted, de-duplicated chunk must touch (Tree.cpp:828-991 restated per leaf)
LINE = 128                   # a random read is served as one 128 B line
ALG_UPSERT = 16 + 2 * LINE + 64   # sorted op in + directory entry + slot line + entry write
ALG_DELETE = 8 + 2 * LINE + 64    # sorted key in + directory entry + slot line + entry write
ALG_STAGED_LEAF = 1024       # a leaf that gets a new key is read whole (free-slot search)
ALG_NEW_PAGE = 1024 + LINE   # a split's new page written + its separator's parent line
ALG_ORDER_PER_OP = 16        # the ordering reads each op (key + value) ...
ALG_ORDER_PER_UNIQUE = 16    # ... and writes each surviving op once
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E peak (MI355X_MICROARCH.md)
N_BATCHES = 8                # distinct resident batches the steps cycle over


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None,
                   help="timed steps (default 1000 for c2: the two-stream pipeline's fill "
                        "and drain are 1 %% of 200 steps; 200 for c3; 20 for c5, whose "
                        "inserts grow the tree)")
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--workload", choices=("c2", "c3", "c5"), default="c2")
    p.add_argument("--keys-log2", type=int, default=None,
                   help="keys per GPU = 2^k (default: 26 at N = 1 (C2), 30 - log2(N) at "
                        "N > 1 (C4: 2^30 keys in all))")
    p.add_argument("--batch-log2", type=int, default=20, help="ops per step per GPU")
    p.add_argument("--theta", type=float, default=0.99, help="c3 zipf skew")
    p.add_argument("--read-ratio", type=int, default=50, help="c3 get percentage")
    p.add_argument("--scan-ratio", type=int, default=5, help="c5 range-scan percentage")
    p.add_argument("--scan-keys", type=int, default=100,
                   help="c5: expected stored keys per range scan")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="CPU baseline sample length (C1: >= 5 two-second windows)")
    p.add_argument("--sort", choices=("auto", "on", "off"), default="auto",
                   help="on: order get batches by key and walk whole pages "
                        "(SHM_FLAG_SORT_GETS, k_get); auto / off: the leaf-summary walk "
                        "(k_get_sum, default)")
    p.add_argument("--scan-out", choices=("slots", "compact"), default="slots",
                   help="c5, N=1: slots = a buffer of --slot-cap values per scan "
                        "(shm_range_query_slots, the reference's per-call buffer, one "
                        "pass); compact = values packed in scan order "
                        "(shm_range_query_batch_async: count, scan, fill)")
    p.add_argument("--pipeline", type=int, default=1, choices=(0, 1),
                   help="c3 / c5 (N=1; c5 with slotted scans on 2 streams): 1 (default "
                        "since round 4, once the ordering stopped waiting on the tree's "
                        "calls: C5 +1.3-3.3 %%, C3 +2.9-3.5 %% over three paired runs) = "
                        "each batch's insert ordering is queued one step ahead on its own "
                        "stream (shm_insert_order), so it runs beside the previous "
                        "batch's gets / scans and tree changes (shm_insert_apply); 0 = "
                        "shm_mixed_batch (c3) / shm_insert_batch_async (c5)")
    p.add_argument("--prio", type=int, default=0, choices=(0, 1),
                   help="c3 / c5 pipelined: 1 = the gets' / scans' and tree changes' "
                        "stream at high priority, the ordering's at normal")
    p.add_argument("--dir-extra-bits", type=int, default=None,
                   help="leaf directory with 2^x entries per tree page (SHM_DIR_EXTRA_BITS)")
    p.add_argument("--order-first", type=int, default=0, choices=(0, 1),
                   help="c5 slotted scans: 1 = the insert ordering is queued "
                        "(shm_insert_order) before the step's scans (pipelined: the next "
                        "batch's), the tree changes (shm_insert_apply) after them")
    p.add_argument("--order-sync", type=int, default=0, choices=(0, 1),
                   help="c5 pipelined: 1 = the step's tree phase waits for the next chunk's "
                        "ordering (an event), so the ordering overlaps the scans only")
    p.add_argument("--order-cus", type=int, default=0,
                   help="c3 / c5 pipelined: the insert ordering's stream is confined to "
                        "this many CUs (hipExtStreamCreateWithCUMask; 0 = all), so the "
                        "ordering of the next chunk leaves the rest to the step's chain")
    p.add_argument("--order-cu-mode", choices=("low", "spread"), default="spread",
                   help="which CUs --order-cus takes: the lowest mask bits, or every "
                        "(total / n)-th bit")
    p.add_argument("--slot-cap", type=int, default=256,
                   help="c5 slotted scans: values per scan buffer (every timed step is "
                        "checked to have no scan past it)")
    p.add_argument("--sync-scans", dest="async_scans", action="store_false",
                   help="c5, N=1: range scans read their total back before the "
                        "batch's inserts are queued (default: async, checked after)")
    p.add_argument("--profile-steps", type=int, default=None,
                   help="steps of the profile pass (default 10; c5: 60, so the "
                        "leaf directory's rebuild, one per ~52 growing chunks, is "
                        "averaged over about as many chunks as it serves)")
    p.add_argument("--latency-steps", type=int, default=None,
                   help="steps of the per-batch latency pass (default: --steps)")
    p.add_argument("--streams", type=int, default=2, choices=(1, 2),
                   help="c2, N=1: consecutive batches alternate over this many HIP "
                        "streams, so one batch's ordering overlaps the previous walk; "
                        "c5, N=1: 2 = scans and inserts on their own streams, so the "
                        "inserts' ordering runs beside the scans (the library still "
                        "orders the inserts' tree changes after the scans)")
    p.add_argument("--sim-world", type=int, default=1,
                   help="N=1 only: build and query shard --sim-rank of a SIM-WORLD-way "
                        "range partition (the per-GPU work of an N-GPU run, no exchange)")
    p.add_argument("--sim-rank", type=int, default=0)
    p.add_argument("--start", choices=("dir", "root", "lds"), default="dir",
                   help="where gets and locates start: the leaf directory (default), the "
                        "root (a descent through the cached upper levels) or an LDS replica "
                        "of the top levels (gets only; A/B for DESIGN §8)")
    p.add_argument("--index-stats", action="store_true",
                   help="c2: an untimed pass over the profile steps counting the walk's "
                        "directory misses, right moves and entry reads (shm_index_stats)")
    p.add_argument("--no-range-hint", action="store_true",
                   help="do not pass the shard key range to the tree (A/B)")
    p.add_argument("--router", choices=("auto", "cabi", "python"), default="auto",
                   help="N > 1: route gets / inserts through the C-ABI shard (C++ over "
                        "RCCL, shm_shard_*) or the Python exchange; auto = the C-ABI on "
                        "the nccl backend once it matched the Python route on one batch")
    p.add_argument("--page-check", type=int, default=0, choices=(0, 1),
                   help="1 = SHM_FLAG_PAGE_CHECK: the get walk also checks the page-level "
                        "version of every page it takes a value from (DESIGN §3.5)")
    p.add_argument("--insert-every", type=int, default=0,
                   help="c2, N=1: one insert chunk of 2^batch-log2 NEW keys (ids past the "
                        "preload, value 2 id, so leaves split) after every K get batches; "
                        "the line then also reports the gets' rate beside the chunks "
                        "against a pure get pass on the same tree (VERDICT r5 #3)")
    a = p.parse_args()
    if a.steps is None:
        # (--insert-every adds 2^20 fresh keys per K steps: 200 steps keep
        # the tree inside its arena)
        a.steps = (20 if a.workload == "c5" else
                   1000 if a.workload == "c2" and not a.insert_every else 200)
    return a


def insert_alg_bytes(ops, uniq, dels, staged, new_pages, ordering):
    """Algorithmic bytes of insert chunks (per touched leaf):
    every unique upsert / delete reads its sorted op, its directory entry and
    the line holding its slot and writes its entry; a leaf that gets a new
    key is read whole; a split writes its new pages and their parents' lines;
    with the ordering inside the window, the ops in and the survivors out."""
    b = uniq * ALG_UPSERT + dels * ALG_DELETE + staged * ALG_STAGED_LEAF + new_pages * ALG_NEW_PAGE
    if ordering:
        b += ops * ALG_ORDER_PER_OP + (uniq + dels) * ALG_ORDER_PER_UNIQUE
    return b


def cap_fracs(d, keys):
    """Refuse a roofline fraction above 1 (it would claim more than the HBM
    peak): the field becomes null and the value moves to d["refused"]."""
    for k in keys:
        v = d.get(k)
        if v is not None and v > 1.0:
            d[k] = None
            d.setdefault("refused", {})[k] = v


class Region:
    """The edges of a profiling window: an empty kernel (shm__mark, tag 1 at
    the start, 2 at the end) whose dispatches tools/fold_roofline.py finds in
    a kernel trace or a counter collection, keeping only the dispatches
    between them.  SHM_BENCH_REGION names the window a profiling run wants
    (tools/roofline_pass.sh): "profile" = the roofline pass whose HIP-event
    times give roofline.achieved, "timed" = the timed steps; unset = no
    markers (the device sees nothing extra)."""

    def __init__(self):
        self.want = os.environ.get("SHM_BENCH_REGION")

    def _mark(self, tag):
        import torch
        import sherman_amd as shm
        torch.cuda.synchronize()
        assert shm._hooks().shm__mark(tag, None) == 0
        torch.cuda.synchronize()

    def begin(self, name):
        if name == self.want:
            self._mark(1)

    def end(self, name):
        if name == self.want:
            self._mark(2)


def cu_masked_stream(n, mode, dev):
    """A torch stream on its own HIP queue restricted to n CUs (the insert
    ordering beside the step's chain, --order-cus)."""
    import ctypes
    import torch
    props = torch.cuda.get_device_properties(dev)
    total = props.multi_processor_count
    n = max(1, min(n, total))
    bits = list(range(n)) if mode == "low" else [int(i * total / n) for i in range(n)]
    words = [0] * ((total + 31) // 32)
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    hip = ctypes.CDLL("libamdhip64.so")
    h = ctypes.c_void_p()
    arr = (ctypes.c_uint32 * len(words))(*words)
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(words)), arr)
    assert rc == 0, f"hipExtStreamCreateWithCUMask failed ({rc})"
    return torch.cuda.ExternalStream(h.value, device=dev)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_name():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def build_shard(tree, n_keys, world, rank, dev):
    """Insert this rank's share of key(1..n_keys*world) (untimed)."""
    import torch
    from sherman_amd.shard import owner_of

    total = n_keys * world
    chunk = 1 << 22
    inserted = 0
    parts = []
    for first in range(1, total + 1, chunk):
        m = min(chunk, total + 1 - first)
        k = torch.empty(m, dtype=torch.int64, device=dev)
        tree.gen_keys(first, m, k)
        ids = torch.arange(first, first + m, dtype=torch.int64, device=dev)
        if world > 1:
            mine = owner_of(k, world) == rank
            k, ids = k[mine], ids[mine]
        parts.append(k)
        for c in range(0, k.numel(), 1 << 20):
            kk = k[c:c + (1 << 20)]
            tree.insert_batch(kk, ids[c:c + (1 << 20)] * 2)
            inserted += kk.numel()
    torch.cuda.synchronize()
    return torch.cat(parts), inserted


def main():
    args = parse()
    if args.profile_steps is None:
        args.profile_steps = 60 if args.workload == "c5" else 10
    if args.dir_extra_bits is not None:
        os.environ["SHM_DIR_EXTRA_BITS"] = str(args.dir_extra_bits)
    import torch

    import sherman_amd as shm
    from sherman_amd.shard import ShardRouter
    from sherman_amd.workload import Zipf, op_is_get

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE {world}"
    assert args.workload != "c3" or world == 1, "c3 is a single-GPU config"
    # one rank per GPU; more ranks than GPUs (a rehearsal of the N > 1 path
    # on a 1-GPU box with SHM_DIST_BACKEND=gloo) share the GPUs round robin
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("SHM_DIST_BACKEND", "nccl")  # nccl == RCCL on ROCm
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    if args.keys_log2 is None:
        # C2 at N = 1; C4 (2^30 keys over N GPUs) and C5 at N > 1
        args.keys_log2 = 26 if world == 1 else 30 - (world.bit_length() - 1)
    n_keys = 1 << args.keys_log2
    batch = 1 << args.batch_log2
    dev = torch.device(f"cuda:{local}")
    assert not args.insert_every or (args.workload == "c2" and world == 1), \
        "--insert-every is a c2, N = 1 option"
    arena = max(2 << 30, n_keys * 48)
    if args.insert_every:
        # room for the chunks of new keys the run inserts (every pass's)
        arena += n_keys * 48 * 2
    from sherman_amd.shard import shard_range
    sim = world == 1 and args.sim_world > 1
    s_rank, s_world = (args.sim_rank, args.sim_world) if sim else (rank, world)
    key_lo, key_bits = (0, 64) if args.no_range_hint else shard_range(s_rank, s_world)
    # N > 1: a rank receives ~batch routed keys (+ a few %), keep one chunk
    tree = shm.Tree(arena_bytes=arena, max_batch=max(1 << 20, batch + (batch >> 2 if world > 1 else 0)), device=local,
                    node_id=rank, sort_gets={"on": True, "off": False}.get(args.sort, "auto"), key_lo=key_lo, key_bits=key_bits,
                    leaf_dir=args.start == "dir", top_lds=args.start == "lds",
                    page_check=bool(args.page_check))

    c1 = None
    if world == 1 and args.workload == "c2" and not args.no_cpu_baseline and not args.insert_every:
        # the reference benchmark's tree, one insert at a time on a host
        # thread while the GPU work runs (cpu_baseline_c1)
        c1 = C1Build()
    t0 = time.time()
    keys_local, inserted = build_shard(tree, n_keys, s_world, s_rank, dev)
    n_keys = inserted if sim else n_keys
    build_s = time.time() - t0
    st = tree.stats()
    cshard, router_kind = None, None
    if world > 1:
        cshard, router_kind = make_cshard(tree, world, rank, dist, dev, args, keys_local)
    log(f"[rank {rank}] built {inserted} keys in {build_s:.1f}s "
        f"({inserted / build_s / 1e6:.2f} M inserts/s), height {st['height']}, "
        f"pages {st['pages_used']}")

    # ---- resident op batches ----------------------------------------------
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0000 + rank)
    vals = torch.empty(batch, dtype=torch.int64, device=dev)
    found = torch.empty(batch, dtype=torch.uint8, device=dev)
    ins = None  # c2 --insert-every: the chunks of new keys (FreshChunks)
    if args.workload == "c2":
        if world == 1:
            # qi: the ids' positions (keys_local[j] = key(j + 1), value 2 (j + 1))
            qi = [torch.randint(0, n_keys, (batch,), device=dev, generator=g)
                  for _ in range(N_BATCHES)]
            qs = [keys_local[i] for i in qi]
        else:
            qs = []
            for _ in range(N_BATCHES):
                # uniform i over the GLOBAL key set, hashed on device
                ids = torch.randint(1, n_keys * world + 1, (batch,), device=dev, generator=g)
                k = torch.empty_like(ids)
                tree.hash_keys(ids, k)
                qs.append(k)
        # independent batches alternate over two streams (each with its own
        # result buffers; N > 1: its own router buffers and RCCL communicator,
        # so one batch's exchange and ordering overlap the previous walk); the
        # library orders the streams' calls on the device
        nstr = args.streams
        streams = [torch.cuda.Stream() for _ in range(nstr)] if nstr > 1 else [None]
        outs = [(vals, found)] + [(torch.empty_like(vals), torch.empty_like(found))
                                  for _ in range(nstr - 1)]
        routes = [None] * nstr
        if world > 1:
            groups = [None] + [dist.new_group(list(range(world))) for _ in range(nstr - 1)]
            routes = [ShardRouter(tree, world, dist, group=gr, cshard=cshard) for gr in groups]
        for sx in streams:
            if sx is not None:
                sx.wait_stream(torch.cuda.current_stream())

        pend = {}
        seq = [0]  # routed batches issued so far (all step loops)

        def on(i):
            sx = streams[i % nstr]
            return torch.cuda.stream(sx if sx is not None else torch.cuda.current_stream())

        ins = FreshChunks(tree, n_keys, batch, dev) if args.insert_every else None

        def step(i):
            if routes[0] is None:
                v, f = outs[i % nstr]
                tree.search_batch(qs[i % N_BATCHES], v, f, stream=streams[i % nstr])
                if ins is not None and (i + 1) % args.insert_every == 0:
                    # a chunk of new keys, queued without a host wait; the
                    # library orders it after both streams' searches
                    ins.insert(stream=streams[i % nstr])
                return
            c = seq[0]
            seq[0] += 1
            v, f = outs[c % nstr]
            if nstr == 1:
                with on(c):
                    routes[0].search(qs[c % N_BATCHES], v, f)
                return
            # N > 1, two streams: batch c + 1's bucketing and count exchange
            # are issued before batch c's exchange and walk
            # (ShardRouter.search_begin); each router serves every other batch
            if c not in pend:
                with on(c):
                    pend[c] = routes[c % nstr].search_begin(qs[c % N_BATCHES])
            with on(c + 1):
                pend[c + 1] = routes[(c + 1) % nstr].search_begin(qs[(c + 1) % N_BATCHES])
            with on(c):
                routes[c % nstr].search_end(pend.pop(c), v, f)

        def done_streams(i):
            # where step i's batch completes (N > 1: every stream, the latest)
            if routes[0] is None:
                return [streams[i % nstr] or torch.cuda.current_stream()]
            return [sx or torch.cuda.current_stream() for sx in streams]
    elif args.workload == "c5":
        from sherman_amd import PendingRange
        from sherman_amd.shard import umin
        assert not sim, "--sim-world is a C2 option"
        n_glob = n_keys * world
        span = (1 << 64) // n_glob * args.scan_keys
        zipf = Zipf(2 * n_glob, args.theta, dev)  # ids > n_glob: new keys
        # a fresh batch for every step the run applies (CPU-baseline parity
        # pair, warmup, timed, latency and profile steps): a batch applied a
        # second time would find its new keys already stored and turn their
        # inserts into updates, leaving the timed steps with few splits
        n_c5 = 2 + args.warmup + args.steps + args.profile_steps + 2 * (
            args.latency_steps if args.latency_steps is not None else args.steps)
        mixed = []
        for b in range(n_c5):
            ids = zipf.sample(batch, g) + 1
            k = torch.empty_like(ids)
            tree.hash_keys(ids, k)
            is_scan = op_is_get(batch, args.scan_ratio, dev, g)
            op_idx = torch.arange(b * batch, (b + 1) * batch, dtype=torch.int64, device=dev)
            op_idx += (rank * n_c5) * batch
            lo = k[is_scan].contiguous()
            hi = lo + span  # wraps past 2^64 - 1 ...
            hi = torch.where((hi ^ (-(1 << 63))) < (lo ^ (-(1 << 63))),
                             torch.full_like(lo, -1), hi)  # ... so saturate
            mixed.append((lo, umin(hi, torch.full_like(lo, -2)), k[~is_scan].contiguous(),
                          (op_idx[~is_scan] + 1).contiguous()))
        del keys_local
        route = ShardRouter(tree, world, dist, cshard=cshard) if world > 1 else None
        # routed scans: every rank passes the same piece-matrix width, the
        # largest scan count of any rank's batches (shm_shard_range_query)
        n_cap = max(m[0].numel() for m in mixed)
        if dist is not None:
            nc = torch.tensor([n_cap], dtype=torch.int64, device=dev)
            dist.all_reduce(nc, op=dist.ReduceOp.MAX)
            n_cap = int(nc.item())
        scan_out = {}
        applied = [0]  # batches applied so far (all step loops)
        s_scan = s_ins = None
        if route is None and args.streams == 2:
            # --prio 1: the stream that carries the step's chain (scans and
            # tree changes when pipelined) at high priority, so the ordering
            # beside it takes the CUs it leaves
            s_scan = torch.cuda.Stream(priority=-1 if args.prio else 0)
            s_ins = (cu_masked_stream(args.order_cus, args.order_cu_mode, dev) if args.order_cus
                     else torch.cuda.Stream())
            s_scan.wait_stream(torch.cuda.current_stream())
            s_ins.wait_stream(torch.cuda.current_stream())

        slots = route is None and args.async_scans and args.scan_out == "slots"
        if slots:
            # two per-scan buffers, alternating (a step's scans never overwrite
            # the previous step's results); ordered on the scans' stream
            sbuf = [(torch.empty((n_cap, args.slot_cap), dtype=torch.int64, device=dev),
                     torch.empty(n_cap, dtype=torch.int64, device=dev)) for _ in range(2)]
            # {scans past the slot, error bits} of every step, accumulated on
            # the device (zeroed here, checked after the timed steps)
            slot_status = torch.zeros(2, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()

        rq_caps = []  # routed async scans: (vals_cap, peer_cap)
        pipe = slots and args.pipeline and s_ins is not None
        ticket = [None]  # the ordered, not yet applied batch (pipeline)
        if pipe:
            # scans and tree changes on one stream (s_scan), the orderings on
            # their own (s_ins): batch i + 1 is ordered while batch i applies
            s_main, s_ord = s_scan or torch.cuda.current_stream(), s_ins

        def step(i):
            lo, hi, pk, pv = mixed[applied[0] % n_c5]
            applied[0] += 1
            if pipe:
                if ticket[0] is None:  # the first batch of the run
                    ticket[0] = tree.insert_order(pk, pv, stream=s_ord)
                _, _, nk, nv = mixed[applied[0] % n_c5]  # the next step's batch
                nxt = None
                if args.order_first:
                    # the next batch's ordering queued before this step's scans,
                    # so it starts with them instead of a host call later
                    nxt = tree.insert_order(nk, nv, stream=s_ord)
                sv, sc = sbuf[applied[0] % 2]
                pr = tree.range_query_slots(lo, hi, args.slot_cap, stream=s_main, vals=sv,
                                            counts=sc, status=slot_status)
                scan_out["r"] = SlotsResult(pr)
                scan_out["slots"] = slot_status
                if nxt is None:
                    nxt = tree.insert_order(nk, nv, stream=s_ord)
                if args.order_sync:
                    # the tree phase waits for the next chunk's ordering, so the
                    # ordering runs beside the scans only, not beside the chain
                    ev = torch.cuda.Event()
                    ev.record(s_ord)
                    s_main.wait_event(ev)
                tree.insert_apply(ticket[0], stream=s_main)
                ticket[0] = nxt
            elif slots:
                # one pass: each scan's values into its own buffer; every
                # step's (scans past the slot, error bits) is checked after the run
                tk = None
                if args.order_first:
                    # the batch's ordering queued before its scans (it reads
                    # only the batch), its tree changes after them
                    tk = tree.insert_order(pk, pv, stream=s_ins)
                sv, sc = sbuf[applied[0] % 2]
                pr = tree.range_query_slots(lo, hi, args.slot_cap, stream=s_scan, vals=sv,
                                            counts=sc, status=slot_status)
                scan_out["r"] = SlotsResult(pr)
                scan_out["slots"] = slot_status
                if tk is None:
                    tree.insert_batch_async(pk, pv, stream=s_ins)
                else:
                    tree.insert_apply(tk, stream=s_ins)
            elif route is None and args.async_scans:
                # scans queued without a host wait; the batch's inserts queue
                # behind them (their ordering beside them, on their own
                # stream); every step's total is checked after the run
                scan_out["r"] = pr = tree.range_query_batch_async(lo, hi, stream=s_scan)
                if pr.tot is not None:  # only the (total, error) words stay alive
                    scan_out.setdefault("all", []).append((pr.tot, pr.vals.numel()))
                tree.insert_batch_async(pk, pv, stream=s_ins)
            elif route is None:
                scan_out["r"] = PendingRange(None, *tree.range_query_batch(lo, hi))
                tree.insert_batch_async(pk, pv)
            elif cshard is not None and rq_caps:
                # routed scans with no host read-back: fixed runs per peer
                # sized from the first (synchronous) batch; every step's
                # status is checked after the run
                c, _, v, st = cshard.range_query_async(lo, hi, rq_caps[0], rq_caps[1], n_cap)
                scan_out["r"] = PendingRange(None, c, v)
                scan_out.setdefault("rstat", []).append(st)
                route.insert(pk, pv)
            else:
                c, v = route.range_query(lo, hi, n_cap)
                scan_out["r"] = PendingRange(None, c, v)
                if cshard is not None:
                    t_ = int(v.numel())
                    rq_caps[:] = [t_ + t_ // 2 + (1 << 16), (t_ * 5) // (4 * world) + (1 << 13)]
                route.insert(pk, pv)

        def done_streams(i):
            # the library orders the inserts after the scans: the insert stream
            # (pipeline: the scans' stream, which applies) completes the step
            if pipe:
                return [s_main]
            return [s_ins if (route is None and args.async_scans and s_ins is not None)
                    else torch.cuda.current_stream()]
    else:
        zipf = Zipf(n_keys, args.theta, dev)
        mixed, c3_ids = [], []
        for b in range(N_BATCHES):
            ids = zipf.sample(batch, g) + 1  # key(1 + zipf_next())
            k = torch.empty_like(ids)
            tree.hash_keys(ids, k)
            is_get = op_is_get(batch, args.read_ratio, dev, g)
            op_idx = torch.arange(b * batch, (b + 1) * batch, dtype=torch.int64, device=dev)
            mixed.append((k[is_get].contiguous(), k[~is_get].contiguous(),
                          (op_idx[~is_get] + 1).contiguous()))
            if b < 2:  # the gets' ids: their preload value is 2 id (parity)
                c3_ids.append(ids[is_get].contiguous())
        del keys_local

        c3_pipe = args.pipeline and world == 1
        c3n = [0]  # batches issued so far (all step loops; the pipeline's order)
        c3_ticket = [None]
        if c3_pipe:
            # gets and tree changes on one stream, the orderings on their own:
            # batch i + 1 is ordered while batch i's gets and inserts run
            c3_main = torch.cuda.Stream(priority=-1 if args.prio else 0)
            c3_ord = (cu_masked_stream(args.order_cus, args.order_cu_mode, dev) if args.order_cus
                      else torch.cuda.Stream())
            c3_main.wait_stream(torch.cuda.current_stream())
            c3_ord.wait_stream(torch.cuda.current_stream())

        def step(i):
            # one mixed batch: the gets see the state before its inserts;
            # queued without a host wait (the status of every insert is
            # checked after the timed steps)
            if not c3_pipe:  # shm_mixed_batch
                gk, pk, pv = mixed[i % N_BATCHES]
                tree.mixed_batch(gk, vals[:gk.numel()], found[:gk.numel()], pk, pv)
                return
            gk, pk, pv = mixed[c3n[0] % N_BATCHES]
            c3n[0] += 1
            if c3_ticket[0] is None:
                c3_ticket[0] = tree.insert_order(pk, pv, stream=c3_ord)
            tree.search_batch(gk, vals[:gk.numel()], found[:gk.numel()], stream=c3_main)
            _, nk, nv = mixed[c3n[0] % N_BATCHES]
            nxt = tree.insert_order(nk, nv, stream=c3_ord)
            tree.insert_apply(c3_ticket[0], stream=c3_main)
            c3_ticket[0] = nxt

        def done_streams(i):
            return [c3_main if c3_pipe else torch.cuda.current_stream()]

    # ---- CPU baseline (rank 0, N = 1): oracle on host cores, same tree -----
    cpu = parity = fresh_ms = None
    if world == 1 and not args.no_cpu_baseline:
        if args.workload == "c2":
            # the form the timed steps walk: the read phase's pair-form
            # directory (built after four searches without an insert,
            # tree.cpp kReadPhase) -- with --insert-every, the form the
            # chunks keep current
            rewarm(tree, dev, seconds=0.0)
            parity = parity_get(qs[0], qi[0], vals, found, step, tree, keys_local, n_keys, g)
            if ins is not None:
                fresh_ms = pure_get_ms(tree, qs, outs, 64)  # before any chunk of new keys
        elif args.workload == "c5":
            cpu, parity = cpu_baseline_c5(tree, mixed, scan_out, args, step, n_keys)
        else:
            cpu, parity = cpu_baseline_mixed(tree, mixed, c3_ids, vals, found, args, step)

    # ---- timed steps --------------------------------------------------------
    if cpu is not None or parity is not None:
        # the CPU baseline left the GPU idle for ~10 s; the first tens of
        # steps after such a pause ran up to 5x slower (measured: C5 563
        # against 3059 Mops/s with a 1 s baseline), so re-warm the device
        # with read-only gets over stored keys before the warmup steps
        rewarm(tree, dev)
    elif args.workload == "c2":
        # a read-only stream's steady state is the library's read phase (its
        # directory rebuilt once, after four searches without an insert):
        # reached here, untimed, whatever --warmup is
        rewarm(tree, dev, seconds=0.0)
    for i in range(args.warmup):
        step(i)
    region = Region()
    barrier()
    splits0 = tree.stats()["splits"]
    region.begin("timed")
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(i)
    host_issue = time.perf_counter() - t_start  # host time to issue the steps
    if cshard is not None:
        # inside the timed region: a routed insert's overflow tails (applied
        # by the next call on the shard) are part of the step's work
        cshard.synchronize()
    barrier()
    elapsed = time.perf_counter() - t_start
    region.end("timed")
    tree.synchronize()  # raises any error of the queued batches
    rank_mops = batch * args.steps / elapsed / 1e6
    cluster_sum = rank_mops
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        # per-rank rates summed over the cluster, as the reference's per-window
        # cluster sum (test/benchmark.cpp:320-337 via DSMKeeper::sum,
        # src/DSMKeeper.cpp:163-176)
        cs = torch.tensor([rank_mops], dtype=torch.float64, device=dev)
        dist.all_reduce(cs, op=dist.ReduceOp.SUM)
        cluster_sum = float(cs.item())
    st_end = tree.stats()
    total_ops = batch * args.steps * world
    if ins is not None:
        total_ops += batch * (args.steps // args.insert_every)  # the chunks' inserts
    if parity is not None and args.workload == "c2" and world == 1:
        # the timed steps' own results: the last batch of each stream holds
        # exactly what the walk wrote in the timed region
        checked = 0
        for i in range(max(0, args.steps - len(outs)), args.steps):
            v, f = outs[i % len(outs)]
            want = (qi[i % N_BATCHES] + 1) * 2
            parity["ok"] = parity["ok"] and bool(torch.equal(v, want)) and bool(f.all())
            checked += 1
        parity["timed_batches_checked"] = checked
        if ins is not None:
            parity["ok"] = parity["ok"] and ins.check_last()
            parity["inserted_chunk_checked"] = True
        log(f"C2 parity incl. the last {checked} timed batches: {parity['ok']}")
    mops = total_ops / elapsed / 1e6
    torch.cuda.synchronize()
    if args.workload == "c2":
        last = (args.steps - 1) if world == 1 else seq[0] - 1  # last routed batch ended
        hit_rate = float(outs[last % len(outs)][1].float().mean().item())
    elif args.workload == "c5":
        for tot, cap in scan_out.pop("all", []):
            total, err = (int(x) for x in tot.cpu().tolist())
            # every timed step's values fit its buffer, with no device error
            assert err == 0 and total <= cap, (total, cap, err)
        if "slots" in scan_out:
            ovf, err = (int(x) for x in scan_out["slots"].cpu().tolist())
            # no scan of any step so far passed its slot, no device error
            assert err == 0 and ovf == 0, (ovf, err)
        for st in scan_out.pop("rstat", []):
            tot_, flags = (int(x) for x in st.cpu().tolist())
            # every routed async batch complete: no run past its peer cap
            assert flags == 0, (tot_, flags)
        c, _ = scan_out["r"].result()
        hit_rate = float(c.float().mean().item())  # mean values per scan
    else:
        last_b = (c3n[0] - 1) if c3_pipe else (args.steps - 1)  # the last step's batch
        n_get = mixed[last_b % N_BATCHES][0].numel()
        hit_rate = float(found[:n_get].float().mean().item())

    # ---- per-batch latency (untimed pass): HIP events around each step on
    # its stream, in the order the reference reports them
    # (test/benchmark.cpp:207-249: p50 / p90 / p95 / p99 / p99.9) ------------
    if args.workload == "c2" and world > 1:
        # the pipeline keeps a batch begun: a separate Python router, or the C
        # shard (two slots: one holds the begun batch)
        lat_route = ShardRouter(tree, world, dist, cshard=cshard)

        def one(i):  # one routed batch, not pipelined with the next
            lat_route.search(qs[i % N_BATCHES], outs[0][0], outs[0][1])
    elif args.workload == "c2":
        def one(i):
            tree.search_batch(qs[i % N_BATCHES], vals, found)
    else:
        one = step
    lat = latency_pass(one, args, dist)
    # per-op latency under load: the timed steps' pipelining, 100 ns buckets
    # (test/benchmark.cpp:207-249)
    depth = (len(outs) if args.workload == "c2" else
             2 if args.workload == "c5" and world == 1 and args.streams == 2 else 1)
    op_lat = op_latency_pass(step, done_streams, batch, depth, args, dist)
    if dist is not None:
        lt = torch.tensor(lat, dtype=torch.float64, device=dev)
        dist.all_reduce(lt, op=dist.ReduceOp.MAX)
        lat = lt.tolist()

    # ---- roofline: the walk timed with HIP events on its launch stream.  C2
    # runs these batches one at a time on one stream, so each launch's
    # duration is the kernel's own (the timed steps overlap two walks) -----
    tree.profile(True)
    tree.profile_read(reset=True)
    prof_splits0 = tree.stats()["splits"]
    region.begin("profile")
    for i in range(args.profile_steps):
        (one if args.workload == "c2" else step)(i)
    torch.cuda.synchronize()
    region.end("profile")
    prof = tree.profile_read(reset=True)
    tree.profile(False)
    # pages the profiled chunks' splits made (early and in k_upper)
    prof_new_pages = tree.stats()["splits"] - prof_splits0
    idx = None
    if args.workload in ("c2", "c3") and args.sort != "on" and (args.profile_steps > 0 or
                                                                args.index_stats):
        # the walk's index statistics over one more batch: how many gets the
        # directory's fingerprints answered (two lines instead of three: the
        # algorithmic bytes per get below)
        tree.profile(False, index_stats=True)
        for i in range(max(args.profile_steps, 1) if args.index_stats else 1):
            if args.workload == "c2":
                one(i)
            else:
                gk = mixed[i % N_BATCHES][0]
                tree.search_batch(gk, vals[:gk.numel()], found[:gk.numel()])
        torch.cuda.synchronize()
        idx = tree.index_stats()
        tree.profile(False)
        g_ = max(idx["gets"], 1)
        idx.update({k + "_per_get": round(idx[k] / g_, 4)
                    for k in ("start_internal", "right_moves", "page_hops", "entry_reads",
                              "dir_fp_hits")})
    brk = (insert_every_breakdown(tree, qs, outs, ins, args.insert_every, fresh_ms=fresh_ms)
           if ins is not None else None)
    dirst = tree.dir_stats() if args.start == "dir" else None
    if c1 is not None:
        # C1 on the host cores, after every GPU measurement (the oracle's
        # build has run beside them)
        cpu = c1.bench(args.cpu_seconds)
    walk_ev_ms = prof["walk_ms"] / max(prof["calls"], 1)  # HIP events of the dispatch
    # the headline duration is the HIP events' (VERDICT / ADVICE r5: the
    # device clock span below -- first block start to last wave's stores
    # issued -- leaves out the dispatch ramp and the store drain, and
    # undercut the rocprof kernel trace by 3-4 %).  Round 6: the events ride
    # on the walk's own dispatch (hipExtLaunchKernel), so they time the
    # kernel as the trace does; event records around the launch added
    # 2-3 us of marker packets (4.7 % over the trace, profiles/r06 first pass)
    walk_clk_ms = prof["walk_kernel_ms"] / max(prof["calls"], 1) if prof["walk_kernel_ms"] > 0 else None
    walk_ms = walk_ev_ms
    ins_ms = prof["insert_ms"] / max(prof["insert_calls"], 1)
    ups_ms = prof["upsert_ms"] / max(prof["insert_calls"], 1)
    ins_per_launch = prof["insert_ops"] / max(prof["insert_calls"], 1)
    range_ms = prof["range_ms"] / max(prof["range_calls"], 1)
    order_ms = prof["order_ms"] / max(prof["calls"], 1)
    q_per_launch = prof["queries"] / max(prof["calls"], 1)
    page_walk = args.sort == "on"  # SHM_FLAG_SORT_GETS: ordered, whole pages (k_get)
    bpg = ALG_BYTES_PER_GET if page_walk else ALG_BYTES_PER_GET_SUM
    fp_frac = None
    if not page_walk and idx is not None and idx["gets"]:
        # a get answered from the directory's fingerprints needs two random
        # lines (directory entry, entry), any other three (+ summary line)
        fp_frac = idx["dir_fp_hits"] / idx["gets"]
        bpg = round(ALG_BYTES_PER_GET_SUM - 128 * fp_frac, 1)
    achieved = q_per_launch * bpg / (walk_ms * 1e-3) / 1e9 if walk_ms else 0.0
    traffic = None
    if args.workload == "c2" and args.start == "dir":
        traffic = _profile_traffic("pmc_walk.json", "hbm_bytes_per_launch", batch,
                                   args.keys_log2, "k_get<" if page_walk else "k_get_sum")

    if rank == 0:
        if args.workload == "c2":
            metric = "batched get Mops/s (64M uint64 keys)"
            workload = ("C2: batched get, 2^%d uint64 keys/GPU, uniform 100%% read, "
                        "2^%d-query batches%s" % (args.keys_log2, args.batch_log2,
                                                    "" if world == 1 else
                                                    ", range shards + RCCL all-to-all"))
            if sim:
                workload += ", shard %d of %d (no exchange)" % (s_rank, s_world)
            data = "synthetic: key(i)=CityHash64(i)+1, value=2i; uniform queries"
            if ins is not None:
                metric = "batched get + insert Mops/s (64M uint64 keys, a chunk of new keys " \
                         "every %d get batches)" % args.insert_every
                workload += (", + one 2^%d-key insert chunk of new keys (ids past the preload, "
                             "value 2 id) after every %d get batches" % (args.batch_log2,
                                                                        args.insert_every))
        else:
            metric = "mixed get/insert Mops/s (64M uint64 keys, zipf %.2f, %d%% get)" % (
                args.theta, args.read_ratio)
            workload = ("C3: 2^%d uint64 keys, 2^%d-op batches, key=to_key(1+zipf(%.2f)), "
                        "%d%% get / %d%% insert (value = op index + 1)" % (
                            args.keys_log2, args.batch_log2, args.theta, args.read_ratio,
                            100 - args.read_ratio))
            data = "synthetic: key(i)=CityHash64(i)+1 preload, zipf op stream"
        if args.workload == "c5":
            metric = ("write-heavy insert + range-scan Mops/s (zipf %.2f, %d%% insert, "
                      "%d%% scan)" % (args.theta, 100 - args.scan_ratio, args.scan_ratio))
            workload = ("C5: 2^%d uint64 keys/GPU, 2^%d-op batches/GPU, key=to_key(1+zipf(%.2f) "
                        "over 2x the global key set), %d%% inserts (value = op index + 1), %d%% "
                        "range scans of ~%d keys%s" % (
                            args.keys_log2, args.batch_log2, args.theta, 100 - args.scan_ratio,
                            args.scan_ratio, args.scan_keys,
                            "" if world == 1 else ", range shards + RCCL all-to-all"))
        out = {
            "metric": metric,
            "value": round(mops, 2),
            "unit": "Mops/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "host_issue_ms_per_step": round(host_issue / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": data,
            "config": {
                "workload": workload,
                "keys_per_gpu": n_keys,
                "batch_per_gpu": batch,
                "tree_height": st["height"],
                "pages": st["pages_used"],
                "get_order": args.sort,
                "streams": (len(outs) if args.workload == "c2" else
                            args.streams if args.workload == "c5" and world == 1 else 1),
                "rccl_groups": (len(outs) if args.workload == "c2" and world > 1 else None),
                "router": router_kind,
                "start": args.start,
                "build_inserts_per_s": round(inserted / build_s, 1),
                "hit_rate": round(hit_rate, 4),
                "splits_in_timed_steps": st_end["splits"] - splits0,
                "pages_after": st_end["pages_used"],
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                # PMC bytes come from a separate rocprofv3 --pmc pass (a run of
                # its own, tools/roofline_pass.sh), committed under profiles/:
                # not measured in this run
                "traffic_source": ("committed: profiles/pmc_walk.json (a separate PMC pass at "
                                   "this config), not this run" if traffic else None),
                "kernel": "k_get<4,1,4>" if page_walk else "k_get_sum",
                "alg_bytes_per_get": bpg,
                # the reference's per-get bytes (a whole 1 KB leaf)
                # over the same walk time: what reading the page would need
                "reference_bytes_per_get": ALG_BYTES_PER_GET,
                "reference_bytes_GBps": round(q_per_launch * ALG_BYTES_PER_GET /
                                              (walk_ms * 1e-3) / 1e9, 1) if walk_ms else None,
                "walk_ms_per_launch": round(walk_ms, 4),
                "walk_ms_basis": "HIP events carried by each walk dispatch on its stream (hipExtLaunchKernel start / stop events, profile pass)",
                "walk_clock_ms_per_launch": round(walk_clk_ms, 4) if walk_clk_ms else None,
                "order_ms_per_launch": round(order_ms, 4),
                "queries_per_launch": int(q_per_launch),
                # measured HBM bytes (PMC, profiles/pmc_walk.json) per get and
                # as a rate over the walk; the reference's root-to-leaf path
                # reads 5 x 1024 B + 16 B per get, for context
                "traffic_per_get": (round(traffic / q_per_launch, 1)
                                    if traffic and q_per_launch else None),
                "traffic_GBps": (round(traffic / (walk_ms * 1e-3) / 1e9, 1)
                                 if traffic and walk_ms else None),
                # the timed steps: two walks in flight, one batch per step
                "step_alg_GBps": round(q_per_launch * bpg / (elapsed / args.steps) / 1e9, 1)
                                 if args.workload == "c2" else None,
                "full_path_bytes_per_get": 5136,
            },
            "cpu_baseline": cpu,
            "parity_vs_oracle": parity,
            "batch_latency_us": dict(zip(("p50", "p90", "p95", "p99", "p99.9", "max"),
                                         [round(x, 1) for x in lat])),
            "op_latency_us": op_lat,
            "cluster_sum_mops": round(cluster_sum, 2),
        }
        if idx is not None:
            out["index_stats"] = idx
        if dirst is not None:
            # the leaf directory the walk starts from: its form, device
            # memory and rebuild cost (shm_dir_stats)
            out["directory"] = {"form": dirst["form"], "entries": dirst["entries"],
                                "bytes": dirst["bytes"], "builds": dirst["builds"],
                                "last_build_ms": round(dirst["last_build_ms"], 4),
                                "total_build_ms": round(dirst["total_build_ms"], 4),
                                "maintained_by_inserts": bool(dirst["maintained"]),
                                "exact": bool(dirst["exact"])}
            out["dir_bytes"] = dirst["bytes"]  # the same two, at the top level
            out["dir_build_ms"] = round(dirst["last_build_ms"], 4)
        if brk is not None:
            out["insert_every"] = brk
        if args.workload == "c2":
            step_s = elapsed / args.steps
            rf = out["roofline"]
            if page_walk:
                note = "SURVEY §8d (1 KB leaf + key + value)"
            elif fp_frac is not None:
                note = ("the summary walk's random 128 B lines, two (directory entry, entry) "
                        "for the gets the directory's fingerprints answered (dir_fp_frac of "
                        "them) and three (+ leaf summary) for the rest, + 8 B key + 8 B value: "
                        "DESIGN §3's redefinition of SURVEY §8d's 1040 B whole-leaf read")
            else:
                note = ("the summary walk's three random 128 B lines (directory entry, leaf "
                        "summary, entry) + 8 B key + 8 B value, DESIGN §3's redefinition of "
                        "SURVEY §8d's 1040 B whole-leaf read")
            rf["alg_bytes_note"] = "%s B/get: %s" % (bpg, note)
            rf["dir_fp_frac"] = round(fp_frac, 4) if fp_frac is not None else None
            rf["reference_bytes_frac"] = (round(rf["reference_bytes_GBps"] / HBM_PEAK_GBS, 4)
                                          if rf["reference_bytes_GBps"] else None)
            # the timed steps themselves (two walks in flight on two streams):
            # algorithmic bytes of one batch over one step
            rf["step_frac"] = round(q_per_launch * bpg / step_s / 1e9 / HBM_PEAK_GBS, 4) \
                if q_per_launch else None
            # request roofline: the walk is bound by random 128 B requests,
            # not bytes: measured TCC read requests per get (PMC)
            # x gets/s of the timed steps / the measured random-request ceiling
            req = _request_roofline(batch, args.keys_log2, mops * 1e6 / world, page_walk)
            if req:
                rf.update(req)
        if args.workload in ("c3", "c5"):
            # the insert chunks of the profile pass, counted on the device
            ic = max(prof["insert_calls"], 1)
            per = {"ops": prof["insert_ops"] / ic, "uniq": prof["insert_unique"] / ic,
                   "dels": prof["insert_dels"] / ic, "staged": prof["insert_staged"] / ic,
                   "new_pages": prof_new_pages / ic}
            pipelined = (args.pipeline and world == 1 and
                         (args.workload == "c3" or bool(args.async_scans and
                                                        args.scan_out == "slots" and
                                                        args.streams == 2)))
            # the profiled window: the tree phase alone when pipelined (the
            # ordering ran a step earlier on its own stream), else the chunk
            alg_win = insert_alg_bytes(per["ops"], per["uniq"], per["dels"], per["staged"],
                                       per["new_pages"], ordering=not pipelined)
            alg_chunk = insert_alg_bytes(per["ops"], per["uniq"], per["dels"], per["staged"],
                                         per["new_pages"], ordering=True)
            pmc = _step_traffic(args.workload, batch, args.keys_log2)
            ins = {
                "insert_ms_per_launch": round(ins_ms, 4),
                "upsert_ms_per_launch": round(ups_ms, 4),
                "window": ("insert_apply chunk (locate + segmentation + upsert + k_upper; the "
                           "ordering runs one chunk ahead on its own stream)" if pipelined else
                           "insert chunk (ordering + locate + segmentation + upsert + k_upper)"),
                "per_chunk": {k: round(v, 1) for k, v in per.items()},
                "alg_bytes_per_chunk": round(alg_win),
                "alg_model": "DESIGN §5: %d B per unique upsert, %d B per delete, %d B per leaf "
                             "read whole, %d B per new page%s" % (
                                 ALG_UPSERT, ALG_DELETE, ALG_STAGED_LEAF, ALG_NEW_PAGE,
                                 "" if pipelined else ", + 16 B per op in and per survivor out"),
                "alg_GBps": round(alg_win / (ins_ms * 1e-3) / 1e9, 1) if ins_ms else None,
                "reference_bytes_per_insert": ALG_BYTES_PER_INSERT,
            }
            ins["alg_frac"] = round(ins["alg_GBps"] / HBM_PEAK_GBS, 4) if ins["alg_GBps"] else None
            if pmc is not None:
                tb = pmc["apply_bytes_per_chunk"] + (0 if pipelined else pmc["order_bytes_per_chunk"])
                ins.update({"traffic": tb,
                            "traffic_GBps": round(tb / (ins_ms * 1e-3) / 1e9, 1) if ins_ms else None,
                            "traffic_source": pmc["source"]})
                ins["traffic_frac"] = (round(ins["traffic_GBps"] / HBM_PEAK_GBS, 4)
                                       if ins["traffic_GBps"] else None)
            cap_fracs(ins, ("alg_frac", "traffic_frac"))
        if args.workload == "c5":
            out["config"]["hit_rate"] = None
            out["config"]["values_per_scan"] = round(hit_rate, 2)
            out["config"]["insert_pipeline"] = bool(pipelined)
            out["config"]["scan_out"] = (("slots of %d values" % args.slot_cap)
                                         if world == 1 and args.async_scans and
                                         args.scan_out == "slots" else "compact")
            rf = out["roofline"]
            for k in ("walk_ms_per_launch", "walk_ms_basis", "walk_clock_ms_per_launch",
                      "order_ms_per_launch", "queries_per_launch",
                      "alg_bytes_per_get", "reference_bytes_per_get", "reference_bytes_GBps",
                      "traffic_per_get", "step_alg_GBps", "full_path_bytes_per_get"):
                rf.pop(k, None)
            rf.update(ins)
            # the headline is the real traffic of the chunk's kernels (PMC) over
            # its measured time, the per-leaf model beside it
            real = ins.get("traffic_GBps") is not None
            rf["kernel"] = ins["window"]
            rf["achieved"] = ins["traffic_GBps"] if real else ins["alg_GBps"]
            rf["achieved_basis"] = ("PMC FETCH_SIZE x2 + WRITE_SIZE of the window's kernels"
                                    if real else "algorithmic (per touched leaf)")
            rf["frac"] = ins["traffic_frac"] if real else ins["alg_frac"]
            rf["traffic"] = ins.get("traffic")
            rf["range_ms_per_launch"] = round(range_ms, 4)
            rf["inserts_per_launch"] = int(ins_per_launch)
            # the whole step: the chunk's algorithmic bytes (ordering included)
            # over the step time
            rf["step_alg_GBps"] = round(alg_chunk / (elapsed / args.steps) / 1e9, 1)
            rf["step_frac"] = round(rf["step_alg_GBps"] / HBM_PEAK_GBS, 4)
        if args.workload == "c3":
            # the whole step: its gets as walked + its insert chunk (ordering
            # included), over the step time; and the step's PMC bytes
            step_s = elapsed / args.steps
            b0 = mixed[0]
            alg = b0[0].numel() * bpg + alg_chunk
            out["config"]["insert_pipeline"] = bool(args.pipeline and world == 1)
            rf = out["roofline"]
            rf["insert"] = ins
            rf["walk_frac"] = rf["frac"]  # the get walk alone (k_get_sum), as C2
            rf["step_alg_GBps"] = round(alg / step_s / 1e9, 1)
            rf["step_frac"] = round(alg / step_s / 1e9 / HBM_PEAK_GBS, 4)
            if pmc is not None and pmc.get("step_bytes"):
                rf["step_traffic"] = pmc["step_bytes"]
                rf["step_traffic_GBps"] = round(pmc["step_bytes"] / step_s / 1e9, 1)
                rf["step_traffic_frac"] = round(rf["step_traffic_GBps"] / HBM_PEAK_GBS, 4)
                # the headline: the step's real traffic
                rf["frac"] = rf["step_traffic_frac"]
                rf["achieved"] = rf["step_traffic_GBps"]
                rf["achieved_basis"] = ("PMC bytes of one step's kernels (gets, ordering, "
                                        "tree phase) over the timed step")
                rf["kernel"] = "C3 step (k_get_sum + insert chunk)"
        cap_fracs(out["roofline"], ("frac", "step_frac", "walk_frac", "step_traffic_frac",
                                    "reference_bytes_frac", "request_frac", "alg_frac",
                                    "traffic_frac"))
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    tree.close()


def rewarm(tree, dev, seconds=0.5):
    """Read-only device work (batched gets of random keys; no tree state
    changes) for about `seconds` of wall clock."""
    import torch
    q = torch.randint(1, 1 << 62, (1 << 20,), device=dev, dtype=torch.int64)
    v = torch.empty_like(q)
    f = torch.empty(q.numel(), dtype=torch.uint8, device=dev)
    t0 = time.perf_counter()
    while True:  # at least one round of 16
        for _ in range(16):
            tree.search_batch(q, v, f)
        torch.cuda.synchronize()
        if time.perf_counter() - t0 >= seconds:
            break


def _profile_traffic(name, field, batch, keys_log2, kernel=None):
    """HBM bytes per launch measured by the committed PMC passes
    (profiles/<name>, tools/roofline_pass.sh + tools/commit_roofline.py) when they were taken at this
    batch and key count (and of this kernel), else None."""
    try:
        pmc = json.load(open(os.path.join(ROOT, "profiles", name)))
    except (OSError, ValueError):
        return None
    if kernel and kernel not in pmc.get("kernel", ""):
        return None
    if pmc.get("batch") == batch and pmc.get("keys_log2") == keys_log2:
        return pmc.get(field)
    return None


def _step_traffic(workload, batch, keys_log2):
    """The C3 / C5 PMC bytes measured over the bench's own profile window
    (profiles/pmc_steps.json, tools/roofline_pass.sh -> tools/fold_roofline.py)
    when taken at this batch and key count: {apply_bytes_per_chunk,
    order_bytes_per_chunk, step_bytes, source} or None."""
    try:
        pmc = json.load(open(os.path.join(ROOT, "profiles", "pmc_steps.json")))[workload]
    except (OSError, ValueError, KeyError):
        return None
    if pmc.get("batch") == batch and pmc.get("keys_log2") == keys_log2:
        return pmc
    return None


def _request_roofline(batch, keys_log2, gets_per_s, page_walk):
    """requests/get from the committed PMC pass (profiles/pmc_walk.json,
    TCC_EA0_RDREQ per launch, tools/fold_c2.py) when it was taken at this
    batch and key count, the random-request ceiling from
    profiles/cal_fetch.json: {request_frac, ...} or {}."""
    if page_walk:
        return {}
    try:
        pmc = json.load(open(os.path.join(ROOT, "profiles", "pmc_walk.json")))
        cal = json.load(open(os.path.join(ROOT, "profiles", "cal_fetch.json")))
    except (OSError, ValueError):
        return {}
    if not (pmc.get("batch") == batch and pmc.get("keys_log2") == keys_log2 and
            pmc.get("tcc_ea_rdreq_per_launch") and "k_get_sum" in pmc.get("kernel", "")):
        return {}
    rpg = pmc["tcc_ea_rdreq_per_launch"] / batch
    ceil = cal["random_request_ceiling_G_per_s"]  # the best calibration kernel's rate
    rate = rpg * gets_per_s / 1e9
    return {"requests_per_get": round(rpg, 3), "requests_G_per_s": round(rate, 2),
            "request_ceiling_G_per_s": ceil, "request_frac": round(rate / ceil, 4),
            "request_source": "committed: profiles/pmc_walk.json (TCC_EA0_RDREQ, a separate PMC "
                              "pass at this config) and profiles/cal_fetch.json, not this run"}


def make_cshard(tree, world, rank, dist, dev, args, keys_local):
    """The C-ABI shard (sherman_amd.CShard: routed get / insert in C++ over
    its own RCCL communicators) when the backend is nccl and --router allows;
    with "auto" it must first return the Python route's results on one batch
    of stored keys on every rank, else the run fails."""
    import torch
    import sherman_amd as shm
    from sherman_amd.shard import ShardRouter
    if args.router == "python" or dist.get_backend() != "nccl":
        return None, "python"
    cs = shm.CShard(tree, world, rank, dist)
    if args.router == "cabi":
        return cs, "cabi"
    g = torch.Generator(device=dev)
    g.manual_seed(0xC0FFEE + rank)
    q = keys_local[torch.randint(0, keys_local.numel(), (1 << 16,), device=dev, generator=g)]
    q = torch.cat([q, q + 1])  # hits and (mostly) misses
    va, fa = torch.empty_like(q), torch.empty(q.numel(), dtype=torch.uint8, device=dev)
    vb, fb = torch.empty_like(q), torch.empty(q.numel(), dtype=torch.uint8, device=dev)
    ShardRouter(tree, world, dist).search(q, va, fa)
    cs.search(q, vb, fb)
    torch.cuda.synchronize()
    ok = torch.tensor([int(torch.equal(va, vb) and torch.equal(fa, fb))], device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 1:
        return cs, "cabi"
    # a routing bug must fail the run, not hide behind the slower Python path
    cs.close()
    raise RuntimeError("C-ABI shard route (shm_shard_search) disagreed with the Python "
                       "route on a self-check batch of stored keys and misses")


def latency_pass(one, args, dist):
    """Latency of single batches: each of the pass's batches is issued alone
    (barrier and device idle before, synchronize after) and timed on the
    host clock, issue included; returns [p50, p90, p95, p99, p99.9, max] in
    us (max over ranks at N > 1), the percentiles the reference prints
    (test/benchmark.cpp:207-249, there per op)."""
    import numpy as np
    import torch
    n = args.latency_steps if args.latency_steps is not None else args.steps
    if n <= 0:
        return [0.0] * 6
    us = []
    for i in range(n):
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        one(i)
        torch.cuda.synchronize()
        us.append((time.perf_counter() - t0) * 1e6)
    us = np.array(us)
    return [float(np.percentile(us, q)) for q in (50, 90, 95, 99, 99.9)] + [float(us.max())]


class SlotsResult:
    """A slotted scan batch read in the compact form (counts, values in scan
    order), as the parity legs compare it."""

    def __init__(self, pend):
        self.pend = pend

    def result(self):
        return self.pend.packed()


LATENCY_BUCKET_US = 0.1  # test/benchmark.cpp: latency[thread][i], i = 100 ns windows


def op_latency_pass(step, done_streams, batch, depth, args, dist):
    """Per-op latency histogram under the timed condition (test/benchmark.cpp:
    207-249 records each op's latency in 100 ns windows and prints p50 / p90 /
    p95 / p99 / p99.9 from the cumulative counts).  The steps run pipelined
    as in the timed region, closed-loop with `depth` batches in flight (a
    batch is issued once the batch `depth` before it has completed, as each
    of the reference's client threads issues its next op after the last
    one returns; an open loop would only measure the queue the host
    builds); an op's latency is its batch's completion (a HIP
    event on the stream that finishes the step, on the device clock) minus
    the host time its step was issued (both relative to one idle-device
    origin).  Every op of a batch shares it, so each batch adds `batch` ops
    to its window.  Max over ranks at N > 1 (per percentile)."""
    import numpy as np
    import torch
    n = args.latency_steps if args.latency_steps is not None else args.steps
    if n <= 0:
        return None
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    e0.synchronize()
    t0 = time.perf_counter()
    issue, done = [], []
    for i in range(n):
        if i >= depth:
            # closed loop, as the reference's client threads: at most `depth`
            # batches in flight (the timed steps' streams), the next one
            # issued once the oldest completes
            for e in done[i - depth]:
                e.synchronize()
        issue.append((time.perf_counter() - t0) * 1e6)
        step(i)
        evs = []
        for sx in done_streams(i):
            e = torch.cuda.Event(enable_timing=True)
            e.record(sx)
            evs.append(e)
        done.append(evs)
    torch.cuda.synchronize()
    lat = np.array([max(e0.elapsed_time(e) for e in evs) * 1e3 - t for evs, t in zip(done, issue)])
    lat = np.maximum(lat, 0.0)
    win = np.floor(lat / LATENCY_BUCKET_US).astype(np.int64)
    hist = np.bincount(win) * batch  # ops per 100 ns window
    cum = np.cumsum(hist)
    tot = int(cum[-1])
    pct = []
    for num, den in ((1, 2), (9, 10), (95, 100), (99, 100), (999, 1000)):
        th = tot * num // den
        pct.append(float(np.searchsorted(cum, th) * LATENCY_BUCKET_US))
    pct.append(float(win.max() * LATENCY_BUCKET_US))
    if dist is not None:
        lt = torch.tensor(pct, dtype=torch.float64, device="cuda")
        dist.all_reduce(lt, op=dist.ReduceOp.MAX)
        pct = lt.tolist()
    out = dict(zip(("p50", "p90", "p95", "p99", "p99.9", "max"), [round(x, 1) for x in pct]))
    out.update({"bucket_us": LATENCY_BUCKET_US, "ops": tot, "in_flight": depth,
                "condition": "the timed steps' pipelining, closed loop with in_flight batches "
                             "queued; op latency = batch completion (device event) - step issue "
                             "(host)"})
    return out


def _oracle_on_gpu_image(tree, spare_bytes=0):
    from oracle.pyoracle import OracleTree
    img, root = tree.dump_image()
    orc = OracleTree(image=img, root_ptr=root, node_id=tree.node_id, spare_bytes=spare_bytes)
    del img
    return orc


def _cgroup_cpus():
    """CPUs granted by the cgroup v2 quota (cpu.max "quota period"), or None
    when unlimited / not readable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q == "max":
            return None
        return max(1, -(-int(q) // int(p)))
    except (OSError, ValueError):
        return None


def _threads():
    """T = the CPUs this process may actually run on, one pinned thread each
    (test/benchmark.cpp:96 bindCore; SURVEY §8d: T = nproc): the affinity
    mask, capped by the cgroup CPU quota.  On the GPU box the mask lists all
    256 host CPUs but cpu.max grants 16; 256 threads there are throttled to
    16 CPUs' worth of time and the C1 leg measures 15 Mops/s against 44 at
    T = 16 (profiles/r02_cpu_threads.txt)."""
    ncpu = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    q = _cgroup_cpus()
    return max(1, min(ncpu, q) if q else ncpu)


C1_KEYSPACE = 64 << 20     # kKeySpace (test/benchmark.cpp:21)
C1_WARM = 0.8              # kWarmRatio (test/benchmark.cpp:22)
C1_PRELOAD = 1024000       # test/benchmark.cpp:269-274


class C1Build:
    """The reference benchmark's tree at C1 (kKeySpace = 2^26 WITH the
    modulus), built the way test/benchmark.cpp builds it: one Tree::insert at
    a time (the oracle's restatement, 27/27 leaf splits), node 0's preload
    to_key(i) -> 2i for i = 1..1,024,000 (benchmark.cpp:269-274), then the
    warm-up to_key(i) -> 2i for i in [1, 0.8 kKeySpace) in order
    (benchmark.cpp:114-120).  ~55 M single inserts take about a minute on one
    core, so the build runs on a host thread (ctypes releases the GIL) while
    the GPU tree is built and measured; bench() joins it and times the read
    phase."""

    def __init__(self):
        import threading
        from oracle.pyoracle import OracleTree
        self.orc = OracleTree(2 << 30)
        self.t0 = time.time()
        self.build_s = None
        self.th = threading.Thread(target=self._run, daemon=True)
        self.th.start()

    def _run(self):
        self.orc.c1_build(C1_KEYSPACE, C1_WARM, C1_PRELOAD)
        self.build_s = time.time() - self.t0

    def bench(self, seconds):
        """C1 (BASELINE.json configs[0]): the reference benchmark's measured
        phase, kNodeCount = 1, kReadRatio = 100, zipf theta = 0 over
        kKeySpace, restated in C (oracle/ orc_c1_bench: pinned threads, key =
        to_key(zipf_next()), Tree::search, per-thread op counters sampled
        every 2 s), on every CPU the process may use; the steady-state mean
        over >= 5 two-second windows (test/benchmark.cpp:165-188, 302-341)."""
        import numpy as np
        self.th.join()
        threads = _threads()
        windows = max(5, int(round(seconds / 2.0)))
        w = self.orc.c1_bench(threads, C1_KEYSPACE, theta=0.0, windows=windows, window_s=2.0)
        rc, shape = self.orc.check()
        self.orc.close()
        return {
            "value": round(float(np.mean(w[1:])), 3),
            "unit": "Mops/s",
            "cores": threads,
            "kind": "port",
            "sample": f"C1: reference test/benchmark read phase restated in C (oracle/), "
                      f"kKeySpace 2^26 with the modulus; tree built one Tree::insert at a time "
                      f"in the reference's order (preload 1,024,000 + warm 0.8, {self.build_s:.0f} s): "
                      f"{shape['keys']} keys, {shape['leaves']} leaves "
                      f"({shape['keys'] / max(shape['leaves'], 1):.1f} keys/leaf = "
                      f"{100 * shape['keys'] / max(shape['leaves'], 1) / 54:.1f} % of 54), "
                      f"height {shape['height']}, check {rc}; uniform to_key(zipf(theta=0)) "
                      f"searches, {threads} pinned threads on {cpu_name()}, {windows} x 2 s "
                      f"windows (first dropped): " + ", ".join("%.2f" % x for x in w),
        }


def parity_get(q, qi, vals, found, step, tree, keys_local, n_keys, g, miss_frac=0.09):
    """One full C2 batch through the GPU path (step 0) against the values the
    build wrote: query j is key(qi[j] + 1), stored with value 2 (qi[j] + 1),
    so every get must be found with exactly that value (what Tree::search
    returns over the same key stream; the expectation is the key stream's,
    not the tree's own image).  The batch runs on the directory form the
    timed steps walk (the caller reached the read phase first) and its
    index statistics say how many gets that form answered (dir_fp_hits).
    Then the same batch with ~9 % of its queries replaced by keys that were
    never stored -- key(i) for ids past the key count, as the reference
    benchmark's C1 read phase misses ~9 % of its gets (kKeySpace with the
    modulus, test/benchmark.cpp:43-46) -- each of which must come back not
    found with value 0 (Tree.cpp:445-448), the rest as above.  Returns
    {"ok", "dir_form", "dir_fp_hits_per_get", ...}; main() adds the timed
    steps' own last batches."""
    import torch
    form = tree.dir_stats()["form"]
    tree.profile(False, index_stats=True)
    step(0)
    torch.cuda.synchronize()
    idx = tree.index_stats()
    tree.profile(False)
    want = (qi + 1) * 2
    ok = bool(torch.equal(vals, want) and bool(found.all()))
    n = q.numel()
    miss = torch.rand(n, device=q.device, generator=g) < miss_frac
    m = int(miss.sum().item())
    mk = torch.empty(m, dtype=torch.int64, device=q.device)
    tree.gen_keys(n_keys + 1, m, mk)  # ids n_keys + 1 .. : never stored
    # the expectation is the key stream's: none of these keys equals a stored
    # one (CityHash64 collisions would show here)
    ok = ok and not bool(torch.isin(mk, keys_local).any())
    q2 = q.clone()
    q2[miss] = mk
    v2 = torch.empty_like(q2)
    f2 = torch.empty(n, dtype=torch.uint8, device=q.device)
    tree.search_batch(q2, v2, f2)
    tree.synchronize()
    want2 = torch.where(miss, torch.zeros_like(want), want)
    ok = ok and bool(torch.equal(v2, want2)) and bool(torch.equal(f2.bool(), ~miss))
    fp = idx["dir_fp_hits"] / max(idx["gets"], 1)
    log(f"C2 parity on the {form} directory: {n} hits ({fp:.6f} answered from the entry) + a "
        f"batch with {m} misses ({m / n:.3f}): {ok}")
    return {"ok": ok, "dir_form": form, "dir_fp_hits": idx["dir_fp_hits"], "gets": idx["gets"],
            "dir_fp_hits_per_get": round(fp, 6), "hit_batch": n, "miss_batch_misses": m,
            "expected": "value 2 id for key(id), the key stream's (test/benchmark.cpp:43-46)"}


class FreshChunks:
    """c2 --insert-every: chunks of keys never stored before, key(i) for ids
    i past the preload in order, value 2 i (as the build), generated on the
    device ahead of the passes that insert them (none inside a timed
    region).  insert() queues the next chunk (shm_insert_batch_async);
    check_last() searches the last chunk inserted: every key found with its
    value."""

    def __init__(self, tree, n_keys, batch, dev, ahead=64):
        self.tree, self.batch, self.dev = tree, batch, dev
        self.next_id = n_keys + 1
        self.ready = []
        self.last = None
        self.inserted = 0
        self.fill(ahead)

    def fill(self, n):
        import torch
        while len(self.ready) < n:
            k = torch.empty(self.batch, dtype=torch.int64, device=self.dev)
            self.tree.gen_keys(self.next_id, self.batch, k)
            v = torch.arange(self.next_id, self.next_id + self.batch, dtype=torch.int64,
                             device=self.dev) * 2
            self.ready.append((k, v))
            self.next_id += self.batch
        torch.cuda.synchronize()

    def insert(self, stream=None):
        if not self.ready:
            self.fill(8)  # (only past the pre-generated chunks)
        k, v = self.ready.pop(0)
        self.tree.insert_batch_async(k, v, stream=stream)
        self.last = (k, v)
        self.inserted += 1

    def check_last(self):
        import torch
        if self.last is None:
            return True
        k, v = self.last
        out = torch.empty_like(k)
        f = torch.empty(k.numel(), dtype=torch.uint8, device=k.device)
        self.tree.search_batch(k, out, f)
        self.tree.synchronize()
        ok = bool(torch.equal(out, v)) and bool(f.all())
        log(f"inserted chunk parity ({k.numel()} new keys): {ok}")
        return ok


def pure_get_ms(tree, qs, outs, batches):
    """ms per get batch of `batches` batches on one stream (HIP events
    around the run): the pure-get reference of --insert-every."""
    import torch
    v, f = outs[0]
    torch.cuda.synchronize()
    pe = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    pe[0].record()
    for j in range(batches):
        tree.search_batch(qs[j % N_BATCHES], v, f)
    pe[1].record()
    torch.cuda.synchronize()
    return pe[0].elapsed_time(pe[1]) / batches


def insert_every_breakdown(tree, qs, outs, ins, every, cycles=8, fresh_ms=None):
    """c2 --insert-every: the gets' rate beside the chunks, one stream, HIP
    events around each cycle's chunk and its `every` get batches (a
    directory rebuild a search calls for runs inside its batch's interval),
    then `cycles` x `every` pure get batches on the same tree the same way.
    Untimed passes after the timed steps."""
    import torch
    v, f = outs[0]
    ins.fill(cycles)
    st0 = tree.dir_stats()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3 * cycles)]
    for c in range(cycles):
        ev[3 * c].record()
        ins.insert()
        ev[3 * c + 1].record()
        for j in range(every):
            tree.search_batch(qs[(c * every + j) % N_BATCHES], v, f)
        ev[3 * c + 2].record()
    torch.cuda.synchronize()
    ins_ms = sum(ev[3 * c].elapsed_time(ev[3 * c + 1]) for c in range(cycles))
    get_ms = sum(ev[3 * c + 1].elapsed_time(ev[3 * c + 2]) for c in range(cycles))
    st1 = tree.dir_stats()
    pure_ms = pure_get_ms(tree, qs, outs, cycles * every) * cycles * every
    gets = cycles * every * qs[0].numel()
    mix = gets / (get_ms * 1e-3) / 1e6
    pure = gets / (pure_ms * 1e-3) / 1e6
    out = {"every": every, "cycles": cycles,
            "get_mops_beside_inserts": round(mix, 1), "get_mops_pure": round(pure, 1),
            "ratio": round(mix / pure, 4),
            "insert_ms_per_chunk": round(ins_ms / cycles, 4),
            "get_ms_per_batch_beside_inserts": round(get_ms / (cycles * every), 4),
            "get_ms_per_batch_pure": round(pure_ms / (cycles * every), 4),
            "dir_builds_in_cycles": st1["builds"] - st0["builds"],
            "dir_form": st1["form"],
            "condition": "one stream; HIP events around each chunk and around its get batches "
                         "(directory rebuilds the searches call for included); pure = the same "
                         "number of get batches after the cycles, same tree; pure_fresh = the "
                         "same measure on the C2 tree before any chunk (the pure C2 rate)"}
    if fresh_ms:
        fresh = qs[0].numel() / (fresh_ms * 1e-3) / 1e6
        out["get_mops_pure_fresh"] = round(fresh, 1)
        out["ratio_vs_fresh"] = round(mix / fresh, 4)
    return out


def c5_model(tree, n_keys, dev):
    """The C5 key -> value contents as sorted host arrays, built from the key
    stream (key(i) -> 2i, i = 1..n_keys), not from the tree: the parity
    model for the C5 scans."""
    import numpy as np
    import torch
    k = torch.empty(n_keys, dtype=torch.int64, device=dev)
    tree.gen_keys(1, n_keys, k)
    sk, order = torch.sort(k ^ (-(1 << 63)))  # u64 order as int64
    keys = (sk ^ (-(1 << 63))).cpu().numpy().view(np.uint64)
    vals = ((order + 1) * 2).cpu().numpy().view(np.uint64)
    del k, sk, order
    return keys, vals


def c5_model_scans(keys, vals, lo, hi):
    """Per scan [lo, hi] the model's values (counts, concatenated values)."""
    import numpy as np
    left = np.searchsorted(keys, lo, "left")
    right = np.maximum(np.searchsorted(keys, hi, "right"), left)
    counts = (right - left).astype(np.int64)
    total = int(counts.sum())
    start = np.repeat(left - (np.cumsum(counts) - counts), counts)
    return counts, vals[np.arange(total) + start]


def c5_model_apply(keys, vals, pk, pv):
    """The model after one insert batch (last writer in batch order)."""
    import numpy as np
    assert not (pv == 0).any()  # C5 values are op index + 1: no deletes
    u, ix = np.unique(pk[::-1], return_index=True)
    uv = pv[::-1][ix]
    pos = np.searchsorted(keys, u)
    hit = (pos < keys.size) & (keys[np.minimum(pos, keys.size - 1)] == u)
    vals[pos[hit]] = uv[hit]
    new = ~hit
    return np.insert(keys, pos[new], u[new]), np.insert(vals, pos[new], uv[new])


def same_multisets(counts, a, b):
    """a and b hold the same values per segment (segments of `counts`)."""
    import numpy as np
    if a.size != b.size:
        return False
    sid = np.repeat(np.arange(counts.size), counts)
    return bool(np.array_equal(a[np.lexsort((a, sid))], b[np.lexsort((b, sid))]))


def cpu_baseline_c5(tree, mixed, scan_out, args, step, n_keys):
    """C5 batches on the oracle over the GPU's image (the CPU timing leg):
    the batch's range scans (restated Tree::range_query) then its inserts
    (restated Tree::insert), on every CPU of the affinity mask (inserts
    partitioned by page lock word, orc_apply_batch_mt), for
    ~args.cpu_seconds.  Parity: the first two batches' scans return, per
    scan, the values of a model of the contents built from the key stream
    and the batches themselves (c5_model: preload, then batch 0's inserts),
    as multisets (slots inside a leaf are unsorted)."""
    import numpy as np
    import torch

    orc = _oracle_on_gpu_image(tree, spare_bytes=2 << 30)  # C5 inserts new keys
    threads = _threads()
    gpu = []
    done, secs, b = 0, 0.0, 0
    while secs < args.cpu_seconds or b < 2:
        lo, hi, pk, pv = mixed[b % len(mixed)]
        if b < 2:
            step(b)  # applies mixed[b]: the first two batches of the run
            torch.cuda.synchronize()
            gc, gv = scan_out["r"].result()
            gpu.append((gc.cpu().numpy(), gv.cpu().numpy().view(np.uint64)))
        loh = lo.cpu().numpy().view(np.uint64)
        hih = hi.cpu().numpy().view(np.uint64)
        pkh = pk.cpu().numpy().view(np.uint64)
        pvh = pv.cpu().numpy().view(np.uint64)
        _, _, s1 = orc.range_query_batch_mt(loh, hih, threads)
        s2 = orc.apply_batch_mt(pkh, pvh, threads)
        secs += s1 + s2
        done += loh.size + pkh.size
        b += 1
    orc.close()
    keys, vals = c5_model(tree, n_keys, torch.device(f"cuda:{tree.device}"))
    parity = True
    for bb in range(2):
        lo, hi, pk, pv = (x.cpu().numpy().view(np.uint64) for x in mixed[bb])
        mc, mv = c5_model_scans(keys, vals, lo, hi)
        gc, gv = gpu[bb]
        parity = parity and bool(np.array_equal(mc, gc.astype(np.int64))) and \
            same_multisets(mc, mv, gv)
        keys, vals = c5_model_apply(keys, vals, pk, pv)
    del keys, vals
    cpu = {
        "value": round(done / secs / 1e6, 3),
        "unit": "Mops/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{b} C5 1 Mi-op batches ({done} ops) over the GPU-built tree image: "
                  f"range scans then inserts, oracle Tree::range_query / Tree::insert "
                  f"restatement, {threads} pinned threads (inserts partitioned by page "
                  f"lock word) on {cpu_name()}",
    }
    return cpu, parity


def cpu_baseline_mixed(tree, mixed, c3_ids, vals, found, args, step):
    """Mixed batches on the oracle over the GPU's image (the CPU timing leg):
    gets on `threads` pinned threads, then the batch's inserts on the same
    threads partitioned by page lock word (orc_apply_batch_mt), for
    ~args.cpu_seconds.  Parity: the first two batches' gets return what the
    stream wrote — batch 0 the preload value 2 id, batch 1 batch 0's last
    write to the key or else 2 id (every get finds its key: the zipf draws
    stored ids)."""
    import numpy as np
    import torch

    orc = _oracle_on_gpu_image(tree)
    threads = _threads()
    parity = True
    last = None  # batch 0's last writer per key (sorted keys, values)
    done, secs, b = 0, 0.0, 0
    while secs < args.cpu_seconds or b < 2:
        gk, pk, pv = mixed[b % N_BATCHES]
        gkh = gk.cpu().numpy().view(np.uint64)
        pkh = pk.cpu().numpy().view(np.uint64)
        pvh = pv.cpu().numpy().view(np.uint64)
        if b < 2:
            step(b)
            torch.cuda.synchronize()
            gv = vals[:gk.numel()].cpu().numpy().view(np.uint64)
            gf = found[:gk.numel()].cpu().numpy()
            want = (c3_ids[b].cpu().numpy() * 2).astype(np.uint64)
            if last is not None:
                u, uv = last
                pos = np.minimum(np.searchsorted(u, gkh), u.size - 1)
                hit = u[pos] == gkh
                want[hit] = uv[pos[hit]]
            parity = parity and bool(np.array_equal(gv, want) and gf.all())
            u, ix = np.unique(pkh[::-1], return_index=True)
            last = (u, pvh[::-1][ix])
        ov, of, s = orc.search_batch_mt(gkh, threads)
        s += orc.apply_batch_mt(pkh, pvh, threads)
        secs += s
        done += gkh.size + pkh.size
        b += 1
    orc.close()
    cpu = {
        "value": round(done / secs / 1e6, 3),
        "unit": "Mops/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{b} mixed 1 Mi-op batches ({done} ops) over the GPU-built tree "
                  f"image on {threads} pinned threads: gets, then inserts partitioned by "
                  f"page lock word (oracle Tree::search / Tree::insert restatement) on "
                  f"{cpu_name()}",
    }
    return cpu, parity


if __name__ == "__main__":
    main()
