"""Host-side cost of one routed C2 step at world 1 over RCCL: the
ShardRouter sequence bench.py runs at N > 1 (bucket, count / key / value
exchanges, local search, un-permute), timed with and without waiting for
the device, next to the plain search_batch.  Diagnostic for whether the
N > 1 path is host-bound.  usage: python tools/host_route.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

import sherman_amd as shm
from sherman_amd.shard import ShardRouter

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
n_keys, batch = 1 << 24, 1 << 20
t = shm.Tree(arena_bytes=1 << 30, max_batch=batch + batch // 4)
k = torch.empty(n_keys, dtype=torch.int64, device="cuda")
t.gen_keys(1, n_keys, k)
for c in range(0, n_keys, batch):
    t.insert_batch(k[c:c + batch], k[c:c + batch])
q = k[torch.randint(0, n_keys, (batch,), device="cuda")]
v = torch.empty_like(q)
f = torch.empty(batch, dtype=torch.uint8, device="cuda")
r = ShardRouter(t, 1, dist)
for name, fn in (("search_batch", lambda: t.search_batch(q, v, f)),
                 ("router.search", lambda: r.search(q, v, f))):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        fn()
    issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    print(f"{name}: host issue {issue / 50 * 1e6:.1f} us/step, wall {total / 50 * 1e6:.1f} us/step",
          flush=True)
# two streams, two communicators, alternating (what bench.py does at N > 1)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
routers = [r, ShardRouter(t, 1, dist, group=dist.new_group([0]))]
outs = [(v, f), (torch.empty_like(v), torch.empty_like(f))]
for sx in streams:
    sx.wait_stream(torch.cuda.current_stream())


def step2(i):
    with torch.cuda.stream(streams[i & 1]):
        routers[i & 1].search(q, *outs[i & 1])


for i in range(6):
    step2(i)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(50):
    step2(i)
issue = time.perf_counter() - t0
torch.cuda.synchronize()
total = time.perf_counter() - t0
print(f"router.search, 2 streams: host issue {issue / 50 * 1e6:.1f} us/step, "
      f"wall {total / 50 * 1e6:.1f} us/step", flush=True)

# pipelined: batch i + 1 begun before batch i ends (bench.py at N > 1)
pend = {0: None}


def step3(i):
    if pend.get(i) is None:
        with torch.cuda.stream(streams[i & 1]):
            pend[i] = routers[i & 1].search_begin(q)
    with torch.cuda.stream(streams[(i + 1) & 1]):
        pend[i + 1] = routers[(i + 1) & 1].search_begin(q)
    with torch.cuda.stream(streams[i & 1]):
        routers[i & 1].search_end(pend.pop(i), *outs[i & 1])


for i in range(6):
    step3(i)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(6, 56):
    step3(i)
issue = time.perf_counter() - t0
torch.cuda.synchronize()
total = time.perf_counter() - t0
print(f"router pipelined, 2 streams: host issue {issue / 50 * 1e6:.1f} us/step, "
      f"wall {total / 50 * 1e6:.1f} us/step", flush=True)
pend.clear()

# the C-ABI shard (shm_shard_*, C++ over RCCL): plain and pipelined
cs = shm.CShard(t, 1, 0, dist)
rc_ = ShardRouter(t, 1, dist, cshard=cs)
for name, fn in (("cabi search", lambda: rc_.search(q, v, f)),):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        fn()
    issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    print(f"{name}: host issue {issue / 50 * 1e6:.1f} us/step, wall {total / 50 * 1e6:.1f} us/step",
          flush=True)
pc = {}


def step4(i):
    if pc.get(i) is None:
        with torch.cuda.stream(streams[i & 1]):
            pc[i] = rc_.search_begin(q)
    with torch.cuda.stream(streams[(i + 1) & 1]):
        pc[i + 1] = rc_.search_begin(q)
    with torch.cuda.stream(streams[i & 1]):
        rc_.search_end(pc.pop(i), *outs[i & 1])


for i in range(6):
    step4(i)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(6, 56):
    step4(i)
issue = time.perf_counter() - t0
torch.cuda.synchronize()
total = time.perf_counter() - t0
print(f"cabi pipelined, 2 streams: host issue {issue / 50 * 1e6:.1f} us/step, "
      f"wall {total / 50 * 1e6:.1f} us/step", flush=True)
pc.clear()
torch.cuda.synchronize()
cs.close()

# per-piece host cost of router.search (no device waits except tolist)
import collections
acc = collections.defaultdict(float)
n = q.numel()
for it in range(60):
    T = time.perf_counter
    a = T(); kb = r._buf("kb", n, torch.int64, q.device); perm = r._buf("perm", n, torch.int32, q.device)
    cnt = r._buf("cnt", 1, torch.int64, q.device); b = T(); acc["bufs"] += b - a
    t.route_bucket(q, 1, kb, perm, cnt); c = T(); acc["route_bucket"] += c - b
    rc = r._buf("rcnt", 1, torch.int64, q.device); r._a2a(rc, cnt); d = T(); acc["a2a counts"] += d - c
    cl, rl = cnt.tolist(), rc.tolist(); e = T(); acc["tolist (sync)"] += e - d
    recv = r._buf("recv", rl[0], torch.int64, q.device); r._a2a(recv, kb, rl, cl); f2 = T(); acc["a2a keys"] += f2 - e
    rv = r._buf("rv", rl[0], torch.int64, q.device); rf = r._buf("rf", rl[0], torch.uint8, q.device)
    t.search_batch(recv, rv, rf); g = T(); acc["search_batch"] += g - f2
    back = r._buf("back", n, torch.int64, q.device); r._a2a(back, rv, cl, rl); h = T(); acc["a2a values"] += h - g
    t.route_unpermute(back, perm, v); i2 = T(); acc["unpermute"] += i2 - h
    torch.ne(v, 0, out=f); j = T(); acc["ne"] += j - i2
    if it == 9:
        acc.clear()
for k2, x in acc.items():
    print(f"  {k2:16s} {x / 50 * 1e6:8.1f} us", flush=True)
t.close()
dist.destroy_process_group()
