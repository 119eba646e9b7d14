"""The routed C2 get through the C-ABI shard (shm_shard_*) at world 1 over
RCCL, pipelined as bench.py does at N > 1 (batch i + 1 begun before batch
i ends, two streams, two slots), next to the local get on the same tree.
Prints us per step; run under rocprofv3 --kernel-trace --stats for the
route's kernels.  usage: python tools/route_c2.py [keys_log2] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

import sherman_amd as shm

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
kl = int(sys.argv[1]) if len(sys.argv) > 1 else 26
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
n_keys, batch = 1 << kl, 1 << 20
t = shm.Tree(arena_bytes=max(2 << 30, n_keys * 48), max_batch=batch + batch // 4)
k = torch.empty(1 << 22, dtype=torch.int64, device="cuda")
for c in range(1, n_keys + 1, 1 << 22):
    m = min(1 << 22, n_keys + 1 - c)
    t.gen_keys(c, m, k[:m])
    for o in range(0, m, batch):
        t.insert_batch(k[o:min(m, o + batch)], k[o:min(m, o + batch)])
ids = torch.randint(1, n_keys + 1, (8, batch), device="cuda")
qs = []
for i in range(8):
    q = torch.empty(batch, dtype=torch.int64, device="cuda")
    t.hash_keys(ids[i], q)
    qs.append(q)
cs = shm.CShard(t, 1, 0, dist)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
outs = [(torch.empty(batch, dtype=torch.int64, device="cuda"),
         torch.empty(batch, dtype=torch.uint8, device="cuda")) for _ in range(2)]
for sx in streams:
    sx.wait_stream(torch.cuda.current_stream())


def local(i):
    v, f = outs[i & 1]
    t.search_batch(qs[i % 8], v, f, stream=streams[i & 1])


pend = {}


def routed(i):
    if i not in pend:
        with torch.cuda.stream(streams[i & 1]):
            pend[i] = cs.search_begin(qs[i % 8])
    with torch.cuda.stream(streams[(i + 1) & 1]):
        pend[i + 1] = cs.search_begin(qs[(i + 1) % 8])
    with torch.cuda.stream(streams[i & 1]):
        cs.search_end(pend.pop(i), *outs[i & 1])


for name, fn in (("local", local), ("routed", routed)):
    for i in range(10):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(10, 10 + steps):
        fn(i)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"{name}: {dt * 1e6:.1f} us/step, {batch / dt / 1e6:.0f} Mops/s", flush=True)
# drain the begun batch
for i in list(pend):
    with torch.cuda.stream(streams[i & 1]):
        cs.search_end(pend.pop(i), *outs[i & 1])
torch.cuda.synchronize()
v0 = torch.empty(batch, dtype=torch.int64, device="cuda")
f0 = torch.empty(batch, dtype=torch.uint8, device="cuda")
t.search_batch(qs[0], v0, f0)
cs.search(qs[0], outs[0][0], outs[0][1])
torch.cuda.synchronize()
print("routed == local:", bool(torch.equal(v0, outs[0][0]) and torch.equal(f0, outs[0][1])))
cs.close()
t.close()
dist.destroy_process_group()
