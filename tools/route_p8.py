"""The routed get's per-step overhead at P = 8, at the C4 shard size, on one
GPU: what one rank of an 8-GPU run does around its walk --
slot placement of its 2^20 queries into 8 runs (shm__route_slots), the walk
over the received runs (8 x cap slots: here this rank's own tree answers
all of them, so the walk has a 2^27-key shard's cost), the gather of the
results to input order (shm__route_gather) -- timed with HIP events on one
stream against the plain local walk of the same queries.  The exchange
itself (RCCL over xGMI) is not in either number.
usage: python tools/route_p8.py [keys_log2] [steps] [P]"""
import ctypes
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import sherman_amd as shm

kl = int(sys.argv[1]) if len(sys.argv) > 1 else 27
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
P = int(sys.argv[3]) if len(sys.argv) > 3 else 8
torch.cuda.set_device(0)
n_keys, batch = 1 << kl, 1 << 20
cap = batch // P + 6 * int(math.sqrt(batch // P)) + 256  # shard.cpp get_slot_cap
t = shm.Tree(arena_bytes=max(2 << 30, n_keys * 48), max_batch=P * cap)
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

L = shm.lib()
L.shm__route_slots.restype = ctypes.c_int
L.shm__route_slots.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                               ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
L.shm__route_slots_ex.restype = ctypes.c_int
L.shm__route_slots_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                  ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
L.shm__route_gather.restype = ctypes.c_int
L.shm__route_gather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
sp = torch.cuda.current_stream().cuda_stream
cursor = torch.zeros(P + 1, dtype=torch.int32, device="cuda")
slots = torch.empty(P * cap, dtype=torch.int64, device="cuda")
spos = torch.empty(batch, dtype=torch.int32, device="cuda")
ovk = torch.zeros(batch, dtype=torch.int64, device="cuda")
ovi = torch.zeros(batch, dtype=torch.int32, device="cuda")
res = torch.empty_like(slots)
out = torch.empty(batch, dtype=torch.int64, device="cuda")
fnd = torch.empty(batch, dtype=torch.uint8, device="cuda")
v = torch.empty(batch, dtype=torch.int64, device="cuda")
f = torch.empty(batch, dtype=torch.uint8, device="cuda")


def local(i):
    t.search_batch(qs[i % 8], v, f)


filled = [False]


def routed(i):
    # as shard.cpp's search_begin: the runs padded once per capacity
    assert L.shm__route_slots_ex(t.h, qs[i % 8].data_ptr(), batch, P, cap, cursor.data_ptr(),
                                 slots.data_ptr(), spos.data_ptr(), ovk.data_ptr(),
                                 ovi.data_ptr(), 0 if filled[0] else 1, sp) == 0
    filled[0] = True
    t.search_batch(slots, res)
    assert L.shm__route_gather(res.data_ptr(), spos.data_ptr(), batch, out.data_ptr(),
                               fnd.data_ptr(), sp) == 0


def timed(fn):
    for i in range(5):
        fn(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for i in range(steps):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / steps


# the bench's pipelining (bench.py at N > 1 through the C shard): two slots
# on two streams, batch i + 1's placement queued before batch i's walk and
# gather, against the local get's two walks in flight
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
pslots = [dict(cursor=torch.zeros(P + 1, dtype=torch.int32, device="cuda"),
               slots=torch.empty(P * cap, dtype=torch.int64, device="cuda"),
               spos=torch.empty(batch, dtype=torch.int32, device="cuda"),
               res=torch.empty(P * cap, dtype=torch.int64, device="cuda"),
               out=torch.empty(batch, dtype=torch.int64, device="cuda"),
               fnd=torch.empty(batch, dtype=torch.uint8, device="cuda"),
               v=torch.empty(batch, dtype=torch.int64, device="cuda"),
               f=torch.empty(batch, dtype=torch.uint8, device="cuda"),
               filled=False) for _ in range(2)]
ctr_lock = [None]  # the hook's claim words are one set: placements stay on one stream order


def place(i):
    ps, st = pslots[i & 1], streams[i & 1]
    with torch.cuda.stream(st):
        # the hook's single claim-word set: placements must not overlap each
        # other, so each waits for the previous placement (the shard has a set
        # per slot and needs no such wait)
        if ctr_lock[0] is not None:
            st.wait_event(ctr_lock[0])
        assert L.shm__route_slots_ex(t.h, qs[i % 8].data_ptr(), batch, P, cap,
                                     ps["cursor"].data_ptr(), ps["slots"].data_ptr(),
                                     ps["spos"].data_ptr(), ovk.data_ptr(), ovi.data_ptr(),
                                     0 if ps["filled"] else 1, st.cuda_stream) == 0
        ps["filled"] = True
        ev = torch.cuda.Event()
        ev.record(st)
        ctr_lock[0] = ev


def finish(i):
    ps, st = pslots[i & 1], streams[i & 1]
    with torch.cuda.stream(st):
        t.search_batch(ps["slots"], ps["res"], stream=st)
        assert L.shm__route_gather(ps["res"].data_ptr(), ps["spos"].data_ptr(), batch,
                                   ps["out"].data_ptr(), ps["fnd"].data_ptr(),
                                   st.cuda_stream) == 0


def routed_pipe(i):
    if i == 0:
        place(0)
    place(i + 1)
    finish(i)


def local_pipe(i):
    ps, st = pslots[i & 1], streams[i & 1]
    t.search_batch(qs[i % 8], ps["v"], ps["f"], stream=st)


def timed_pipe(fn):
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
    for i in range(5):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
    for i in range(steps):
        fn(i + 5)
    for st in streams:
        torch.cuda.current_stream().wait_stream(st)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / steps


for _ in range(6):  # the read phase's pair-form directory
    local(0)
us_local = timed(local)
us_routed = timed(routed)
us_local2 = timed(local)
us_local_pipe = timed_pipe(local_pipe)
us_routed_pipe = timed_pipe(routed_pipe)
routed(0)
local(0)
torch.cuda.synchronize()
assert torch.equal(out, v) and torch.equal(fnd, f), "routed results differ from the local get"
assert int(cursor[P].item()) == 0, "overflow at this capacity"
print(json.dumps({"keys": n_keys, "batch": batch, "P": P, "cap": cap, "steps": steps,
                  "local_us_per_step": round(min(us_local, us_local2), 2),
                  "routed_us_per_step": round(us_routed, 2),
                  "overhead_us": round(us_routed - min(us_local, us_local2), 2),
                  "pipelined": {"local_us_per_step": round(us_local_pipe, 2),
                                "routed_us_per_step": round(us_routed_pipe, 2),
                                "overhead_us": round(us_routed_pipe - us_local_pipe, 2)},
                  "condition": "one stream, HIP events around the steps; the exchange is not in "
                               "either number (one tree answers all 8 runs)"}))
