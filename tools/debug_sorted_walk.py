import ctypes, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import sherman_amd as shm
from oracle.pyoracle import OracleTree, to_key
U64 = np.uint64
def dev(a): return torch.from_numpy(np.ascontiguousarray(a, dtype=U64).view(np.int64)).cuda()
def host(t): return t.cpu().numpy().view(U64)
L = shm.lib()
L.shm__debug_sort.argtypes = [ctypes.c_void_p]*5 + [ctypes.c_uint, ctypes.c_void_p]
L.shm__debug_sort.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
L.shm__debug_walk.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
t = shm.Tree(arena_bytes=256 << 20, max_batch=1 << 17)
rng = np.random.default_rng(5)
keys = np.array([to_key(i) for i in range(1, 21001)], dtype=U64)
for n in (1000, 5000, 8192, 21000, 100000):
    ks = rng.integers(0, 1 << 63, n, dtype=np.uint64) * U64(2) + U64(1)
    kd = dev(ks)
    ko = torch.empty_like(kd); po = torch.empty(n, dtype=torch.int32, device="cuda")
    for bb in (0,):
        rc = L.shm__debug_sort(t.h, kd.data_ptr(), n, ko.data_ptr(), po.data_ptr(), bb, None)
        p = po.cpu().numpy().astype(np.int64)
        okperm = np.array_equal(np.sort(p), np.arange(n))
        kh = host(ko)
        sortedok = np.all(np.diff((kh >> U64(bb)).astype(np.float64)) >= 0) if n > 1 else True
        match = np.array_equal(ks[p], kh) if okperm else False
        print(f"sort n={n} begin={bb} rc={rc} perm_ok={okperm} keys_match={match} sorted={sortedok}", flush=True)
# tree + walks
ins = keys[:3000]
t.insert_batch(dev(ins), dev(ins + U64(1)))
probe = keys
for depth in (4, 8):
    for use_perm in (False, True):
        kd = dev(probe); n = probe.size
        v = torch.zeros_like(kd); f = torch.zeros(n, dtype=torch.uint8, device="cuda")
        if use_perm:
            perm = torch.arange(n, dtype=torch.int32, device="cuda")
            rc = L.shm__debug_walk(t.h, kd.data_ptr(), perm.data_ptr(), n, v.data_ptr(), f.data_ptr(), depth, None)
        else:
            rc = L.shm__debug_walk(t.h, kd.data_ptr(), None, n, v.data_ptr(), f.data_ptr(), depth, None)
        vh, fh = host(v), f.cpu().numpy()
        exp_f = np.zeros(n, np.uint8); exp_f[:3000] = 1
        print(f"walk depth={depth} perm={use_perm} rc={rc} found_ok={np.array_equal(fh, exp_f)} bad={(fh!=exp_f).sum()} vals_ok={np.array_equal(vh[:3000], ins + U64(1))}", flush=True)
    # sorted probe
    sp = np.sort(probe)
    kd = dev(sp); n = sp.size
    v = torch.zeros_like(kd); f = torch.zeros(n, dtype=torch.uint8, device="cuda")
    rc = L.shm__debug_walk(t.h, kd.data_ptr(), None, n, v.data_ptr(), f.data_ptr(), depth, None)
    fh = f.cpu().numpy(); exp = np.isin(sp, ins).astype(np.uint8)
    print(f"walk sorted depth={depth} bad={(fh!=exp).sum()}", flush=True)
print("err", t.stats()["last_error"])
t.synchronize()
print("done")
