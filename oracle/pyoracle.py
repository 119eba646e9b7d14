"""ctypes binding for the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker / CPU baseline, never as
the measured or shipped path.  See oracle/sherman_oracle.h for what the oracle
restates (reference file:line) and how it is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

u64 = ctypes.c_uint64
vp = ctypes.c_void_p


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.orc_tree_create.restype = vp
        L.orc_tree_create.argtypes = [u64]
        L.orc_tree_wrap_image.restype = vp
        L.orc_tree_wrap_image.argtypes = [vp, u64, u64, u64, ctypes.c_uint16]
        L.orc_tree_destroy.argtypes = [vp]
        L.orc_search.restype = ctypes.c_int
        L.orc_search.argtypes = [vp, u64, ctypes.POINTER(u64)]
        L.orc_insert.restype = ctypes.c_int
        L.orc_insert.argtypes = [vp, u64, u64]
        L.orc_del.argtypes = [vp, u64]
        L.orc_range_query.restype = u64
        L.orc_range_query.argtypes = [vp, u64, u64, vp, u64]
        L.orc_range_query_batch.restype = u64
        L.orc_range_query_batch.argtypes = [vp, vp, vp, u64, vp, vp, u64]
        L.orc_search_batch.argtypes = [vp, vp, u64, vp, vp]
        L.orc_search_batch_mt.restype = ctypes.c_double
        L.orc_search_batch_mt.argtypes = [vp, vp, u64, vp, vp, ctypes.c_int]
        L.orc_apply_batch.argtypes = [vp, vp, vp, u64]
        L.orc_apply_batch_mt.restype = ctypes.c_double
        L.orc_apply_batch_mt.argtypes = [vp, vp, vp, u64, ctypes.c_int]
        L.orc_range_query_batch_mt.restype = u64
        L.orc_range_query_batch_mt.argtypes = [vp, vp, vp, u64, vp, vp, u64, ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_double)]
        L.orc_c1_build.argtypes = [vp, u64, ctypes.c_double, u64]
        L.orc_c1_bench.argtypes = [vp, ctypes.c_int, u64, ctypes.c_double, u64, ctypes.c_int,
                                   ctypes.c_double, vp]
        L.orc_root_ptr.restype = u64
        L.orc_root_ptr.argtypes = [vp]
        L.orc_root_level.restype = ctypes.c_int
        L.orc_root_level.argtypes = [vp]
        L.orc_pages_used.restype = u64
        L.orc_pages_used.argtypes = [vp]
        L.orc_arena.restype = vp
        L.orc_arena.argtypes = [vp]
        L.orc_arena_bytes_used.restype = u64
        L.orc_arena_bytes_used.argtypes = [vp]
        L.orc_read_pages.restype = u64
        L.orc_read_pages.argtypes = [vp]
        L.orc_dump_pairs.restype = u64
        L.orc_dump_pairs.argtypes = [vp, vp, vp, u64]
        L.orc_check.restype = ctypes.c_int
        L.orc_check.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(u64),
                                ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_int)]
        L.orc_cityhash64.restype = u64
        L.orc_cityhash64.argtypes = [vp, ctypes.c_size_t]
        L.orc_to_key.restype = u64
        L.orc_to_key.argtypes = [u64, u64]
        L.orc_zipf_fill.argtypes = [u64, ctypes.c_double, u64, vp, u64]
        L.orc_op_mix.argtypes = [ctypes.c_uint, ctypes.c_int, vp, u64]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(vp)


class OracleTree:
    """Reference-semantics tree on a host arena (the checker)."""

    def __init__(self, arena_bytes=1 << 26, image=None, root_ptr=0, node_id=0,
                 spare_bytes=0):
        """New tree, or (image=...) a tree over a page image; spare_bytes of
        free pages after the image take the splits of later inserts."""
        L = lib()
        self._image = None
        if image is not None:
            used = image.nbytes
            if spare_bytes:
                self._image = np.zeros(used + spare_bytes, dtype=np.uint8)
                self._image[:used] = np.asarray(image, dtype=np.uint8).reshape(-1)
            else:
                self._image = np.ascontiguousarray(image, dtype=np.uint8)
            self.h = L.orc_tree_wrap_image(_p(self._image), used, self._image.nbytes,
                                           root_ptr, node_id)
        else:
            self.h = L.orc_tree_create(arena_bytes)
        if not self.h:
            raise MemoryError("oracle arena")

    def close(self):
        if self.h:
            lib().orc_tree_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def insert(self, k, v):
        return lib().orc_insert(self.h, k, v)

    def search(self, k):
        v = u64(0)
        f = lib().orc_search(self.h, k, ctypes.byref(v))
        return bool(f), v.value

    def delete(self, k):
        lib().orc_del(self.h, k)

    def range_query(self, lo, hi, cap=1 << 20):
        out = np.zeros(cap, dtype=np.uint64)
        n = lib().orc_range_query(self.h, lo, hi, _p(out), cap)
        return out[: min(n, cap)].copy(), n

    def range_query_batch(self, lo, hi):
        """Scans [lo_i, hi_i] in order: (counts, values concatenated)."""
        lo = np.ascontiguousarray(lo, dtype=np.uint64)
        hi = np.ascontiguousarray(hi, dtype=np.uint64)
        counts = np.zeros(lo.size, dtype=np.uint64)
        cap = max(1024, 128 * lo.size)
        while True:
            out = np.empty(cap, dtype=np.uint64)
            total = lib().orc_range_query_batch(self.h, _p(lo), _p(hi), lo.size, _p(counts),
                                                _p(out), cap)
            if total <= cap:
                return counts, out[:total].copy()
            cap = int(total)

    def search_batch(self, keys):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        vals = np.zeros(keys.size, dtype=np.uint64)
        found = np.zeros(keys.size, dtype=np.uint8)
        lib().orc_search_batch(self.h, _p(keys), keys.size, _p(vals), _p(found))
        return vals, found

    def search_batch_mt(self, keys, nthreads):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        vals = np.zeros(keys.size, dtype=np.uint64)
        found = np.zeros(keys.size, dtype=np.uint8)
        secs = lib().orc_search_batch_mt(self.h, _p(keys), keys.size, _p(vals),
                                         _p(found), nthreads)
        return vals, found, secs

    def apply_batch(self, keys, vals):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        vals = np.ascontiguousarray(vals, dtype=np.uint64)
        lib().orc_apply_batch(self.h, _p(keys), _p(vals), keys.size)

    def apply_batch_mt(self, keys, vals, nthreads):
        """apply_batch on `nthreads` threads partitioned by page lock word
        (same contents); returns seconds."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        vals = np.ascontiguousarray(vals, dtype=np.uint64)
        return lib().orc_apply_batch_mt(self.h, _p(keys), _p(vals), keys.size, nthreads)

    def range_query_batch_mt(self, lo, hi, nthreads):
        """range_query_batch on `nthreads` threads: (counts, values, seconds)."""
        lo = np.ascontiguousarray(lo, dtype=np.uint64)
        hi = np.ascontiguousarray(hi, dtype=np.uint64)
        counts = np.zeros(lo.size, dtype=np.uint64)
        cap = max(1024, 128 * lo.size)
        secs = ctypes.c_double()
        while True:
            out = np.empty(cap, dtype=np.uint64)
            total = lib().orc_range_query_batch_mt(self.h, _p(lo), _p(hi), lo.size, _p(counts),
                                                   _p(out), cap, nthreads, ctypes.byref(secs))
            if total <= cap:
                return counts, out[:total].copy(), secs.value
            cap = int(total)

    def c1_build(self, keyspace, warm_ratio=0.8, preload=1024000):
        """The reference benchmark's tree, one insert at a time in the
        reference's order (orc_c1_build; ctypes releases the GIL, so this
        can run beside other work)."""
        lib().orc_c1_build(self.h, keyspace, warm_ratio, preload)

    def c1_bench(self, nthreads, keyspace, theta=0.0, seed_base=0x5EED0000, windows=5,
                 window_s=2.0):
        """The reference benchmark's read phase on pinned threads
        (test/benchmark.cpp:165-188, 302-341): Mops/s of each window."""
        out = np.zeros(windows, dtype=np.float64)
        lib().orc_c1_bench(self.h, nthreads, keyspace, theta, seed_base, windows, window_s,
                           _p(out))
        return out

    def dump(self, cap=None):
        L = lib()
        if cap is None:
            cap = L.orc_dump_pairs(self.h, None, None, 0)
        ks = np.zeros(cap, dtype=np.uint64)
        vs = np.zeros(cap, dtype=np.uint64)
        n = L.orc_dump_pairs(self.h, _p(ks), _p(vs), cap)
        return ks[:n], vs[:n]

    def check(self):
        a, b, c, h = u64(), u64(), u64(), ctypes.c_int()
        rc = lib().orc_check(self.h, ctypes.byref(a), ctypes.byref(b),
                             ctypes.byref(c), ctypes.byref(h))
        return rc, dict(leaves=a.value, internal=b.value, keys=c.value,
                        height=h.value)

    @property
    def root_ptr(self):
        return lib().orc_root_ptr(self.h)

    @property
    def root_level(self):
        return lib().orc_root_level(self.h)

    @property
    def read_pages(self):
        return lib().orc_read_pages(self.h)

    def image(self):
        L = lib()
        n = L.orc_arena_bytes_used(self.h)
        buf = (ctypes.c_uint8 * n).from_address(L.orc_arena(self.h))
        return np.frombuffer(buf, dtype=np.uint8).copy()


def cityhash64_u64(i):
    x = u64(i)
    return lib().orc_cityhash64(ctypes.byref(x), 8)


def to_key(i, keyspace=0):
    return lib().orc_to_key(i, keyspace)


def zipf_fill(n_items, theta, seed, count):
    out = np.zeros(count, dtype=np.uint64)
    lib().orc_zipf_fill(n_items, theta, seed, _p(out), count)
    return out


def op_mix(seed, read_ratio, count):
    out = np.zeros(count, dtype=np.uint8)
    lib().orc_op_mix(seed, read_ratio, _p(out), count)
    return out
