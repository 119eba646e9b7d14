"""sherman_amd — MI355X-native Sherman B+tree hot path (batched get / insert).

Python view of the C-ABI in include/sherman_amd.h (libsherman_amd.so, built
in-tree by `make -C sherman_amd`).  The host interface mirrors the reference
`Tree` (include/Tree.h:42-63): `search`, `insert`, `del_`, `range_query`,
plus the batched forms the GPU path is built around.  Batch methods take
torch CUDA (HIP) tensors or raw device pointers; torch is used only as the
device-memory / stream plumbing.

There is no CPU fallback: if the HIP library is missing or no GPU is
visible, constructing a Tree raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SHM_LIB_PATH: another build of the library (A/B of builds, tools/ab_builds.sh)
LIB_PATH = os.environ.get("SHM_LIB_PATH") or os.path.join(_HERE, "libsherman_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "sherman_amd.h")

SHM_OK = 0
SHM_EINVAL = -22
SHM_ENOMEM = -12
SHM_EIO = -5
SHM_EAGAIN = -11
SHM_E2BIG = -7
SHM_ENOSPC = -28
SHM_FLAG_SORT_GETS = 0x1
SHM_FLAG_LEAF_DIR = 0x2
SHM_FLAG_AUTO_SORT_GETS = 0x4
SHM_FLAG_TOP_LDS = 0x8
SHM_FLAG_PAGE_CHECK = 0x10

KEY_MAX = (1 << 64) - 1
PAGE_SIZE = 1024
LEAF_CARDINALITY = 54       # include/Tree.h:193-195
INTERNAL_CARDINALITY = 61   # include/Tree.h:189-191

u64 = ctypes.c_uint64
u32 = ctypes.c_uint32
vp = ctypes.c_void_p


class ShmConfig(ctypes.Structure):
    _fields_ = [
        ("struct_size", ctypes.c_uint32),
        ("device", ctypes.c_int32),
        ("node_id", ctypes.c_uint16),
        ("reserved0", ctypes.c_uint16),
        ("flags", ctypes.c_uint32),
        ("arena_bytes", u64),
        ("max_batch", u64),
        ("num_locks", u32),
        ("sort_bits", u32),
        ("key_lo", u64),
        ("key_bits", u32),
        ("reserved1", u32),
    ]


class ShmStats(ctypes.Structure):
    _fields_ = [
        ("root_ptr", u64),
        ("root_level", u32),
        ("height", u32),
        ("pages_used", u64),
        ("pages_capacity", u64),
        ("arena_bytes", u64),
        ("batches", u64),
        ("splits", u64),
        ("last_error", u32),
        ("reserved", u32),
    ]


class ShermanError(RuntimeError):
    def __init__(self, rc, what=""):
        self.rc = rc
        msg = lib().shm_strerror(rc).decode()
        super().__init__(f"{what}: {msg} ({rc})" if what else f"{msg} ({rc})")


class ShmError(ctypes.Structure):
    _fields_ = [("bits", u32), ("chunk", u32), ("status", ctypes.c_int32), ("resumed", u32)]


class ShmIndexStats(ctypes.Structure):
    _fields_ = [(f, u64) for f in ("gets", "start_internal", "right_moves", "page_hops",
                                   "entry_reads", "hits", "dir_fp_hits")]


class ShmDirStats(ctypes.Structure):
    _fields_ = [("form", u32), ("bits", u32), ("entries", u64), ("bytes", u64), ("builds", u64),
                ("pages_at_build", u64), ("pages_since_build", u64),
                ("last_build_ms", ctypes.c_double), ("total_build_ms", ctypes.c_double),
                ("maintained", u32), ("exact", u32)]


DIR_FORMS = {0: "none", 1: "fingerprints", 2: "pairs"}


class ShmProfile(ctypes.Structure):
    _fields_ = [
        ("calls", u64),
        ("queries", u64),
        ("order_ms", ctypes.c_double),
        ("walk_ms", ctypes.c_double),
        ("insert_calls", u64),
        ("insert_ops", u64),
        ("insert_ms", ctypes.c_double),
        ("upsert_ms", ctypes.c_double),
        ("range_calls", u64),
        ("range_queries", u64),
        ("range_ms", ctypes.c_double),
        ("insert_unique", u64),
        ("insert_dels", u64),
        ("insert_staged", u64),
        ("walk_kernel_ms", ctypes.c_double),
    ]


_lib = None
ABI_VERSION = 11  # SHM_ABI_VERSION in include/sherman_amd.h

# (name, restype, argtypes) — every symbol declared in include/sherman_amd.h
_SIGNATURES = [
    ("shm_config_init", ctypes.c_int, [ctypes.POINTER(ShmConfig)]),
    ("shm_tree_create", ctypes.c_int, [ctypes.POINTER(ShmConfig), ctypes.POINTER(vp)]),
    ("shm_tree_destroy", ctypes.c_int, [vp]),
    ("shm_strerror", ctypes.c_char_p, [ctypes.c_int]),
    ("shm_abi_version", ctypes.c_int, []),
    ("shm_search_batch", ctypes.c_int, [vp, vp, u64, vp, vp, vp]),
    ("shm_insert_batch", ctypes.c_int, [vp, vp, vp, u64, vp]),
    ("shm_insert_batch_async", ctypes.c_int, [vp, vp, vp, u64, vp]),
    ("shm_insert_order", ctypes.c_int, [vp, vp, vp, u64, vp, ctypes.POINTER(u32)]),
    ("shm_insert_apply", ctypes.c_int, [vp, u32, vp]),
    ("shm_mixed_batch", ctypes.c_int, [vp, vp, u64, vp, vp, vp, vp, u64, vp]),
    ("shm_del_batch", ctypes.c_int, [vp, vp, u64, vp]),
    ("shm_range_query", ctypes.c_int, [vp, vp, vp, u64, vp, vp, vp, vp]),
    ("shm_range_query_batch", ctypes.c_int,
     [vp, vp, vp, u64, vp, vp, vp, u64, ctypes.POINTER(u64), vp]),
    ("shm_range_query_batch_async", ctypes.c_int,
     [vp, vp, vp, u64, vp, vp, vp, u64, vp, vp]),
    ("shm_range_query_slots", ctypes.c_int, [vp, vp, vp, u64, u64, vp, vp, vp, vp]),
    ("shm_stats", ctypes.c_int, [vp, ctypes.POINTER(ShmStats)]),
    ("shm_dump_image", ctypes.c_int, [vp, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
    ("shm_load_image", ctypes.c_int, [vp, vp, u64, u64]),
    ("shm_check", ctypes.c_int, [vp, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]),
    ("shm_synchronize", ctypes.c_int, [vp]),
    ("shm_read_words", ctypes.c_int, [vp, vp, u64, vp, vp]),
    ("shm_last_error", ctypes.c_int, [vp, ctypes.POINTER(ShmError), ctypes.c_int]),
    ("shm_last_chunk", u32, [vp]),
    ("shm_profile_enable", ctypes.c_int, [vp, ctypes.c_int]),
    ("shm_profile_read", ctypes.c_int, [vp, ctypes.POINTER(ShmProfile), ctypes.c_int]),
    ("shm_index_stats", ctypes.c_int, [vp, ctypes.POINTER(ShmIndexStats), ctypes.c_int]),
    ("shm_dir_stats", ctypes.c_int, [vp, ctypes.POINTER(ShmDirStats)]),
    ("shm_route_bucket", ctypes.c_int, [vp, vp, u64, u32, vp, vp, vp, vp]),
    ("shm_route_permute", ctypes.c_int, [vp, vp, vp, u64, vp, vp]),
    ("shm_route_unpermute", ctypes.c_int, [vp, vp, vp, u64, vp, vp]),
    ("shm_route_unpermute_found", ctypes.c_int, [vp, vp, vp, u64, vp, vp, vp]),
    ("shm_tree_max_batch", u64, [vp]),
    ("shm_nccl_unique_id", ctypes.c_int, [vp, u64]),
    ("shm_shard_create", ctypes.c_int, [vp, vp, u64, u32, u32, ctypes.POINTER(vp)]),
    ("shm_shard_create_with_comm", ctypes.c_int, [vp, vp, u32, u32, ctypes.POINTER(vp)]),
    ("shm_shard_destroy", ctypes.c_int, [vp]),
    ("shm_shard_search", ctypes.c_int, [vp, vp, u64, vp, vp, vp]),
    ("shm_shard_search_begin", ctypes.c_int, [vp, vp, u64, vp, ctypes.POINTER(u32)]),
    ("shm_shard_search_end", ctypes.c_int, [vp, u32, vp, vp]),
    ("shm_shard_insert", ctypes.c_int, [vp, vp, vp, u64, vp]),
    ("shm_shard_range_query", ctypes.c_int,
     [vp, vp, vp, u64, u64, vp, vp, vp, u64, ctypes.POINTER(u64), vp]),
    ("shm_shard_range_query_async", ctypes.c_int,
     [vp, vp, vp, u64, u64, vp, vp, vp, u64, u64, vp, vp]),
    ("shm_shard_synchronize", ctypes.c_int, [vp]),
    ("shm_shard_range_values", ctypes.c_int, [vp, vp, u64, vp]),
    ("shm_lock_bench", ctypes.c_int, [vp, vp, u64, vp]),
    ("shm_gen_keys", ctypes.c_int, [vp, u64, u64, u64, vp, vp]),
    ("shm_hash_keys", ctypes.c_int, [vp, vp, u64, u64, vp, vp]),
]


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", _HERE, "-j8"])


def lib():
    """Load libsherman_amd.so (fails loudly if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} missing: build it with `make -C sherman_amd` "
                "(there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in _SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.shm_abi_version() != ABI_VERSION:
            raise ImportError(f"{LIB_PATH} has ABI {L.shm_abi_version()}, this package "
                              f"expects {ABI_VERSION}: rebuild with `make -C sherman_amd`")
        _lib = L
    return _lib


def _check(rc, what):
    if rc != SHM_OK:
        raise ShermanError(rc, what)


def _ptr(x):
    """Device pointer of a torch tensor / int / None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    return x.data_ptr()


def _stream_ptr(stream):
    """hipStream_t for the C-ABI; default = torch's current stream so the
    library is ordered after the torch ops that produced its inputs."""
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    if isinstance(stream, int):
        return stream or None
    return stream.cuda_stream or None


class _StreamDone:
    """Completion of the work queued so far on a raw hipStream_t (None = the
    null stream) of `device`, for a pending result: .synchronize() waits for
    that stream.  No event is recorded at issue time -- a record between two
    kernels leaves the device idle ~5-7 us (tools/event_gap.hip) -- so the
    wait may also cover work queued there later, never less."""

    def __init__(self, stream_ptr, device):
        self.stream_ptr, self.device = stream_ptr, device

    def synchronize(self):
        import torch
        s = (torch.cuda.ExternalStream(self.stream_ptr, device=self.device) if self.stream_ptr
             else torch.cuda.default_stream(self.device))
        s.synchronize()


def _record_on(stream_ptr, device):
    return _StreamDone(stream_ptr, device)


class PendingRange:
    """Result of Tree.range_query_batch_async: (counts, values) once the
    scans have run.  tot = device (total, error bits); done = the stream the
    scans were queued on (_StreamDone: resolved when they were issued, so
    .result() waits for them whatever stream is current then)."""

    def __init__(self, tree, counts, vals, tot=None, done=None):
        self.tree, self.counts, self.vals, self.tot, self.done = tree, counts, vals, tot, done

    def result(self):
        if self.tot is None:  # ran synchronously
            return self.counts, self.vals
        import torch
        if self.done is not None:
            self.done.synchronize()
        else:
            torch.cuda.synchronize()
        total, err = (int(x) for x in self.tot.cpu().tolist())
        if err:
            self.tree.synchronize()  # raises the device error
            raise ShermanError(SHM_EIO, "range_query_batch_async")
        # learn the size even when this batch overflowed, so the next async
        # batch gets a buffer that fits
        self.tree._rq_cap = max(self.tree._rq_cap, total + total // 4)
        if total > self.vals.numel():
            raise ShermanError(SHM_ENOSPC, "range_query_batch_async: %d values, buffer %d"
                               % (total, self.vals.numel()))
        self.tot = None
        self.vals = self.vals[:total]
        return self.counts, self.vals


class PendingSlots:
    """Result of Tree.range_query_slots: (counts, vals[n, slot_cap]) once the
    scans have run; .result() raises the device error, if any, and
    SHM_ENOSPC when some scan's count passed slot_cap (its buffer then holds
    its first slot_cap values)."""

    def __init__(self, tree, counts, vals, slot_cap, status, done):
        self.tree, self.counts, self.slot_cap = tree, counts, slot_cap
        self.vals = vals.view(-1)[:counts.numel() * slot_cap].view(counts.numel(), slot_cap)
        self.status, self.done = status, done

    def check(self):
        """Scans over slot_cap once the scans have run (device errors raise)."""
        if self.done is not None:
            self.done.synchronize()
        self.tree.synchronize()  # raises a device error of the queued calls
        return int((self.counts > self.slot_cap).sum().item())

    def result(self):
        ovf = self.check()
        if ovf:
            raise ShermanError(SHM_ENOSPC, "range_query_slots: %d scans passed slot_cap %d"
                               % (ovf, self.slot_cap))
        return self.counts, self.vals

    def packed(self):
        """(counts, values concatenated in scan order): the compact form."""
        import torch
        c, v = self.result()
        if c.numel() == 0:
            return c, v.view(-1)[:0]
        mask = torch.arange(self.slot_cap, device=c.device)[None, :] < c[:, None]
        return c, v[mask]


class Tree:
    """One shard's B+tree in HBM (reference: class Tree, include/Tree.h:42)."""

    def __init__(self, arena_bytes=1 << 30, max_batch=1 << 20, device=0,
                 node_id=0, sort_gets="auto", num_locks=None, sort_bits=16,
                 key_lo=0, key_bits=64, leaf_dir=True, top_lds=False, page_check=False):
        L = lib()
        cfg = ShmConfig()
        _check(L.shm_config_init(ctypes.byref(cfg)), "config")
        cfg.device = device
        cfg.node_id = node_id
        cfg.arena_bytes = arena_bytes
        cfg.max_batch = max_batch
        if num_locks is not None:
            cfg.num_locks = num_locks
        cfg.sort_bits = sort_bits
        cfg.key_lo = key_lo
        cfg.key_bits = key_bits
        # sort_gets: True (always order get batches by key), False (never),
        # "auto" (order dense batches, SHM_FLAG_AUTO_SORT_GETS)
        cfg.flags = ((SHM_FLAG_SORT_GETS if sort_gets is True else 0) |
                     (SHM_FLAG_AUTO_SORT_GETS if sort_gets == "auto" else 0) |
                     (SHM_FLAG_LEAF_DIR if leaf_dir else 0) |
                     (SHM_FLAG_TOP_LDS if top_lds else 0) |
                     (SHM_FLAG_PAGE_CHECK if page_check else 0))
        h = vp()
        _check(L.shm_tree_create(ctypes.byref(cfg), ctypes.byref(h)), "shm_tree_create")
        self.h = h
        self.device = device
        self.node_id = node_id
        self.max_batch = max_batch
        self._scratch = {}

    # -- lifecycle ----------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            lib().shm_tree_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- batched hot path (device tensors) -----------------------------------
    def search_batch(self, keys, vals_out, found_out=None, stream=None):
        _check(lib().shm_search_batch(self.h, _ptr(keys), keys.numel(),
                                      _ptr(vals_out), _ptr(found_out),
                                      _stream_ptr(stream)), "search_batch")

    def insert_batch(self, keys, vals, stream=None):
        """Apply the batch and return its status (one host synchronisation)."""
        _check(lib().shm_insert_batch(self.h, _ptr(keys), _ptr(vals), keys.numel(),
                                      _stream_ptr(stream)), "insert_batch")

    def insert_batch_async(self, keys, vals, stream=None):
        """Queue the batch on the device without a host wait; its status is
        raised by the next synchronising call (synchronize, insert_batch)."""
        _check(lib().shm_insert_batch_async(self.h, _ptr(keys), _ptr(vals), keys.numel(),
                                            _stream_ptr(stream)), "insert_batch_async")

    def insert_order(self, keys, vals, stream=None):
        """shm_insert_order: queue one chunk's ordering (n <= max_batch) on
        `stream`; returns the ticket for insert_apply.  keys / vals must stay
        alive until the ordering has run."""
        t = u32(0)
        _check(lib().shm_insert_order(self.h, _ptr(keys), _ptr(vals), keys.numel(),
                                      _stream_ptr(stream), ctypes.byref(t)), "insert_order")
        return int(t.value)

    def insert_apply(self, ticket, stream=None):
        """shm_insert_apply: queue the tree changes of an ordered chunk."""
        _check(lib().shm_insert_apply(self.h, ticket, _stream_ptr(stream)), "insert_apply")

    def mixed_batch(self, get_keys, vals_out, found_out, ins_keys, ins_vals, stream=None):
        """One mixed batch (shm_mixed_batch): the gets see the tree before the
        batch's inserts; the inserts are queued as insert_batch_async."""
        _check(lib().shm_mixed_batch(self.h, _ptr(get_keys), get_keys.numel(), _ptr(vals_out),
                                     _ptr(found_out) if found_out is not None else None,
                                     _ptr(ins_keys), _ptr(ins_vals), ins_keys.numel(),
                                     _stream_ptr(stream)), "mixed_batch")

    def del_batch(self, keys, stream=None):
        _check(lib().shm_del_batch(self.h, _ptr(keys), keys.numel(),
                                   _stream_ptr(stream)), "del_batch")

    def range_query_batch(self, lo, hi, stream=None):
        """Batched inclusive scans [lo_i, hi_i]: (counts, values concatenated
        in query order), both on the device; one host synchronisation (the
        total).  Results are stream-ordered on `stream`."""
        import torch
        n = lo.numel()
        dev = lo.device
        counts = torch.empty(n, dtype=torch.int64, device=dev)
        offs = torch.empty(n, dtype=torch.int64, device=dev)
        cap = getattr(self, "_rq_cap", 1 << 16)
        vals = torch.empty(cap, dtype=torch.int64, device=dev)
        total = u64(0)
        rc = lib().shm_range_query_batch(self.h, _ptr(lo), _ptr(hi), n, _ptr(counts),
                                         _ptr(offs), _ptr(vals), cap, ctypes.byref(total),
                                         _stream_ptr(stream))
        total = int(total.value)
        if rc == SHM_ENOSPC:
            vals = torch.empty(total, dtype=torch.int64, device=dev)
            rc = lib().shm_range_query(self.h, _ptr(lo), _ptr(hi), n, _ptr(counts),
                                       _ptr(offs), _ptr(vals), _stream_ptr(stream))
        _check(rc, "range_query_batch")
        self._rq_cap = max(cap, total + total // 4)
        return counts, vals[:total]

    def range_query_batch_async(self, lo, hi, stream=None):
        """range_query_batch without the host synchronisation (n <= max_batch):
        the scans are queued on `stream` and the returned PendingRange gives
        (counts, values) on .result().  The value buffer is sized from earlier
        totals (the first call on a handle runs synchronously to learn one);
        .result() raises SHM_ENOSPC if this batch's total outgrew it, which
        cannot be redone after later mutating calls."""
        import torch
        cap = getattr(self, "_rq_cap", None)
        if cap is None:
            return PendingRange(None, *self.range_query_batch(lo, hi, stream))
        n = lo.numel()
        dev = lo.device
        counts = torch.empty(n, dtype=torch.int64, device=dev)
        offs = torch.empty(n, dtype=torch.int64, device=dev)
        vals = torch.empty(cap, dtype=torch.int64, device=dev)
        tot = torch.empty(2, dtype=torch.int64, device=dev)
        sp = _stream_ptr(stream)
        _check(lib().shm_range_query_batch_async(self.h, _ptr(lo), _ptr(hi), n, _ptr(counts),
                                                 _ptr(offs), _ptr(vals), cap, _ptr(tot), sp),
               "range_query_batch_async")
        return PendingRange(self, counts, vals, tot, _record_on(sp, dev))

    def range_query_slots(self, lo, hi, slot_cap, stream=None, vals=None, counts=None,
                          status=None):
        """Batched scans with a buffer per scan (shm_range_query_slots, the
        reference's Tree::range_query(from, to, buffer) per scan): queued on
        `stream` without a host wait.  Returns PendingSlots: .result() gives
        (counts, vals[n, slot_cap]); scan i's first min(counts[i], slot_cap)
        values are vals[i, :counts[i]].  vals / counts may be passed in
        (reused buffers); status (2 device words, zeroed by the caller)
        accumulates {scans past slot_cap, error bits} over calls."""
        import torch
        n = lo.numel()
        dev = lo.device
        if counts is None:
            counts = torch.empty(n, dtype=torch.int64, device=dev)
        if vals is None:
            vals = torch.empty((n, slot_cap), dtype=torch.int64, device=dev)
        assert vals.numel() >= n * slot_cap and counts.numel() >= n
        sp = _stream_ptr(stream)
        _check(lib().shm_range_query_slots(self.h, _ptr(lo), _ptr(hi), n, slot_cap, _ptr(counts),
                                           _ptr(vals), _ptr(status), sp),
               "range_query_slots")
        return PendingSlots(self, counts[:n], vals, slot_cap, status, _record_on(sp, dev))

    # -- reference single-op API (Tree.h:47-54) -------------------------------
    def _dev(self, name, n):
        import torch
        t = self._scratch.get(name)
        if t is None or t.numel() < n:
            t = torch.empty(max(n, 1), dtype=torch.int64, device=f"cuda:{self.device}")
            self._scratch[name] = t
        return t[:n]

    def insert(self, k, v):
        import torch
        ks = torch.tensor([to_i64(k)], dtype=torch.int64, device=f"cuda:{self.device}")
        vs = torch.tensor([to_i64(v)], dtype=torch.int64, device=f"cuda:{self.device}")
        self.insert_batch(ks, vs)

    def search(self, k):
        import torch
        ks = torch.tensor([to_i64(k)], dtype=torch.int64, device=f"cuda:{self.device}")
        vs = self._dev("sv", 1)
        fs = torch.empty(1, dtype=torch.uint8, device=f"cuda:{self.device}")
        self.search_batch(ks, vs, fs)
        self.synchronize()
        return bool(fs.item()), from_i64(vs.item())

    def del_(self, k):
        import torch
        ks = torch.tensor([to_i64(k)], dtype=torch.int64, device=f"cuda:{self.device}")
        self.del_batch(ks)

    # -- introspection ---------------------------------------------------------
    def synchronize(self):
        _check(lib().shm_synchronize(self.h), "synchronize")

    def last_error(self, reset=False):
        """shm_last_error: the device error block as the last synchronising
        call that found bits read it (bits, the chunk that first saw them, the
        status returned, resumed chunks so far)."""
        e = ShmError()
        _check(lib().shm_last_error(self.h, ctypes.byref(e), 1 if reset else 0), "last_error")
        return {f: getattr(e, f) for f, _ in ShmError._fields_}

    def last_chunk(self):
        """Id of the last insert chunk queued (shm_last_chunk)."""
        return int(lib().shm_last_chunk(self.h))

    def stats(self):
        s = ShmStats()
        _check(lib().shm_stats(self.h, ctypes.byref(s)), "stats")
        return {f: getattr(s, f) for f, _ in ShmStats._fields_}

    def check(self):
        a, b, c = u64(), u64(), u64()
        _check(lib().shm_check(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
               "check")
        return dict(leaves=a.value, internal=b.value, keys=c.value)

    def dump_image(self):
        import numpy as np
        used, root = u64(), u64()
        _check(lib().shm_dump_image(self.h, None, 0, ctypes.byref(used), ctypes.byref(root)),
               "dump")
        buf = np.zeros(used.value, dtype=np.uint8)
        _check(lib().shm_dump_image(self.h, buf.ctypes.data_as(vp), used.value,
                                    ctypes.byref(used), ctypes.byref(root)), "dump")
        return buf, root.value

    def load_image(self, image, root_ptr):
        import numpy as np
        image = np.ascontiguousarray(image, dtype=np.uint8)
        _check(lib().shm_load_image(self.h, image.ctypes.data_as(vp), image.nbytes,
                                    root_ptr), "load_image")

    def profile(self, on=True, index_stats=False):
        _check(lib().shm_profile_enable(self.h, (1 if on else 0) | (2 if index_stats else 0)),
               "profile_enable")

    def index_stats(self, reset=True):
        """The get walk's index statistics (shm_index_stats; collected while
        profile(index_stats=True))."""
        st = ShmIndexStats()
        _check(lib().shm_index_stats(self.h, ctypes.byref(st), 1 if reset else 0), "index_stats")
        return {f: getattr(st, f) for f, _ in ShmIndexStats._fields_}

    def dir_stats(self):
        """The leaf directory: form ("none" / "fingerprints" / "pairs"),
        entries, device bytes, builds and their device time (shm_dir_stats)."""
        st = ShmDirStats()
        _check(lib().shm_dir_stats(self.h, ctypes.byref(st)), "dir_stats")
        d = {f: getattr(st, f) for f, _ in ShmDirStats._fields_}
        d["form"] = DIR_FORMS.get(d["form"], str(d["form"]))
        return d

    def dir_config(self, maint=None, mem_limit=0):
        """Test hook (shm__dir_config): directory upkeep by the chunks on /
        off (None: as is; "always": every chunk, also those with no search
        since the last one) and a byte cap on directory allocations."""
        m = -1 if maint is None else 2 if maint == "always" else int(bool(maint))
        _check(_hooks().shm__dir_config(self.h, m, mem_limit), "dir_config")

    def dir_verify(self):
        """Diagnostics (shm__dir_verify): every directory entry the walks
        trust checked against the tree as it is now."""
        out = (u64 * 8)()
        _check(_hooks().shm__dir_verify(self.h, out), "dir_verify")
        return {"checked": out[0], "bad_lists": out[1], "bad_pairs": out[2], "bad_fps": out[3],
                "first_bad": [x - 1 for x in out[4:8] if x]}

    def profile_read(self, reset=True):
        p = ShmProfile()
        _check(lib().shm_profile_read(self.h, ctypes.byref(p), 1 if reset else 0),
               "profile_read")
        return {f: getattr(p, f) for f, _ in ShmProfile._fields_}

    # -- routing / generators ---------------------------------------------------
    def read_i64(self, t, stream=None):
        """A small device int64 tensor (<= 32 words) as a list of ints, via
        the zero-copy read-back (shm_read_words); CPU tensors via tolist()."""
        if t.device.type != "cuda":
            return t.tolist()
        n = t.numel()
        buf = (ctypes.c_int64 * n)()
        _check(lib().shm_read_words(self.h, _ptr(t), 8 * n, buf, _stream_ptr(stream)),
               "read_words")
        return list(buf)

    def route_bucket(self, keys, num_shards, keys_out, perm_out, counts_out, stream=None):
        _check(lib().shm_route_bucket(self.h, _ptr(keys), keys.numel(), num_shards,
                                      _ptr(counts_out), _ptr(keys_out), _ptr(perm_out),
                                      _stream_ptr(stream)), "route_bucket")

    def route_permute(self, vals_in, perm, out, stream=None):
        _check(lib().shm_route_permute(self.h, _ptr(vals_in), _ptr(perm), vals_in.numel(),
                                       _ptr(out), _stream_ptr(stream)), "permute")

    def route_unpermute(self, vals_in, perm, out, stream=None, found=None):
        if found is not None:  # found[perm[i]] = vals_in[i] != 0 in the same pass
            _check(lib().shm_route_unpermute_found(self.h, _ptr(vals_in), _ptr(perm),
                                                   vals_in.numel(), _ptr(out), _ptr(found),
                                                   _stream_ptr(stream)), "unpermute")
            return
        _check(lib().shm_route_unpermute(self.h, _ptr(vals_in), _ptr(perm), vals_in.numel(),
                                         _ptr(out), _stream_ptr(stream)), "unpermute")

    def lock_bench(self, keys, stream=None):
        """Tree::lock_bench for every key: its lock word taken and released."""
        _check(lib().shm_lock_bench(self.h, _ptr(keys), keys.numel(), _stream_ptr(stream)),
               "lock_bench")

    def hash_keys(self, ids, out, keyspace=0, stream=None):
        _check(lib().shm_hash_keys(self.h, _ptr(ids), ids.numel(), keyspace, _ptr(out),
                                   _stream_ptr(stream)), "hash_keys")

    def gen_keys(self, first, n, out, keyspace=0, stream=None):
        _check(lib().shm_gen_keys(self.h, first, n, keyspace, _ptr(out),
                                  _stream_ptr(stream)), "gen_keys")


def to_i64(x):
    """u64 -> signed int64 bit pattern (torch has no uint64 arithmetic)."""
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= (1 << 63) else x


def from_i64(x):
    return x & ((1 << 64) - 1)


# library-internal test hooks (csrc/shard.cpp): an in-process group of P
# shard handles on one GPU whose collectives are device copies
_HOOKS = [
    ("shm__local_group_create", ctypes.c_int, [u32, ctypes.POINTER(vp)]),
    ("shm__local_group_destroy", ctypes.c_int, [vp]),
    ("shm__shard_create_local", ctypes.c_int, [vp, vp, u32, ctypes.POINTER(vp)]),
    ("shm__upper_force", ctypes.c_int, [vp, u32]),
    ("shm__hog", ctypes.c_int, [u32, u64, vp]),
    ("shm__mark", ctypes.c_int, [u32, vp]),
    ("shm__early_pages", ctypes.c_int, [vp, ctypes.POINTER(u64)]),
    ("shm__dir_config", ctypes.c_int, [vp, ctypes.c_int, u64]),
    ("shm__shard_force_route", ctypes.c_int, [vp, ctypes.c_int]),
    ("shm__dir_verify", ctypes.c_int, [vp, ctypes.POINTER(u64)]),
]


def _hooks():
    L = lib()
    for name, res, args in _HOOKS:
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    return L


class LocalGroup:
    """P in-process ranks on one GPU for CShard.local (test hook): every
    rank is driven by its own host thread, all on one shared stream."""

    def __init__(self, world):
        g = vp()
        _check(_hooks().shm__local_group_create(world, ctypes.byref(g)), "local_group")
        self.h, self.world = g, world

    def close(self):
        if getattr(self, "h", None):
            _hooks().shm__local_group_destroy(self.h)
            self.h = None


class CShard:
    """A range shard of a multi-GPU tree behind the C-ABI (shm_shard_*): the
    routed get / insert / range scan (slots, RCCL all-to-all, the overflow
    rounds, local batch, gather) runs in C++ over its own RCCL
    communicators.  All ranks construct it together (ncclCommInitRank); rank
    0's unique id travels over `dist`."""

    @classmethod
    def local(cls, tree, group, rank):
        """Rank `rank` of a LocalGroup (test hook; call from that rank's
        thread: creation is a collective)."""
        self = cls.__new__(cls)
        h = vp()
        _check(_hooks().shm__shard_create_local(tree.h, group.h, rank, ctypes.byref(h)),
               "shard_create_local")
        self.h, self.tree, self.world, self.rank = h, tree, group.world, rank
        return self

    def __init__(self, tree, world, rank, dist, group=None):
        import torch
        L = lib()
        idb = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            _check(L.shm_nccl_unique_id(idb.data_ptr(), 128), "nccl_unique_id")
        backend = dist.get_backend(group)
        t = idb.to(f"cuda:{tree.device}") if backend == "nccl" else idb
        dist.broadcast(t, 0, group=group)
        idb = t.cpu()
        h = vp()
        _check(L.shm_shard_create(tree.h, idb.data_ptr(), 128, world, rank, ctypes.byref(h)),
               "shard_create")
        self.h, self.tree, self.world, self.rank = h, tree, world, rank

    def close(self):
        if getattr(self, "h", None):
            lib().shm_shard_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def force_route(self, on=True):
        """Test hook (shm__shard_force_route): every get and insert takes the
        routed path through the transport even at world 1 (RCCL sends each
        run to this rank itself)."""
        _check(_hooks().shm__shard_force_route(self.h, 1 if on else 0), "force_route")

    def search(self, keys, vals_out, found_out, stream=None):
        _check(lib().shm_shard_search(self.h, _ptr(keys), keys.numel(), _ptr(vals_out),
                                      _ptr(found_out), _stream_ptr(stream)), "shard_search")

    def search_begin(self, keys, stream=None):
        tk = u32()
        _check(lib().shm_shard_search_begin(self.h, _ptr(keys), keys.numel(),
                                            _stream_ptr(stream), ctypes.byref(tk)),
               "shard_search_begin")
        return tk.value

    def search_end(self, ticket, vals_out, found_out):
        _check(lib().shm_shard_search_end(self.h, ticket, _ptr(vals_out), _ptr(found_out)),
               "shard_search_end")

    def insert(self, keys, vals, stream=None):
        _check(lib().shm_shard_insert(self.h, _ptr(keys), _ptr(vals), keys.numel(),
                                      _stream_ptr(stream)), "shard_insert")

    def range_query(self, lo, hi, n_cap=None, stream=None):
        """Routed scans [lo_i, hi_i]: (counts, values in key order across
        shards).  n_cap: the same on every rank, >= lo.numel() (default: the
        tree's max_batch // P, so every rank may pass any n up to it)."""
        import torch
        n, dev = lo.numel(), lo.device
        if n_cap is None:
            n_cap = self.tree.max_batch // self.world
        counts = torch.empty(n, dtype=torch.int64, device=dev)
        offs = torch.empty(n, dtype=torch.int64, device=dev)
        cap = getattr(self, "_rq_cap", 1 << 16)
        vals = torch.empty(cap, dtype=torch.int64, device=dev)
        total = u64(0)
        rc = lib().shm_shard_range_query(self.h, _ptr(lo), _ptr(hi), n, n_cap, _ptr(counts),
                                         _ptr(offs), _ptr(vals), cap, ctypes.byref(total),
                                         _stream_ptr(stream))
        total = int(total.value)
        self._rq_cap = max(cap, total + total // 4)
        if rc == SHM_ENOSPC:
            # the exchange completed: copy its values into a buffer that fits
            # (local, no second collective)
            vals = torch.empty(self._rq_cap, dtype=torch.int64, device=dev)
            rc = lib().shm_shard_range_values(self.h, _ptr(vals), self._rq_cap,
                                              _stream_ptr(stream))
        _check(rc, "shard_range_query")
        return counts, vals[:total]

    def range_query_async(self, lo, hi, vals_cap, peer_cap, n_cap=None, stream=None,
                          status=None):
        """range_query with no host synchronisation (shm_shard_range_query_async):
        the values travel in fixed runs of peer_cap per peer.  Returns
        (counts, offsets, vals[vals_cap], status): status[0] the total,
        status[1] flags (nonzero: incomplete, repeat with range_query before
        any tree change), all written on `stream`."""
        import torch
        n, dev = lo.numel(), lo.device
        if n_cap is None:
            n_cap = self.tree.max_batch // self.world
        counts = torch.empty(n, dtype=torch.int64, device=dev)
        offs = torch.empty(n, dtype=torch.int64, device=dev)
        vals = torch.empty(max(vals_cap, 1), dtype=torch.int64, device=dev)
        if status is None:
            status = torch.zeros(2, dtype=torch.int64, device=dev)
        _check(lib().shm_shard_range_query_async(self.h, _ptr(lo), _ptr(hi), n, n_cap,
                                                 _ptr(counts), _ptr(offs), _ptr(vals), vals_cap,
                                                 peer_cap, _ptr(status), _stream_ptr(stream)),
               "shard_range_query_async")
        return counts, offs, vals, status

    def synchronize(self):
        _check(lib().shm_shard_synchronize(self.h), "shard_synchronize")


def header_symbols(path=HEADER_PATH):
    """Names of every function declared in include/sherman_amd.h."""
    import re
    txt = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:int|uint32_t|uint64_t|const char \*)\s*(shm_\w+)\s*\(",
                                 txt, re.M)))
