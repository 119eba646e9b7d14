"""C-ABI boundary checks that run without a GPU: the library loads, exports
every symbol include/sherman_amd.h declares, and its host-only entry points
behave (no compute calls here)."""
import ctypes
import os
import re
import subprocess

import pytest

import sherman_amd as shm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_builds_for_gfx950():
    """The shared object embeds gfx950 code objects (hipcc --offload-arch)."""
    assert os.path.exists(shm.LIB_PATH), "run __graft_entry__.build() first"
    blob = open(shm.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"__hip_fatbin" in blob or b".hip_fatbin" in blob


def test_exports_every_header_symbol():
    L = shm.lib()
    names = shm.header_symbols()
    assert len(names) >= 15
    for n in names:
        assert hasattr(L, n), f"{n} declared in include/sherman_amd.h but not exported"
    declared = {n for n, _, _ in shm._SIGNATURES}
    assert declared == set(names), "python binding out of sync with the header"


def test_exported_symbols_are_c_abi():
    out = subprocess.run(["nm", "-D", "--defined-only", shm.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (shm_\w+)$", out, re.M))
    for n in shm.header_symbols():
        assert n in exported  # unmangled => extern "C"


def test_config_layout_and_defaults():
    assert ctypes.sizeof(shm.ShmConfig) == 56
    cfg = shm.ShmConfig()
    assert shm.lib().shm_config_init(ctypes.byref(cfg)) == 0
    assert cfg.struct_size == 56
    assert cfg.key_lo == 0 and cfg.key_bits == 64
    assert cfg.flags == shm.SHM_FLAG_LEAF_DIR | shm.SHM_FLAG_AUTO_SORT_GETS
    assert cfg.max_batch == 1 << 20 and cfg.num_locks == 16384  # kNumOfLock (Common.h:87-93)
    assert shm.lib().shm_abi_version() == shm.ABI_VERSION == 11
    assert shm.lib().shm_strerror(shm.SHM_EINVAL).startswith(b"invalid")


def test_create_rejects_bad_config_without_touching_gpu():
    L = shm.lib()
    cfg = shm.ShmConfig()
    L.shm_config_init(ctypes.byref(cfg))
    h = ctypes.c_void_p()
    cfg.struct_size = 12
    assert L.shm_tree_create(ctypes.byref(cfg), ctypes.byref(h)) == shm.SHM_EINVAL
    L.shm_config_init(ctypes.byref(cfg))
    cfg.max_batch = 0
    assert L.shm_tree_create(ctypes.byref(cfg), ctypes.byref(h)) == shm.SHM_EINVAL
    L.shm_config_init(ctypes.byref(cfg))
    cfg.key_bits = 65
    assert L.shm_tree_create(ctypes.byref(cfg), ctypes.byref(h)) == shm.SHM_EINVAL
    # the insert ordering's bin counts are 24-bit fields (isort.hip bin_prefix)
    L.shm_config_init(ctypes.byref(cfg))
    cfg.max_batch = 1 << 24
    assert L.shm_tree_create(ctypes.byref(cfg), ctypes.byref(h)) == shm.SHM_EINVAL
    assert L.shm_tree_destroy(None) == shm.SHM_EINVAL


def test_layout_constants_match_reference():
    """include/Tree.h:189-195 cardinalities from the packed sizes."""
    header, leaf_entry, int_entry = 35, 18, 16
    assert (1024 - header - 2 - 8) // int_entry == shm.INTERNAL_CARDINALITY
    assert (1024 - header - 2 - 8) // leaf_entry == shm.LEAF_CARDINALITY
    txt = open(os.path.join(ROOT, "sherman_amd", "csrc", "layout.h")).read()
    for name, val in [("kOffRecords", 44), ("kOffInternalRear", 1020),
                      ("kOffLeafRear", 1016), ("kOffLowest", 28), ("kOffHighest", 36)]:
        assert re.search(rf"{name} = {val};", txt), name


def test_no_cpu_fallback_without_library(tmp_path, monkeypatch):
    """The product path fails loudly when the HIP library is absent."""
    monkeypatch.setattr(shm, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(shm, "_lib", None)
    with pytest.raises(ImportError):
        shm.lib()
