"""The reference's own tree_test (test/tree_test.cpp:31-68), as C++ over the
host facade (sherman_amd/csrc/Tree.hpp -> C-ABI -> HIP), run on the GPU."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_native_tree_test():
    exe = os.path.join(ROOT, "tests", "native", "_build", "tree_test")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "native")])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "tree_test ok" in r.stdout
