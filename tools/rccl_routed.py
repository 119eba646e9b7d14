"""tests/test_gpu_shard.py's forced-route case (nccl, world 1, "routed") in
this process instead of an mp.spawn child, so a profiler attached to this
command sees the exchange's RCCL kernels (tools/rccl_trace.sh)."""
import os
import sys
import tempfile

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "tests"))
sys.path.insert(0, R)

from test_gpu_shard import gpu_worker  # noqa: E402
from test_multi_rank import free_port, verify_against_unsharded  # noqa: E402

with tempfile.TemporaryDirectory() as d:
    gpu_worker(0, 1, free_port(), d, "nccl", "routed")
    verify_against_unsharded(d, 1)
print("routed world-1 RCCL path matches the unsharded oracle")
