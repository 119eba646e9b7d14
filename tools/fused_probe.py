"""Single-op inserts with the fused segmentation (SHM_FUSED_SEG=1), one line
per insert (diagnostic): python tools/fused_probe.py N"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

assert torch.cuda.is_available()
import sherman_amd as shm  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
t = shm.Tree(arena_bytes=64 << 20, max_batch=1 << 14)
for i in range(1, n):
    t0 = time.time()
    t.insert(i, i * 2)
    print(f"insert {i} ok {time.time() - t0:.4f}s", flush=True)
print("stats", t.stats(), flush=True)
