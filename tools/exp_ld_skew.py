"""Experiment: ga_diloco_outer time vs the replica stride ld (skewing the K
replica streams across HBM channels).  Standalone diagnostic."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_amd import ops  # noqa: E402

n, K = 124475904, 8
dev = torch.device("cuda:0")
master = torch.randn(n, device=dev) * 0.02
mom = torch.zeros(n, device=dev)
for pad in [0, 64, 256, 1024, 4096, 16384, 65536 + 1024, 1 << 20]:
    ld = n + pad
    src = torch.randn(K, ld, device=dev) * 0.02
    for _ in range(3):
        ops.diloco_outer(src, master, mom, src, n, K, 0.7, 0.9, 0.0, 0.0, True, False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.diloco_outer(src, master, mom, src, n, K, 0.7, 0.9, 0.0, 0.0, True, False)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"pad {pad:8d} floats: {ms:.4f} ms  {(2 * K + 4) * 4 * n / ms / 1e9:.1f} GB/s", flush=True)
    del src
