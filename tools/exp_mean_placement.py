"""Does the replica mean-reduce (SimpleReduce / FedAvg in replica mode: every
replica row <- the mean of the K rows, in place, ga_replica_mean) depend on
where its [K, ld] set sits physically, as the DiLoCo step does?  Diagnostic
(round 5): GPT-2 124M, K = 8, fp32; C fresh [K, ld] allocations created one at a
time and all held (distinct physical memory, gym_amd.placement.DeviceBuffer),
the in-place mean timed on each.  One JSON line: ms per candidate, in creation
order, the ordinary allocation first.  Usage: python tools/exp_mean_placement.py [C]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_amd import ops  # noqa: E402
from gym_amd.arena import ArenaLayout  # noqa: E402
from gym_amd.placement import DeviceBuffer, time_probe  # noqa: E402
from gym_amd.shapes import MODELS  # noqa: E402


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    dev = torch.device("cuda:0")
    n = ArenaLayout(MODELS["gpt2-124m"]()).n
    K = 8
    base = torch.randn(K, n, device=dev) * 1e-3
    times = [time_probe(lambda: ops.replica_mean(base, base, n=n), reps=5)]
    held = []
    torch.cuda.empty_cache()
    for _ in range(C):
        b = DeviceBuffer(4 * K * n, dev)
        held.append(b)
        t = b.tensor()[:K * n].view(K, n)
        t.copy_(base)
        times.append(time_probe(lambda: ops.replica_mean(t, t, n=n), reps=5))
    gb = 2 * K * 4 * n / 1e9
    print(json.dumps({"what": "in-place replica mean over [8, n] fp32, GPT-2 124M", "bytes_GB": round(gb, 3),
                      "ms": [round(x, 4) for x in times], "min": round(min(times), 4), "max": round(max(times), 4),
                      "frac_hbm_min_ms": round(gb / (min(times) * 1e-3) / 8000.0, 4),
                      "frac_hbm_ordinary": round(gb / (times[0] * 1e-3) / 8000.0, 4)}))


if __name__ == "__main__":
    main()
