"""r04 experiment: the fused AdamW step's four streams (gradient, parameters,
moments) placed one at a time in fresh device allocations
(gym_amd.placement.place_each, probe = ga_probe_adam_placement, the step's access
pattern with every value written back), GPT-2 124M, one node, three rounds in one
process: how much beyond the moments-only placement.  Diagnostic."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_amd import ops  # noqa: E402
from gym_amd.arena import ArenaLayout  # noqa: E402
from gym_amd.placement import place_each  # noqa: E402
from gym_amd.shapes import MODELS  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    n = ArenaLayout(MODELS["gpt2-124m"]()).n
    P = torch.randn(1, n, device=dev) * 0.02
    G = torch.randn(1, n, device=dev) * 1e-3
    M, V = torch.zeros(1, n, device=dev), torch.zeros(1, n, device=dev)
    for order in (("M", "V", "G", "P"), ("G", "P", "M", "V")):
        ts = {"P": P, "G": G, "M": M, "V": V}
        bufs, cur, stages = place_each([ts[k] for k in order],
                                       lambda *a: ops.probe_adam_placement(*[a[order.index(k)] for k in "PGMV"]),
                                       32, 0.3)
        print(f"order {order}: stage times (ordinary first) " + " ".join(f"{t:.4f}" for t in stages)
              + f"  moved {[b is not None for b in bufs]}", flush=True)
        del bufs, cur
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
