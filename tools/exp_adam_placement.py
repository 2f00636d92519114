"""r04 experiment: is the fused AdamW step (ga_adam_step) placement-sensitive the
way the DiLoCo step is (profiles/r04i_placement_map.txt)?  GPT-2 124M, one node:
param / grad ordinary allocations, the optimizer moments (exp_avg, exp_avg_sq,
one 1 GiB physical allocation each pair) in 48 candidates created one by one
(gym_amd.placement.PlacedBuffer), each timed; then the same for the DeMo
8-source decode's grad output (GPT-2 350M).  Diagnostic, not part of the library."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_amd import ops  # noqa: E402
from gym_amd.arena import ArenaLayout  # noqa: E402
from placed_buffer import PlacedBuffer  # noqa: E402
from gym_amd.shapes import MODELS  # noqa: E402


def qms(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    n = ArenaLayout(MODELS["gpt2-124m"]()).n
    P = torch.randn(n, device=dev) * 0.02
    G = torch.randn(n, device=dev) * 1e-3
    hp = dict(lerp_w=0.1, beta2=0.999, one_m_beta2=1 - 0.999, eps=1e-8, wd_factor=1 - 1e-5, l2_wd=0.0,
              step_size=-1e-2, bc2_sqrt=0.0316)
    M0, V0 = torch.zeros_like(P), torch.zeros_like(P)
    base = qms(lambda: ops.adam_step(P, G, M0, V0, **hp))
    print(f"adam, ordinary moments: {base:.4f} ms", flush=True)
    bufs, line = [], []
    for i in range(48):
        b = PlacedBuffer(8 * n, dev)
        bufs.append(b)
        t = b.tensor()
        M, V = t[:n], t[n:2 * n]
        M.zero_(), V.zero_()
        line.append(f"{qms(lambda: ops.adam_step(P, G, M, V, **hp)):.3f}")
    print("adam, moments in physical candidate i (ms):", " ".join(line), flush=True)
    for b in bufs:
        b.release()
    del bufs
    torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
