"""r04 experiment: does the DeMo encode / decode rate depend on where the delta
buffer sits physically relative to the gradient (as the DiLoCo step does on
master/momentum, profiles/r04b_placement_search_p*.txt)?  GPT-2 350M, one node:
six separately allocated delta buffers against one gradient / parameter set,
each timed (encode, 1-source decode, the chunk-stream probe) interleaved over
three rounds in ONE process.  Diagnostic, not part of the library."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_amd import ops  # noqa: E402
from gym_amd.arena import ArenaLayout  # noqa: E402
from gym_amd.demo_codec import DemoPlan  # noqa: E402
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
    L = ArenaLayout(MODELS["gpt2-350m"]())
    plan = DemoPlan(L, chunk=64, topk=32).to(dev)
    n = L.n
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    P = torch.randn(1, n, device=dev, generator=g) * 0.02
    G = torch.randn(1, n, device=dev, generator=g) * 1e-3
    payload = torch.zeros(1, 2 * plan.M, dtype=torch.int32, device=dev)
    Ds = [torch.zeros(1, n, device=dev) for _ in range(6)]
    cols = 1024
    rows = (n // cols) // 64 * 64
    for r in range(3):
        for i, D in enumerate(Ds):
            enc = qms(lambda: ops.demo_encode(plan, P, G, D, payload, 1e-3, 0.999, 1.0))
            dec = qms(lambda: ops.demo_decode(plan, payload, P, D, 1e-3))  # grad written into the candidate
            prb = qms(lambda: ops.probe_chunk_stream(D.view(-1), G.view(-1), rows, cols, 0))
            print(f"round {r} delta#{i} (ptr % 1G = {D.data_ptr() % (1 << 30) >> 20} MiB): encode {enc:.4f} ms  "
                  f"decode(1 src, grad -> this buffer) {dec:.4f} ms  chunk-stream probe {prb:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
