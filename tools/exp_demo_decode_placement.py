"""r04 experiment: is the DeMo 8-source decode (GPT-2 350M, what every GPU runs at
8 nodes) placement-sensitive like the 1-source decode (profiles/r04g_demo_placement.txt)?
The gathered payload of 8 distinct nodes; (a) the grad output in 24 physical
candidates (gym_amd.placement.PlacedBuffer, created one by one) with the params in
an ordinary allocation, (b) the params in 24 candidates with the grad ordinary;
each timed.  Diagnostic, not part of the library."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_amd import ops  # noqa: E402
from gym_amd.arena import ArenaLayout  # noqa: E402
from gym_amd.demo_codec import DemoPlan  # noqa: E402
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
    L = ArenaLayout(MODELS["gpt2-350m"]())
    plan = DemoPlan(L, chunk=64, topk=32).to(dev)
    n = L.n
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    P = torch.randn(1, n, device=dev, generator=g) * 0.02
    G = torch.zeros(1, n, device=dev)
    payload = torch.zeros(8, 2 * plan.M, dtype=torch.int32, device=dev)
    D = torch.zeros(1, n, device=dev)
    for k in range(8):
        G.normal_(0.0, 1e-3, generator=g)
        D.zero_()
        ops.demo_encode(plan, P, G, D, payload[k:k + 1], 1e-3, 0.999, 1.0)
    del D
    base = qms(lambda: ops.demo_decode(plan, payload, P, G, 1e-3))
    print(f"8-source decode, ordinary buffers: {base:.4f} ms", flush=True)
    for what in ("grad", "param"):
        bufs, line = [], []
        for i in range(24):
            b = PlacedBuffer(4 * n, dev)
            bufs.append(b)
            t = b.tensor()[:n].view(1, n)
            if what == "grad":
                t.zero_()
                line.append(qms(lambda: ops.demo_decode(plan, payload, P, t, 1e-3)))
            else:
                t.copy_(P)
                line.append(qms(lambda: ops.demo_decode(plan, payload, t, G, 1e-3)))
        print(f"8-source decode, {what} in physical candidate i (ms): " + " ".join(f"{x:.3f}" for x in line),
              flush=True)
        print(f"   best {min(line):.4f} median {sorted(line)[12]:.4f} worst {max(line):.4f}", flush=True)
        for b in bufs:
            b.release()
        del bufs
        torch.cuda.empty_cache()
    print(f"8-source decode, ordinary buffers again: {qms(lambda: ops.demo_decode(plan, payload, P, G, 1e-3)):.4f} ms",
          flush=True)


if __name__ == "__main__":
    main()
