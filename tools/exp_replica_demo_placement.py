"""Replica-mode DeMo (K local nodes, one [K, ld] parameter / gradient / delta set,
ReplicaRunner) with and without the placement of its three sets (diagnostic,
round 5): GPT-2 124M, K = 8, fp32, one process.  The codec's step (K-row encode
+ the world-1 exchange + decode of the K payloads) is timed on the ordinary
sets, then DeMoCodec.place moves the sets (what ReplicaRunner._place_demo does
after the first step) and the step is timed again.  Alternates OFF / ON per
repetition in fresh sets.  One JSON line per repetition.
Usage: python tools/exp_replica_demo_placement.py [reps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_amd.arena import ArenaLayout  # noqa: E402
from gym_amd.comm import Collective  # noqa: E402
from gym_amd.engine import DeMoCodec  # noqa: E402
from gym_amd.placement import time_probe  # noqa: E402
from gym_amd.shapes import MODELS  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    dev = torch.device("cuda:0")
    layout = ArenaLayout(MODELS["gpt2-124m"]())
    K, lr = 8, 1e-3
    codec = DeMoCodec(Collective(), K, layout, dev)
    for r in range(reps):
        g = torch.Generator(device=dev).manual_seed(r)
        P = torch.randn(K, layout.n, device=dev, generator=g) * 0.02
        G = torch.randn(K, layout.n, device=dev, generator=g) * 1e-3
        D = torch.zeros_like(P)
        codec(P, G, D, lr, 0.999, 0.0)  # the first step (its gathered payload feeds the probe)
        off = time_probe(lambda: codec(P, G, D, lr, 0.999, 0.0), reps=10)
        bufs, tens, rec = codec.place(P, G, D, lr, 0.999)
        if tens is not None:
            P2, G2, D2 = tens
        else:
            P2, G2, D2 = P, G, D
        on = time_probe(lambda: codec(P2, G2, D2, lr, 0.999, 0.0), reps=10)
        print(json.dumps({"rep": r, "K": K, "model": "gpt2-124m", "step_ms_ordinary": round(off, 4),
                          "step_ms_placed": round(on, 4), "record": rec}), flush=True)
        del P, G, D, P2, G2, D2, bufs, tens
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
