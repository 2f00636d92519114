"""Experiment (not product): the replica loop's SPARTA step (configs[3], K = 32,
GPT-2 124M, reference draw as packed words) overlapped with the inner AdamW.
The arena is cut into S slabs of whole 4096-element chunks; the AdamW for slab s
(all K rows, one launch) runs on the main stream while the rows average of slab
s - 1 (ga_sparta_average_local on the slab's rows and mask words) runs on a side
stream.  Prints the step time per S against AdamW alone and the serial
two-launch step, and checks the result is bit-identical to the serial step."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gym_amd import ops  # noqa: E402
from gym_amd.arena import ArenaLayout  # noqa: E402
from gym_amd.shapes import MODELS  # noqa: E402

dev = torch.device("cuda", 0)
K, p = 32, 0.005
layout = ArenaLayout(MODELS["gpt2-124m"]())
ld = layout.n
g = torch.Generator(device=dev)
g.manual_seed(3)
P = torch.randn(K, ld, device=dev, generator=g).mul_(0.02)
G = torch.randn(K, ld, device=dev, generator=g).mul_(1e-3)
M, V = torch.zeros_like(P), torch.zeros_like(P)
table, nb = ops.sparta_bernoulli_table(layout.offsets, layout.numels, dev)
bits = torch.zeros(ops.sparta_mask_words(ld), dtype=torch.int64, device=dev)
hp = dict(lerp_w=0.1, beta2=0.999, one_m_beta2=1 - 0.999, eps=1e-8, wd_factor=1 - 1e-3 * 0.01, l2_wd=0.0,
          step_size=-1e-3 / 0.1, bc2_sqrt=(1 - 0.999) ** 0.5)
side = torch.cuda.Stream(device=dev)


def slabs(S):
    ch = 4096
    nch = -(-ld // ch)
    cuts = [min(ld, (nch * i // S) * ch) for i in range(S + 1)]
    return [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]


def adam_only():
    ops.adam_step(P, G, M, V, **hp)


def serial():
    ops.sparta_torch_bernoulli(table, nb, p, 42, 0, 12, bits)
    ops.adam_step(P, G, M, V, **hp)
    ops.sparta_average_local(P, ld, float(K), mask=bits, layout="rows")


def overlapped(S):
    parts = slabs(S)
    main = torch.cuda.current_stream()

    def run():
        ops.sparta_torch_bernoulli(table, nb, p, 42, 0, 12, bits)
        evs = []
        for a, b in parts:
            ops.adam_step(P[:, a:b], G[:, a:b], M[:, a:b], V[:, a:b], **hp)
            e = torch.cuda.Event()
            e.record(main)
            evs.append(e)
        with torch.cuda.stream(side):
            for (a, b), e in zip(parts, evs):
                side.wait_event(e)
                ops.sparta_average_local(P[:, a:b], b - a, float(K), mask=bits[a // 64:], layout="rows")
        main.wait_stream(side)
    return run


def timeit(fn, reps=8):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


out = {"K": K, "ld": ld}
snap = [t.clone() for t in (P, G, M, V)]
serial()
ref = P.clone()
for t, s in zip((P, G, M, V), snap):
    t.copy_(s)
overlapped(8)()
out["bit_identical_S8"] = bool(torch.equal(P, ref))
out["adam_ms"] = round(timeit(adam_only), 4)
out["serial_ms"] = round(timeit(serial), 4)
for S in (1, 2, 4, 8, 16, 32):
    out[f"overlap_S{S}_ms"] = round(timeit(overlapped(S)), 4)
out["adam_ms_again"] = round(timeit(adam_only), 4)
print(json.dumps(out))
