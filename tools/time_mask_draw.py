"""Time the reference-draw SPARTA mask (draw_masks over GPT-2 124M's 148
tensors) eager vs as one HIP graph replay; prints one JSON line."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gym_amd.arena import ArenaLayout  # noqa: E402
from gym_amd.shapes import MODELS  # noqa: E402
from gym_amd.strategy.sparta import MaskDraw, RandomIndexSelector, draw_masks  # noqa: E402

dev = torch.device("cuda:0")
shapes = MODELS["gpt2-124m"]()
L = ArenaLayout(shapes)
mask = torch.zeros(L.n, dtype=torch.uint8, device=dev)
views = L.views(mask)
sel = RandomIndexSelector(0.005)
out = {}
for mode in ("eager", "graph", "fused"):
    MaskDraw.use_graphs = mode == "graph"
    MaskDraw.fused = mode == "fused"
    st = MaskDraw()
    for _ in range(3):
        draw_masks(sel, views, views, set(), 0, st)
    torch.cuda.synchronize()
    reps = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(reps):
        draw_masks(sel, views, views, set(), 0, st)
    e1.record()
    e1.synchronize()
    out[mode] = {"wall_ms": (time.perf_counter() - t0) * 1e3 / reps, "gpu_ms": e0.elapsed_time(e1) / reps,
                 "graph": st.graph is not None}
print(json.dumps(out), flush=True)
# bit check: fused vs eager draws, same generator state
st = MaskDraw()
ref = torch.zeros_like(mask)
rv = L.views(ref)
ok = True
for step in range(3):
    g0 = torch.cuda.get_rng_state()
    MaskDraw.fused = MaskDraw.use_graphs = False
    draw_masks(sel, rv, rv, set(), step, MaskDraw())
    g1 = torch.cuda.get_rng_state()
    torch.cuda.set_rng_state(g0)
    MaskDraw.fused = True
    draw_masks(sel, views, views, set(), step, st)
    ok &= bool(torch.equal(ref, mask)) and bool(torch.equal(g1, torch.cuda.get_rng_state()))
print(json.dumps({"fused_equals_eager_124m": ok}), flush=True)
