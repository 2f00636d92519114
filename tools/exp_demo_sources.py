"""The DeMo wave decode (ga_demo_decode_sym) of GPT-2 350M over S = 1, 2, 4, 8
gathered payloads, for one or more builds of libgym_amd.so, in ONE process on
the same buffers (the physical placement of P / G, which moves the kernel by
up to 10% from process to process, is then common to every number), 25
interleaved rounds per (S, build).  Usage:
python tools/exp_demo_sources.py [--sources 1,2,4,8] lib1.so [lib2.so ...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from exp_demo_ablate import bind  # noqa: E402
from gym_amd.arena import ArenaLayout  # noqa: E402
from gym_amd.demo_codec import DemoPlan  # noqa: E402
from gym_amd.shapes import MODELS  # noqa: E402


def main():
    args = sys.argv[1:]
    sources = [1, 2, 4, 8]
    if args and args[0] == "--sources":
        sources, args = [int(x) for x in args[1].split(",")], args[2:]
    import ctypes
    dev = torch.device("cuda:0")
    layout = ArenaLayout(MODELS["gpt2-350m"]())
    plan = DemoPlan(layout).to(dev)
    torch.manual_seed(0)
    P = torch.randn(layout.n, device=dev) * 0.02
    G = torch.randn(layout.n, device=dev) * 1e-3
    P0 = P.clone()
    from gym_amd import ops
    Smax = max(sources)
    gathered = torch.zeros(Smax, 2 * plan.M, dtype=torch.int32, device=dev)
    for j in range(Smax):
        Dj = torch.randn(layout.n, device=dev) * 1e-4
        ops.demo_encode(plan, P.view(1, -1), G.view(1, -1), Dj.view(1, -1), gathered[j:j + 1], 1e-3, 0.999, 1.0)
    P.copy_(P0)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    vp = ctypes.c_void_p
    fns = {}
    for path in args:
        L = bind(path)
        for S in sources:
            def dec(L=L, S=S):
                rc = L.ga_demo_decode_sym(0, vp(plan.desc64.data_ptr()), plan.n64tensors, plan.n64chunks,
                                          vp(plan.groups.data_ptr()), plan.ngroups, vp(plan.F64.data_ptr()),
                                          vp(gathered.data_ptr()), gathered.stride(0), plan.M, S,
                                          vp(P.data_ptr()), vp(G.data_ptr()), 1, layout.n, 1e-3, s)
                assert rc == 0
            fns[(os.path.basename(path), S)] = dec
    for f in fns.values():
        for _ in range(10):
            f()
    torch.cuda.synchronize()
    times = {key: [] for key in fns}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(25):
        for key, f in fns.items():
            P.copy_(P0)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            times[key].append(e0.elapsed_time(e1))
    for (name, S), t in times.items():
        t = sorted(t)
        print(f"{name:28s} decode S={S} median {t[len(t) // 2]:.4f} ms  min {t[0]:.4f}", flush=True)


if __name__ == "__main__":
    main()
