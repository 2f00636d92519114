"""Per-phase cycle shares of ga_demo_encode (diagnostic build, make stamps).

Loads build/libgym_amd_stamps.so (same kernels + s_memtime stamps at phase
boundaries), runs the encode of GPT-2 350M once, and prints the median
cycles each workgroup spent per phase.  Read the shares, not the absolute
time (the stamps themselves perturb the kernel)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gym_amd import _lib  # noqa: E402
from gym_amd.arena import ArenaLayout  # noqa: E402
from gym_amd.demo_codec import DemoPlan  # noqa: E402
from gym_amd.shapes import MODELS  # noqa: E402

PHASES = ["error-feedback+prefetch", "DCT product 1", "DCT product 2", "top-k select+emit", "residual (MFMA)",
          "delta store"]


WAVE_PHASES = ["64x64: load+error feedback", "64x64: row product+park", "64x64: column product",
               "64x64: top-k", "64x64: residual", "64x64: delta store", "row groups: load", "row groups: rest"]


def main():
    wave = "--wave" in sys.argv
    argv = [a for a in sys.argv[1:] if a != "--wave"]
    model = argv[0] if argv else "gpt2-350m"
    L = ctypes.CDLL(os.path.join(ROOT, "build", "libgym_amd_stamps.so"))
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    L.ga_demo_stamps_set.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    layout = ArenaLayout(MODELS[model]())
    plan = DemoPlan(layout).to(dev)
    P = torch.randn(layout.n, device=dev) * 0.02
    G = torch.randn(layout.n, device=dev) * 1e-3
    D = torch.zeros(layout.n, device=dev)
    pl = torch.zeros(2 * plan.M, dtype=torch.int32, device=dev)
    stamps = torch.zeros(plan.nchunks * 16, dtype=torch.int64, device=dev)
    assert L.ga_demo_stamps_set(ctypes.c_void_p(stamps.data_ptr())) == 0
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    if wave:
        assert plan.wave_encode, "the plan does not qualify for ga_demo_encode_sym"
        L.ga_demo_stamps_set_wave.argtypes = [ctypes.c_void_p]
        assert L.ga_demo_stamps_set_wave(ctypes.c_void_p(stamps.data_ptr())) == 0

    def run():
        if wave:
            rc = L.ga_demo_encode_sym(0, ctypes.c_void_p(plan.desc64.data_ptr()), plan.n64tensors, plan.n64chunks,
                                      ctypes.c_void_p(plan.groups.data_ptr()), plan.ngroups,
                                      ctypes.c_void_p(plan.F64.data_ptr()), ctypes.c_void_p(P.data_ptr()),
                                      ctypes.c_void_p(G.data_ptr()), ctypes.c_void_p(D.data_ptr()), 1, layout.n,
                                      1e-3, 0.999, 1.0, ctypes.c_void_p(pl.data_ptr()), 2 * plan.M, plan.M, s)
        else:
            rc = L.ga_demo_encode(0, ctypes.c_void_p(plan.desc.data_ptr()), plan.ntensors, plan.nchunks,
                                  ctypes.c_void_p(plan.F.data_ptr()), ctypes.c_void_p(plan.B.data_ptr()),
                                  ctypes.c_void_p(P.data_ptr()), ctypes.c_void_p(G.data_ptr()),
                                  ctypes.c_void_p(D.data_ptr()), 1, layout.n, 1e-3, 0.999, 1.0,
                                  ctypes.c_void_p(pl.data_ptr()), 2 * plan.M, plan.M, s)
        assert rc == 0, L.ga_last_error()

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run()
    e1.record()
    torch.cuda.synchronize()
    st = stamps.view(-1, 16).cpu().numpy().astype(np.int64)
    if wave:  # one row per wave: 7 phase sums, [8] all-keys selections, [9] chunks
        st = st[st[:, 9] > 0]
        tot = st[:, :8].sum(axis=1) + st[:, 10:14].sum(axis=1)
        nch = st[:, 9]
        print(f"{model}: {plan.nchunks} chunks over {len(st)} waves, kernel {e0.elapsed_time(e1):.3f} ms "
              f"(stamped build); all-keys selections {st[:, 8].sum()} of {nch.sum()} chunks")
        print(f"cycles per chunk (wave view): median {np.median(tot / nch):.0f}")
        for i, name in enumerate(WAVE_PHASES):
            v = st[:, i] / nch
            print(f"  {name:22s} median {np.median(v):8.0f} cyc/chunk  share {np.median(st[:, i] / tot):6.1%}")
        for i, name in zip(range(10, 14), ["top-k: max/T0/count", "top-k: compaction", "top-k: bitmap ranks",
                                           "top-k: k-th key+ties"]):
            v = st[:, i] / nch
            if v.any():
                print(f"    {name:22s} median {np.median(v):8.0f} cyc/chunk  (part of the phases above)")
        return
    st = st[st[:, 8] > 0]  # workgroups that ran (persistent grid)
    tot = st[:, :6].sum(axis=1)
    nch = st[:, 8]
    print(f"{model}: {plan.nchunks} chunks over {len(st)} workgroups, kernel {e0.elapsed_time(e1):.3f} ms "
          f"(stamped build)")
    print(f"cycles per chunk (workgroup view): median {np.median(tot / nch):.0f}")
    for i, name in enumerate(PHASES):
        v = st[:, i] / nch
        print(f"  {name:22s} median {np.median(v):8.0f} cyc/chunk  share {np.median(st[:, i] / tot):6.1%}")


if __name__ == "__main__":
    main()
