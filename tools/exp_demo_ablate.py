"""Time ga_demo_encode_sym of GPT-2 350M in several builds of libgym_amd.so
(diagnostic: ablated or alternative kernel variants built by hand under
build/abl/).  Every timed encode starts from the same delta: a fresh
N(0, 1e-4) one, or (--evolve N) the delta after N encodes of one fixed grad
(the bench's regime: the removed top-k flattens the spectrum step by step).
With the stamps build (build/libgym_amd_stamps.so) also counts the chunks that
took the all-keys selection (more than 128 candidates).
--codec N instead runs N whole DeMo steps first (encode + decode, the decode
writing sign(g) into the grad buffer, as bench.py's DeMo line does) and times
the encode from that state.
--decode S times ga_demo_decode_sym instead, over S distinct gathered payloads
(S nodes' encodes of independent deltas), parameters restored before each run.
Usage: python tools/exp_demo_ablate.py [--evolve N | --codec N | --decode S] build/abl/lib_*.so"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gym_amd import _lib  # noqa: E402
from gym_amd.arena import ArenaLayout  # noqa: E402
from gym_amd.demo_codec import DemoPlan  # noqa: E402
from gym_amd.shapes import MODELS  # noqa: E402


def bind(path):
    L = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    return L


def main():
    args = sys.argv[1:]
    evolve = codec_steps = 0
    if args and args[0] == "--evolve":
        evolve, args = int(args[1]), args[2:]
    if args and args[0] == "--codec":
        codec_steps, args = int(args[1]), args[2:]
    dec_S = 0
    if args and args[0] == "--decode":
        dec_S, args = int(args[1]), args[2:]
    libs = args
    dev = torch.device("cuda:0")
    layout = ArenaLayout(MODELS["gpt2-350m"]())
    plan = DemoPlan(layout).to(dev)
    assert plan.wave_encode
    torch.manual_seed(0)
    P = torch.randn(layout.n, device=dev) * 0.02
    G = torch.randn(layout.n, device=dev) * 1e-3
    D = torch.randn(layout.n, device=dev) * 1e-4
    pl = torch.zeros(2 * plan.M, dtype=torch.int32, device=dev)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    vp = ctypes.c_void_p
    gathered = None
    if dec_S:  # S nodes' payloads from independent deltas (the default library's encode)
        from gym_amd import ops
        gathered = torch.zeros(dec_S, 2 * plan.M, dtype=torch.int32, device=dev)
        for j in range(dec_S):
            Dj = torch.randn(layout.n, device=dev) * 1e-4
            ops.demo_encode(plan, P.view(1, -1), G.view(1, -1), Dj.view(1, -1), gathered[j:j + 1], 1e-3, 0.999, 1.0)
    fns = {}
    for path in libs:
        L = bind(path)

        def enc(L=L):
            rc = L.ga_demo_encode_sym(0, vp(plan.desc64.data_ptr()), plan.n64tensors, plan.n64chunks,
                                      vp(plan.groups.data_ptr()), plan.ngroups, vp(plan.F64.data_ptr()),
                                      vp(P.data_ptr()), vp(G.data_ptr()), vp(D.data_ptr()), 1, layout.n,
                                      1e-3, 0.999, 1.0, vp(pl.data_ptr()), 2 * plan.M, plan.M, s)
            assert rc == 0

        def dec(L=L):
            rc = L.ga_demo_decode_sym(0, vp(plan.desc64.data_ptr()), plan.n64tensors, plan.n64chunks,
                                      vp(plan.groups.data_ptr()), plan.ngroups, vp(plan.F64.data_ptr()),
                                      vp(gathered.data_ptr()), gathered.stride(0), plan.M, dec_S,
                                      vp(P.data_ptr()), vp(G.data_ptr()), 1, layout.n, 1e-3, s)
            assert rc == 0

        fns[path] = dec if dec_S else enc
    for _ in range(evolve):
        fns[libs[0]]()
    if codec_steps:  # bench.py's regime: P, G as bench_demo builds them, the decode writes sign into G
        from gym_amd.comm import Collective
        from gym_amd.engine import DeMoCodec
        sys.argv = sys.argv[:1]
        import bench
        P.copy_(bench.synth_replicas(layout, 1, 0, dev).data[0, :layout.n])
        G.copy_(bench.synth_replicas(layout, 1, 7, dev).data[0, :layout.n])
        D.zero_()
        codec = DeMoCodec(Collective(), 1, layout, dev)
        for _ in range(codec_steps):
            codec(P.view(1, -1), G.view(1, -1), D.view(1, -1), 1e-3, 0.999, 0.0)
        evolve = f"codec {codec_steps}"
    D0 = D.clone()
    P0 = P.clone()
    st = os.path.join(ROOT, "build", "libgym_amd_stamps.so")
    if os.path.exists(st) and not dec_S:
        S = bind(st)
        S.ga_demo_stamps_set_wave.argtypes = [ctypes.c_void_p]
        stamps = torch.zeros(plan.nchunks * 16, dtype=torch.int64, device=dev)
        assert S.ga_demo_stamps_set_wave(vp(stamps.data_ptr())) == 0
        rc = S.ga_demo_encode_sym(0, vp(plan.desc64.data_ptr()), plan.n64tensors, plan.n64chunks,
                                  vp(plan.groups.data_ptr()), plan.ngroups, vp(plan.F64.data_ptr()),
                                  vp(P.data_ptr()), vp(G.data_ptr()), vp(D.data_ptr()), 1, layout.n,
                                  1e-3, 0.999, 1.0, vp(pl.data_ptr()), 2 * plan.M, plan.M, s)
        assert rc == 0
        st16 = stamps.view(-1, 16)
        print(f"evolve {evolve}: all-keys selections {int(st16[:, 8].sum())} of {int(st16[:, 9].sum())} "
              f"64x64 chunks", flush=True)
        D.copy_(D0)
    times = {p: [] for p in libs}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for f in fns.values():  # warm every build (and the clocks)
        for _ in range(20):
            f()
    torch.cuda.synchronize()
    for _ in range(25):  # interleaved rounds: box clock drift hits every build alike
        for p, f in fns.items():
            (P if dec_S else D).copy_(P0 if dec_S else D0)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            times[p].append(e0.elapsed_time(e1))
    for p in libs:
        t = sorted(times[p])
        print(f"{os.path.basename(p):28s} {'decode S=%d' % dec_S if dec_S else 'encode'} median {t[len(t) // 2]:.4f} ms  min {t[0]:.4f}", flush=True)


if __name__ == "__main__":
    main()
