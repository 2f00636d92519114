"""Fused inner optimizer on the MI355X (ga_adam_step, ga_grad_clip_coef through
the C ABI) against torch.optim.AdamW / Adam + clip_grad_norm_ running on the
same GPU (the reference's inner optimizer).  fp32 tolerance: reordered norm
sums and FMA contraction differ at the ulp level; 1e-5 relative after 5 steps."""
import pytest
import torch

import optim_cases as C

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,cls,kw,max_norm,skip", C.CASES, ids=[c[0] for c in C.CASES])
def test_arena_adam_matches_torch_on_gpu(name, cls, kw, max_norm, skip):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ours, ref = C.run_pair("cuda:0", cls, kw, max_norm=max_norm, skip=skip)
    C.assert_close(ours, ref)


def test_clip_coef_kernel():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gym_amd import ops
    g = torch.randn(1_000_003, device="cuda") * 0.01
    part, out = ops.sumsq_partials(g.device), torch.zeros(2, device="cuda")
    ops.grad_clip_coef(g, g.numel(), 0.5, part, out)
    ref = torch.linalg.vector_norm(g.double()).item()
    assert abs(out[1].item() - ref) <= 1e-5 * ref
    assert abs(out[0].item() - min(1.0, 0.5 / (ref + 1e-6))) <= 1e-5


@pytest.mark.parametrize("K,n,src,clip", [(2, 70_016, "torch", True), (5, 200_000, "bits", False),
                                          (32, 1_000_064, "torch", True), (8, 300_032, "philox", True),
                                          (3, 65_536, "bytes", False), (1, 4096, "torch", False)])
def test_adam_sparta_step_matches_two_launches(K, n, src, clip):
    """The replica loop's fused inner AdamW + SPARTA average (ga_adam_sparta_step)
    against ga_adam_step followed by ga_sparta_average_local on the same [K, ld]
    rows: bit-identical parameters, moments and (clipped) gradients, for every
    mask source (the reference's torch.bernoulli draw in-kernel, packed words,
    a uint8 arena, the Philox stream with a skipped range), K = 1 ... 32,
    per-replica clip coefficients on and off, over two steps."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import numpy as np
    from gym_amd import ops
    from gym_amd.arena import ArenaLayout
    from oracle import sparta as osparta
    dev = torch.device("cuda:0")
    ld = n + 64
    g = torch.Generator(device=dev)
    g.manual_seed(K * 1000 + n % 997)
    P0 = torch.randn(K, ld, device=dev, generator=g) * 0.02
    P0[:, n:] = 0
    G0 = torch.randn(K, ld, device=dev, generator=g) * 1e-2
    G0[:, n:] = 0
    skip = None
    if src == "philox":
        skip = torch.tensor([[4096, 8192]], dtype=torch.int64, device=dev)
    out = {}
    for fused in (True, False):
        P, Gr = P0.clone(), G0.clone()
        M, V = torch.zeros_like(P), torch.zeros_like(P)
        part, coef = ops.sumsq_partials(dev, K), torch.ones(2 * K, device=dev)
        for t in (1, 2):
            kw = dict(p=0.01, seed=77, iteration=t, skip=skip) if src == "philox" else {}
            if src == "torch":
                L = ArenaLayout([(n // 2,), (n - n // 2,)])
                table, _ = ops.sparta_bernoulli_table(L.offsets, L.numels, dev)
                kw["mask"] = ops.TorchDraw(table, 0.01, 1234, 24 * t, 12)
            elif src == "bits":
                m = np.zeros(ld, bool)
                m[:n] = np.random.default_rng(t).random(n) < 0.02
                kw["mask"] = torch.from_numpy(osparta.pack_mask(m).view(np.int64)).to(dev)
            elif src == "bytes":
                m = np.zeros(ld, np.uint8)
                m[:n] = np.random.default_rng(t).random(n) < 0.05
                kw["mask"] = torch.from_numpy(m).to(dev)
            if clip:
                ops.grad_clip_coef(Gr, ld, 0.05, part, coef)
            hp = dict(lerp_w=0.1, beta2=0.999, one_m_beta2=1 - 0.999, eps=1e-8, wd_factor=1 - 1e-3 * 0.01,
                      l2_wd=0.0, step_size=-(1e-3 / (1 - 0.9 ** t)), bc2_sqrt=(1 - 0.999 ** t) ** 0.5)
            c = coef if clip else None
            if fused:
                ops.adam_sparta_step(P, Gr, M, V, divisor=float(K), clip_coef=c, n=ld, **kw, **hp)
            else:
                ops.adam_step(P, Gr, M, V, clip_coef=c, **hp)
                ops.sparta_average_local(P, ld, float(K), layout="rows", **kw)
        torch.cuda.synchronize()
        out[fused] = [x.cpu().numpy() for x in (P, Gr, M, V)]
    for a, b, what in zip(out[True], out[False], ("param", "grad", "exp_avg", "exp_avg_sq")):
        assert np.array_equal(a, b), (what, int((a != b).sum()))
    changed = (out[True][0] != P0.cpu().numpy()).any(axis=0)  # sanity: the average touched something
    assert changed.any()
