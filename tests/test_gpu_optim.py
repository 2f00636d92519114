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



def _adam_hp(t=1):
    b1, b2, lr, wd = 0.9, 0.999, 1e-3, 1e-2
    return dict(lerp_w=1 - b1, beta2=b2, one_m_beta2=1 - b2, eps=1e-8, wd_factor=1 - lr * wd, l2_wd=0.0,
                step_size=-(lr / (1 - b1 ** t)), bc2_sqrt=(1 - b2 ** t) ** 0.5)


@pytest.mark.parametrize("p,per_row", [(0.005, False), (0.005, True), (0.3, False), (1.0, True)])
def test_adam_select_rows_step_matches_two_launch_step(p, per_row):
    """The replica loop's read-free SPARTA step (ga_sparta_mask_chunks ->
    ga_adam_step_select -> ga_sparta_rows_mean_scatter) against the two-launch
    step (ga_adam_step, then ga_sparta_average_local on the same packed mask):
    parameters, moments and clipped gradients bit-identical, every replica.
    p = 0.3 / 1.0 fill the 256-entry list windows several times per chunk;
    per_row: one launch per replica (ArenaAdam with per-replica moment placement)."""
    from gym_amd import ops
    dev = torch.device("cuda", 0)
    K = 5
    numels = [3 * 4096 + 17, 64 * 700, 1, 4096 * 8 - 3, 999]
    offs, o = [], 0
    for m in numels:
        offs.append(o)
        o += -(-m // 64) * 64
    n = -(-o // 512) * 512
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    P0 = torch.randn(K, n, device=dev, generator=g) * 0.02
    G0 = torch.randn(K, n, device=dev, generator=g) * 1e-2
    M0 = torch.randn(K, n, device=dev, generator=g).abs_() * 1e-3
    V0 = torch.randn(K, n, device=dev, generator=g).abs_() * 1e-6
    for t in (P0, G0, M0, V0):  # the layout's padding stays 0
        pad = torch.ones(n, dtype=torch.bool, device=dev)
        for a, m in zip(offs, numels):
            pad[a:a + m] = False
        t[:, pad] = 0
    table, nb = ops.sparta_bernoulli_table(offs, numels, dev)
    bits = torch.zeros(ops.sparta_mask_words(n), dtype=torch.int64, device=dev)
    ops.sparta_torch_bernoulli(table, nb, p, 1234, 8, 12, bits)
    clip = torch.tensor([0.5, 0.0] * K, device=dev)  # clipped: the grads are written back too
    hp = _adam_hp(3)
    # two launches
    A = [t.clone() for t in (P0, G0, M0, V0)]
    ops.adam_step(*A, clip_coef=clip, **hp)
    ops.sparta_average_local(A[0], n, float(K), mask=bits, layout="rows")
    # read-free step
    B = [t.clone() for t in (P0, G0, M0, V0)]
    from gym_amd.engine import sparta_capacity
    cap = sparta_capacity(n, p) if p < 1 else n
    cb = torch.empty(ops.sparta_chunk_count(n), dtype=torch.int32, device=dev)
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    sv = torch.full((K, cap), float("nan"), device=dev)
    sel = ops.RowsSelect(bits, cb, sv, cap)
    ops.sparta_mask_chunks(bits, n, cb, cap, cnt)
    if per_row:
        for k in range(K):
            ops.adam_step(B[0][k], B[1][k], B[2][k], B[3][k], clip_coef=clip[2 * k:2 * k + 2], select=sel.row(k), **hp)
    else:
        ops.adam_step(*B, clip_coef=clip, select=sel, **hp)
    ops.sparta_rows_mean_scatter(B[0], n, sel, float(K))
    total = int(sum(bin(int(w) & (2**64 - 1)).count("1") for w in bits.cpu().tolist()))
    assert int(cnt[0]) == total and int(cnt[1]) == 0
    assert total > 0
    for a, b in zip(A, B):
        assert torch.equal(a, b)


def test_adam_select_capacity_overflow_is_flagged():
    """More selected elements than the capacity: count[1] = 1 (the engine raises
    on it) and nothing is written past the capacity."""
    from gym_amd import ops
    dev = torch.device("cuda", 0)
    n = 4096 * 4
    bits = torch.full((n // 64,), -1, dtype=torch.int64, device=dev)  # every element selected
    cap = 1000
    cb = torch.empty(ops.sparta_chunk_count(n), dtype=torch.int32, device=dev)
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    sv = torch.zeros(2, cap + 64, device=dev)
    ops.sparta_mask_chunks(bits, n, cb, cap, cnt)
    assert cnt.tolist() == [n, 1]
    P = torch.randn(2, n, device=dev)
    G, M, V = torch.randn_like(P), torch.zeros_like(P), torch.zeros_like(P)
    ops.adam_step(P, G, M, V, select=ops.RowsSelect(bits, cb, sv[:, :cap], cap), **_adam_hp())
    assert torch.equal(sv[:, cap:], torch.zeros(2, 64, device=dev))
    assert torch.equal(sv[:, :cap], P[:, :cap])
