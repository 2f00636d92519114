"""Parity at the sizes BASELINE.json names (GPT-2 124M / 350M arenas), through
properties that do not need the oracle to process the whole arena:
  - DiLoCo, 8 nodes on one GPU, two outer steps: every replica equals the master
    afterwards; sampled elements match the oracle's outer step (elementwise op).
  - SPARTA, 32 nodes (configs[3]), p = 0.005: the selected index list equals the oracle's
    Philox draw over all 124M elements (bit-exact), and in sampled windows the
    selected elements hold the ascending-replica fp32 mean, the rest untouched.
  - DeMo, GPT-2 350M, chunk 64 / top-k 32: in sampled chunks of every tensor
    kind the payload is the oracle's top-k (where the k-th magnitude is not
    tied), the residual delta matches, and the decode's sign step matches.
Tolerances as in test_gpu_kernels.py (bit-exact for indices and same-order
fp32 sums; 1e-6 relative for reordered fp32)."""
import copy

import numpy as np
import pytest
import torch

from oracle import demo as odemo
from oracle import diloco as odiloco
from oracle import sparta as osparta
import demo_checks

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gym_amd import _lib
    _lib.lib()


def _arena(model, K, seed):
    from gym_amd.arena import ArenaLayout
    from gym_amd.shapes import MODELS
    L = ArenaLayout(MODELS[model]())
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    x = torch.randn(K, L.n, device=DEV, generator=g)
    return L, x


def test_diloco_gpt2_124m_8_nodes_two_outer_steps():
    from gym_amd.engine import DiLoCoOuter
    from gym_amd.comm import Collective
    K = 8
    L, x = _arena("gpt2-124m", K, 1)
    x.mul_(1e-3).add_(torch.randn(L.n, device=DEV) * 0.02)
    eng = DiLoCoOuter(Collective(), K, L.n, x.device, torch.float32)
    eng.init_master(x[0])
    rng = np.random.default_rng(0)
    sample = np.sort(rng.choice(L.n, 200_000, replace=False))
    si = torch.as_tensor(sample, device=DEV)
    master = x[0, si].double().cpu().numpy().astype(np.float32)
    mom = None
    for step in range(2):
        reps = x[:, si].cpu().numpy()
        eng(x)
        master, mom, _ = odiloco.outer_step(master, mom, list(reps))
        torch.cuda.synchronize()
        for k in range(1, K):  # every node holds the new master
            assert torch.equal(x[k], x[0])
        np.testing.assert_allclose(x[0, si].cpu().numpy(), master, rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(eng.master[si].cpu().numpy(), master, rtol=1e-6, atol=1e-9)
        # next outer step from drifted nodes
        x.add_(torch.randn(K, L.n, device=DEV) * 1e-3)


def test_sparta_gpt2_124m_32_nodes_full_index_list():
    """configs[3]: SPARTA p=0.005 over 32 simulated GPT-2 124M nodes on one GPU
    (a [32, N] replica set, 15.9 GB)."""
    from gym_amd import ops
    from gym_amd.engine import sparta_capacity
    K, p, seed, it = 32, 0.005, 42, 3
    L, x = _arena("gpt2-124m", K, 2)
    n = L.n
    rng = np.random.default_rng(1)
    starts = rng.integers(0, n - 50_000, 6)
    before = [x[:, s0:s0 + 50_000].cpu().numpy() for s0 in starts]
    cap = sparta_capacity(n, p)
    idx = torch.empty(cap, dtype=torch.int32, device=DEV)
    vals = torch.empty(cap, device=DEV)
    count = torch.zeros(2, dtype=torch.int64, device=DEV)
    work = ops.sparta_workspace(n, DEV)
    ops.sparta_average_local(x, n, float(K), seed=seed, iteration=it, p=p, idx=idx, vals=vals, cap=cap,
                             count=count, work=work)
    c = count.cpu().numpy()
    assert c[1] == 0
    got = idx[: int(c[0])].cpu().numpy().astype(np.int64)
    # the whole Philox draw, 1M elements at a time
    want, step = [], 1 << 20
    for s0 in range(0, n, step):
        m = osparta.philox_mask(min(step, n - s0), seed, it, p, start=s0)
        want.append(np.flatnonzero(m) + s0)
    want = np.concatenate(want)
    assert len(got) == len(want) and np.array_equal(got, want)
    for s0, b in zip(starts, before):
        mask = osparta.philox_mask(50_000, seed, it, p, start=int(s0))
        exp = osparta.sparse_average(list(b), mask, divisor=K)
        after = x[:, s0:s0 + 50_000].cpu().numpy()
        for k in range(K):
            assert np.array_equal(after[k], exp[k])


def test_simple_reduce_char_gpt_8_nodes_bit_exact():
    """configs[1]: the char-level GPT-2 (gpt2_small, vocab 66: 932,864 parameters
    in 52 tensors) under SimpleReduceStrategy with 8 nodes, hosted as batched
    replicas of one process (gym_amd.replica): after the step every node's
    gradient is the oracle's ascending fp32 sum / 8, bit for bit."""
    from gym_amd.replica import ReplicaRunner
    from gym_amd.shapes import MODELS
    from gym_amd.strategy import OptimSpec, SimpleReduceStrategy
    from oracle.reduce import mean_reduce
    from strategy_scenarios import ShapeModel
    shapes = MODELS["gpt2-char"]()
    assert len(shapes) == 52
    models = [ShapeModel(shapes, seed=9).to(DEV) for _ in range(8)]
    assert sum(p.numel() for p in models[0].parameters()) == 932_864
    runner = ReplicaRunner(SimpleReduceStrategy(optim_spec=OptimSpec(torch.optim.SGD, lr=0.0)), models, rank=0,
                           num_nodes=8)
    runner.zero_grad()
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    grads = torch.randn(8, runner.ra.ld, device=DEV, generator=g) * 1e-3
    for k, m in enumerate(models):
        with torch.no_grad():
            for prm, v in zip(m.parameters(), runner.ra.layout.views(grads[k])):
                prm.grad.copy_(v)
    want_in = [np.concatenate([prm.grad.detach().cpu().numpy().ravel() for prm in m.parameters()]) for m in models]
    runner.step()
    want = mean_reduce(want_in)
    for k, m in enumerate(models):
        got = np.concatenate([prm.grad.detach().cpu().numpy().ravel() for prm in m.parameters()])
        assert np.array_equal(got, want), k


def test_demo_gpt2_350m_sampled_chunks():
    from gym_amd import ops
    from gym_amd.demo_codec import DemoPlan
    lr, decay = 1e-3, 0.999
    L, gx = _arena("gpt2-350m", 1, 3)
    plan = DemoPlan(L, chunk=64, topk=32)
    assert plan.wave_encode
    G = gx.mul_(1e-2)
    P = torch.randn(1, L.n, device=DEV) * 0.02
    D = torch.zeros(1, L.n, device=DEV)
    G0, P0 = G.cpu().numpy()[0], P.cpu().numpy()[0]
    payload = torch.zeros(1, 2 * plan.M, dtype=torch.int32, device=DEV)
    ops.demo_encode(plan, P, G, D, payload, lr, decay, 1.0)
    ops.demo_decode(plan, payload, P, G, lr)
    torch.cuda.synchronize()
    pl = payload.cpu().numpy()[0]
    gidx, gval = pl[: plan.M], pl[plan.M: 2 * plan.M].view(np.float32)
    gD, gP, gS = D.cpu().numpy()[0], P.cpu().numpy()[0], G.cpu().numpy()[0]
    rng = np.random.default_rng(2)
    e0 = 0
    checked = 0
    kinds = set()
    tally = demo_checks.SignTally()
    for ti, (shape, off, nel) in enumerate(zip(L.shapes, L.offsets, L.numels)):
        ne = plan.entries_per_tensor[ti]
        R, C, n1, n2 = odemo.tensor_view(shape, 64)
        kind = (len(shape), shape[-1])
        if kind in kinds and ti not in (0, len(L.shapes) - 1):
            e0 += ne
            continue
        kinds.add(kind)
        kk = max(1, min(32, n1 * n2))
        gy, gxc = R // n1, C // n2
        x2 = (np.float32(lr) * G0[off:off + nel]).reshape(R, C)  # delta = 0: x = RN(lr * g)
        for cidx in rng.choice(gy * gxc, min(256, gy * gxc), replace=False):
            y, xx = divmod(int(cidx), gxc)
            xc = x2[y * n1:(y + 1) * n1, xx * n2:(xx + 1) * n2]
            Y = odemo.encode(xc, (n1, n2), 64)
            oidx, oval = odemo.topk_chunks(Y, 32)
            margin = odemo.kth_margin(Y, 32)[0]
            scale = np.abs(oval).max()
            s = e0 + int(cidx) * kk
            dchunk = gD[off:off + nel].reshape(R, C)[y * n1:(y + 1) * n1, xx * n2:(xx + 1) * n2]
            if margin > 1e-5 * scale:
                assert np.array_equal(gidx[s:s + kk], oidx.reshape(-1)), (shape, y, xx)
                np.testing.assert_allclose(gval[s:s + kk], oval.reshape(-1), rtol=0, atol=1e-5 * scale)
                Ym = np.zeros(n1 * n2)
                Ym[oidx.reshape(-1)] = oval.reshape(-1)
                R_ = odemo.decode(Ym.reshape(1, 1, n1, n2), (n1, n2), 64)
                np.testing.assert_allclose(dchunk, xc - R_, rtol=0, atol=1e-6 * np.abs(xc).max())
                # decode of the own payload: p -= lr * sign(IDCT(top-k)), grad = the sign
                sg = np.sign(R_)
                gs = gS[off:off + nel].reshape(R, C)[y * n1:(y + 1) * n1, xx * n2:(xx + 1) * n2]
                tally.check(gs, sg, np.abs(R_) > 1e-5 * np.abs(R_).max(), what=f"{shape} chunk {y},{xx}")
                ok = gs == sg
                p0 = P0[off:off + nel].reshape(R, C)[y * n1:(y + 1) * n1, xx * n2:(xx + 1) * n2]
                pg = gP[off:off + nel].reshape(R, C)[y * n1:(y + 1) * n1, xx * n2:(xx + 1) * n2]
                np.testing.assert_allclose(pg[ok], (p0 - np.float32(lr) * sg)[ok], rtol=0, atol=1e-7)
                checked += 1
        e0 += ne
    assert checked > 500
    tally.done()


def test_demo_gpt2_350m_whole_arena_fp64():
    """configs[4], ONE node, EVERY chunk of GPT-2 350M (86.7k 64x64 chunks and the
    1x64 rows): the codec kernels against the oracle's arithmetic in float64,
    evaluated on the GPU (oracle.demo's DCT-II bases, Y = F1^T X F2 per chunk,
    top-k by |y| with the lowest index winning ties, the residual X - IDCT(top-k),
    the decode's sign(IDCT(top-k)) and p - lr * sign; demo.py:159-209, 315-352).
    Where the k-th magnitude is firm (k-th minus (k+1)-th > 1e-5 of the chunk's
    largest): the index set exact, the values within 1e-5 of the largest, the
    residual within 1e-6 of the chunk's largest input; every decided sign exact.
    At least 99.5% of the chunks must be firm."""
    from gym_amd import ops
    from gym_amd.demo_codec import DemoPlan
    lr, decay = 1e-3, 0.999
    L, gx = _arena("gpt2-350m", 1, 21)
    plan = DemoPlan(L, chunk=64, topk=32)
    assert plan.wave_encode
    G = gx.mul_(1e-2)
    X32 = G * torch.tensor(lr, dtype=torch.float32, device=DEV)  # delta = 0: x = RN(lr * g), as the kernel
    P = torch.randn(1, L.n, device=DEV) * 0.02
    P0 = P.clone()
    D = torch.zeros(1, L.n, device=DEV)
    payload = torch.zeros(1, 2 * plan.M, dtype=torch.int32, device=DEV)
    ops.demo_encode(plan, P, G, D, payload, lr, decay, 1.0)
    Gout = torch.zeros(1, L.n, device=DEV)
    ops.demo_decode(plan, payload, P, Gout, lr)
    torch.cuda.synchronize()
    gidx = payload[0, :plan.M]
    gval = payload[0, plan.M:2 * plan.M].view(torch.float32)
    f64 = torch.float64
    bases = {}

    def basis(n):
        if n not in bases:
            bases[n] = torch.as_tensor(odemo.dct_basis(n), dtype=f64, device=DEV)
        return bases[n]

    def chunked(v, R, C, n1, n2):  # [gy * gx, n1, n2]
        return v.reshape(R // n1, n1, C // n2, n2).permute(0, 2, 1, 3).reshape(-1, n1, n2)

    e0, chunks, firm_chunks = 0, 0, 0
    dec_firm = dec_total = 0
    for ti, (shape, off, nel) in enumerate(zip(L.shapes, L.offsets, L.numels)):
        ne = plan.entries_per_tensor[ti]
        R, C, n1, n2 = odemo.tensor_view(shape, 64)
        kk = max(1, min(32, n1 * n2))
        x = chunked(X32[0, off:off + nel], R, C, n1, n2).to(f64)
        F1, F2 = basis(n1), basis(n2)
        Y = torch.einsum("chw,hb,wd->cbd", x, F1, F2).reshape(x.shape[0], n1 * n2)
        a, order = torch.sort(Y.abs(), dim=1, descending=True, stable=True)
        scale = a[:, 0]
        firm = (a[:, kk - 1] - a[:, kk] > 1e-5 * scale) if kk < n1 * n2 else torch.ones_like(scale, dtype=torch.bool)
        oidx = torch.sort(order[:, :kk], dim=1).values
        oval = torch.gather(Y, 1, oidx)
        nch = x.shape[0]
        gi = gidx[e0:e0 + nch * kk].reshape(nch, kk).long()
        gv = gval[e0:e0 + nch * kk].reshape(nch, kk).to(f64)
        bad = firm & (gi != oidx).any(dim=1)
        assert not bad.any(), (shape, int(bad.sum()), int(bad.nonzero()[0]))
        dv = ((gv - oval).abs() > 1e-5 * scale[:, None]).any(dim=1) & firm
        assert not dv.any(), (shape, int(dv.sum()))
        # the residual delta = x - IDCT(top-k) and the decode of this payload
        Ym = torch.zeros_like(Y).scatter_(1, oidx, oval).reshape(nch, n1, n2)
        Rk = torch.einsum("cbd,hb,wd->chw", Ym, F1, F2)  # IDCT: B = F^T
        dch = chunked(D[0, off:off + nel], R, C, n1, n2).to(f64)
        xmax = x.abs().reshape(nch, -1).amax(dim=1)
        dd = ((dch - (x - Rk)).abs().reshape(nch, -1).amax(dim=1) > 1e-6 * xmax) & firm
        assert not dd.any(), (shape, int(dd.sum()))
        sg = torch.sign(Rk)
        decided = (Rk.abs() > 1e-5 * Rk.abs().reshape(nch, -1).amax(dim=1)[:, None, None]) & firm[:, None, None]
        gs = chunked(Gout[0, off:off + nel], R, C, n1, n2).to(f64)
        assert not ((gs != sg) & decided).any(), (shape, int(((gs != sg) & decided).sum()))
        pg = chunked(P[0, off:off + nel], R, C, n1, n2)
        p0 = chunked(P0[0, off:off + nel], R, C, n1, n2)
        want_p = p0 - torch.tensor(lr, dtype=torch.float32, device=DEV) * sg.float()
        assert not (((pg - want_p).abs() > 1e-7) & decided).any(), shape
        chunks += nch
        firm_chunks += int(firm.sum())
        dec_firm += int(decided.sum())
        dec_total += decided.numel()
        e0 += ne
    assert e0 == plan.M and chunks > 86000, (e0, plan.M, chunks)
    assert firm_chunks >= 0.995 * chunks, (firm_chunks, chunks)
    assert dec_firm >= 0.95 * dec_total, (dec_firm, dec_total)


def test_demo_gpt2_350m_four_nodes_whole_arena_fp64():
    """configs[4] as four nodes run it, EVERY chunk of GPT-2 350M: each node
    encodes its OWN gradient, the four payloads are decoded in node order on the
    shared parameters.  Against float64 on the GPU: each node's index set where
    its k-th magnitude is firm; the decoded sign -- the gathered entries'
    scatter-mean (demo.py:331-352) -> IDCT -> sign -- exact wherever decided,
    with p = p0 - lr * sign there (the sampled oracle test above, whole-arena)."""
    from gym_amd import ops
    from gym_amd.demo_codec import DemoPlan
    lr, decay, S = 1e-3, 0.999, 4
    L, G = _arena("gpt2-350m", S, 23)
    plan = DemoPlan(L, chunk=64, topk=32)
    G.mul_(1e-2)
    X32 = G * torch.tensor(lr, dtype=torch.float32, device=DEV)
    P = torch.randn(1, L.n, device=DEV) * 0.02
    P0 = P.clone()
    D = torch.zeros(S, L.n, device=DEV)
    payload = torch.zeros(S, 2 * plan.M, dtype=torch.int32, device=DEV)
    for k in range(S):
        ops.demo_encode(plan, P, G[k:k + 1], D[k:k + 1], payload[k:k + 1], lr, decay, 1.0)
    Gout = torch.zeros(1, L.n, device=DEV)
    ops.demo_decode(plan, payload, P, Gout, lr)
    torch.cuda.synchronize()
    f64 = torch.float64
    gidx = payload[:, :plan.M].long()
    gval = payload[:, plan.M:2 * plan.M].contiguous().view(torch.float32).to(f64)

    def chunked(v, R, C, n1, n2):
        return v.reshape(R // n1, n1, C // n2, n2).permute(0, 2, 1, 3).reshape(-1, n1, n2)

    e0, chunks, firm_sets, sets = 0, 0, 0, 0
    dec_firm = dec_total = 0
    for ti, (shape, off, nel) in enumerate(zip(L.shapes, L.offsets, L.numels)):
        ne = plan.entries_per_tensor[ti]
        R, C, n1, n2 = odemo.tensor_view(shape, 64)
        kk = max(1, min(32, n1 * n2))
        F1 = torch.as_tensor(odemo.dct_basis(n1), dtype=f64, device=DEV)
        F2 = torch.as_tensor(odemo.dct_basis(n2), dtype=f64, device=DEV)
        nch = (R // n1) * (C // n2)
        sums = torch.zeros(nch, n1 * n2, dtype=f64, device=DEV)
        hits = torch.zeros(nch, n1 * n2, dtype=f64, device=DEV)
        for k in range(S):  # each node's own top-k set, where it is decided
            x = chunked(X32[k, off:off + nel], R, C, n1, n2).to(f64)
            Y = torch.einsum("chw,hb,wd->cbd", x, F1, F2).reshape(nch, n1 * n2)
            a, order = torch.sort(Y.abs(), dim=1, descending=True, stable=True)
            firm = (a[:, kk - 1] - a[:, kk] > 1e-5 * a[:, 0]) if kk < n1 * n2 else torch.ones(nch, dtype=torch.bool,
                                                                                               device=DEV)
            oidx = torch.sort(order[:, :kk], dim=1).values
            gi = gidx[k, e0:e0 + nch * kk].reshape(nch, kk)
            assert not (firm & (gi != oidx).any(dim=1)).any(), (shape, k)
            firm_sets += int(firm.sum())
            sets += nch
            gv = gval[k, e0:e0 + nch * kk].reshape(nch, kk)
            sums.scatter_add_(1, gi, gv)
            hits.scatter_add_(1, gi, torch.ones_like(gv))
        Xm = torch.where(hits > 0, sums / hits.clamp(min=1), torch.zeros_like(sums)).reshape(nch, n1, n2)
        ghat = torch.einsum("cbd,hb,wd->chw", Xm, F1, F2)
        decided = ghat.abs() > 1e-5 * ghat.abs().reshape(nch, -1).amax(dim=1).clamp(min=1e-30)[:, None, None]
        sg = torch.sign(ghat)
        gs = chunked(Gout[0, off:off + nel], R, C, n1, n2).to(f64)
        assert not ((gs != sg) & decided).any(), (shape, int(((gs != sg) & decided).sum()))
        pg = chunked(P[0, off:off + nel], R, C, n1, n2)
        p0 = chunked(P0[0, off:off + nel], R, C, n1, n2)
        want_p = p0 - torch.tensor(lr, dtype=torch.float32, device=DEV) * sg.float()
        assert not (((pg - want_p).abs() > 1e-7) & decided).any(), shape
        chunks += nch
        dec_firm += int(decided.sum())
        dec_total += decided.numel()
        e0 += ne
    assert e0 == plan.M and chunks > 86000
    assert firm_sets >= 0.995 * sets, (firm_sets, sets)
    assert dec_firm >= 0.95 * dec_total, (dec_firm, dec_total)


def _chunks(t2d, R, C, n1, n2, cidx):
    """[len(cidx), n1, n2] chunks (row-major chunk ids) of a [R, C] device view, on the host."""
    gy, gxc = R // n1, C // n2
    ci = torch.as_tensor(np.asarray(cidx), device=t2d.device)
    v = t2d.reshape(gy, n1, gxc, n2).permute(0, 2, 1, 3).reshape(gy * gxc, n1, n2)
    return v.index_select(0, ci).cpu().numpy()


def test_demo_gpt2_350m_four_nodes_multi_source_decode():
    """configs[4] as four nodes run it: every node encodes its OWN gradient, the
    four payloads are gathered in node order and decoded on the shared
    parameters (batch_decompress -> decode -> sign, demo.py:183-206,331-352).
    256 sampled chunks of every tensor kind of GPT-2 350M: each node's index set
    equals the oracle's top-k where the k-th magnitude is firm, and the decoded
    sign -- from the gathered payloads through oracle.demo.scatter_mean and the
    IDCT -- is exact wherever it is decided, with p = p0 - lr * sign there."""
    from gym_amd import ops
    from gym_amd.demo_codec import DemoPlan
    lr, decay, S = 1e-3, 0.999, 4
    L, G = _arena("gpt2-350m", S, 11)
    plan = DemoPlan(L, chunk=64, topk=32)
    assert plan.wave_encode
    G.mul_(1e-2)
    P = torch.randn(1, L.n, device=DEV) * 0.02
    P0 = P.clone()
    D = torch.zeros(S, L.n, device=DEV)
    payload = torch.zeros(S, 2 * plan.M, dtype=torch.int32, device=DEV)
    for k in range(S):  # each node's own encode (its own arena), as on its own GPU
        ops.demo_encode(plan, P, G[k:k + 1], D[k:k + 1], payload[k:k + 1], lr, decay, 1.0)
    Gout = torch.zeros(1, L.n, device=DEV)
    ops.demo_decode(plan, payload, P, Gout, lr)
    torch.cuda.synchronize()
    pl = payload.cpu().numpy()
    gidx, gval = pl[:, :plan.M], pl[:, plan.M:2 * plan.M].view(np.float32)
    rng = np.random.default_rng(4)
    e0, checked, expected, kinds = 0, 0, 0, set()
    tally = demo_checks.SignTally()
    hitters = []
    for ti, (shape, off, nel) in enumerate(zip(L.shapes, L.offsets, L.numels)):
        ne = plan.entries_per_tensor[ti]
        R, C, n1, n2 = odemo.tensor_view(shape, 64)
        kind = (len(shape), shape[-1])
        if kind in kinds and ti not in (0, len(L.shapes) - 1):
            e0 += ne
            continue
        kinds.add(kind)
        kk = max(1, min(32, n1 * n2))
        gy, gxc = R // n1, C // n2
        cidx = np.sort(rng.choice(gy * gxc, min(256, gy * gxc), replace=False))
        expected += len(cidx)
        xs = [np.float32(lr) * _chunks(G[k, off:off + nel], R, C, n1, n2, cidx) for k in range(S)]
        sg_got = _chunks(Gout[0, off:off + nel], R, C, n1, n2, cidx)
        p_got = _chunks(P[0, off:off + nel], R, C, n1, n2, cidx)
        p_0 = _chunks(P0[0, off:off + nel], R, C, n1, n2, cidx)
        for j, c in enumerate(cidx):
            s = e0 + int(c) * kk
            il = [gidx[k, s:s + kk].reshape(1, 1, kk) for k in range(S)]
            vl = [gval[k, s:s + kk].reshape(1, 1, kk) for k in range(S)]
            for k in range(S):  # the node's own top-k set, where it is decided
                Y = odemo.encode(xs[k][j], (n1, n2), 64)
                oidx, _ = odemo.topk_chunks(Y, 32)
                if odemo.kth_margin(Y, 32)[0] > 1e-5 * np.abs(Y).max():
                    assert np.array_equal(il[k].reshape(-1), oidx.reshape(-1)), (shape, int(c), k)
            ghat = odemo.decode(odemo.scatter_mean(il, vl, n1, n2), (n1, n2), 64)
            hitters.append(len(np.unique(np.concatenate([i.reshape(-1) for i in il]))))
            firm = np.abs(ghat) > 1e-5 * max(np.abs(ghat).max(), 1e-30)
            sg = np.sign(ghat)
            tally.check(sg_got[j], sg, firm, what=f"{shape} chunk {int(c)}")
            np.testing.assert_allclose(p_got[j][firm], (p_0[j] - np.float32(lr) * sg)[firm], rtol=0, atol=1e-7)
            checked += 1
        e0 += ne
    assert checked == expected and checked >= 600, (checked, expected)  # 256 per kind (fewer in small 1-D tensors)
    tally.done()
    # the sources really are distinct: a 64x64 chunk of four nodes holds well over 32 distinct entries
    assert np.mean(hitters) > 40, np.mean(hitters)


def test_sparta_reference_draw_gpt2_124m_32_nodes():
    """The drop-in default SPARTA draw at configs[3]'s size: the average kernel
    drawing torch.bernoulli's stream itself (GA_MASK_TORCH) and the fused draw's
    packed mask select the same elements as the 148 per-tensor torch.bernoulli
    calls on this GPU (the reference's draw, sparta.py:80-85), and the two
    averages of the 32 nodes' [n, K] set are bit-identical."""
    from gym_amd import ops
    from gym_amd.arena import ArenaLayout
    from gym_amd.shapes import MODELS
    from gym_amd.strategy.sparta import MaskDraw, RandomIndexSelector, draw_masks
    L = ArenaLayout(MODELS["gpt2-124m"]())
    K, p = 32, 0.005
    params = L.views(torch.empty(L.n, device=DEV))
    sel = RandomIndexSelector(p)
    torch.manual_seed(2024)
    gen0 = torch.cuda.get_rng_state()
    want = torch.zeros(L.n, dtype=torch.bool, device=DEV)  # the reference's draws
    for v, prm in zip(L.views(want), params):
        v.copy_(sel.get_indices(prm, 0))
    after = torch.cuda.get_rng_state()
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    em = torch.randn(L.n, K, device=DEV, generator=g)
    outs = []
    for defer in (True, False):
        torch.cuda.set_rng_state(gen0)
        mask = torch.zeros(L.n, dtype=torch.uint8, device=DEV)
        bits = torch.zeros(ops.sparta_mask_words(L.n), dtype=torch.int64, device=DEV)
        m = draw_masks(sel, params, L.views(mask), set(), 0, MaskDraw(), bits=bits, defer=defer)
        assert torch.equal(torch.cuda.get_rng_state(), after)
        if not defer:
            got = torch.from_numpy(osparta.unpack_mask(m.cpu().numpy(), L.n)).to(DEV)
            assert torch.equal(got, want)
        x = em.clone()
        ops.sparta_average_local(x, L.n, float(K), mask=m, layout="elem")
        outs.append(x)
    assert torch.equal(outs[0], outs[1])
    sel_idx = want.nonzero().view(-1)
    rest = ~want
    assert torch.equal(outs[0][rest], em[rest])  # unselected elements untouched
    i = sel_idx[:: max(1, sel_idx.numel() // 2000)]
    exp = torch.from_numpy(np.stack([osparta.sparse_average(list(em[j].cpu().numpy().reshape(K, 1)),
                                                            np.ones(1, bool))[0] for j in i.tolist()]).reshape(-1))
    assert torch.equal(outs[0][i, 0].cpu(), exp)


def test_candidate_buffer_round_trip_and_diloco_placement():
    """gym_amd.placement: a candidate buffer read as a torch tensor reads back
    what was written and is released; DiLoCoOuter's placement probe leaves the
    replicas untouched and the outer step bit-identical to an engine that kept
    its ordinary allocation."""
    from gym_amd import engine as E
    from gym_amd.comm import Collective
    from gym_amd.placement import DeviceBuffer
    b = DeviceBuffer(3 << 20, DEV)
    t = b.tensor()
    assert t.numel() * 4 >= 3 << 20 and t.is_cuda
    t.copy_(torch.arange(t.numel(), device=DEV, dtype=torch.float32))
    assert torch.equal(t[-5:].cpu(), torch.arange(t.numel() - 5, t.numel(), dtype=torch.float32))
    b.release()
    K = 4
    n = (48 << 20) // 4  # 48 MB per replica: above the placement threshold
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    x0 = torch.randn(K, n, device=DEV, generator=g)
    drift = torch.randn(K, n, device=DEV, generator=g) * 1e-3
    outs = []
    for cands in (64, 1):
        old = E.PLACEMENT_CANDIDATES
        E.PLACEMENT_CANDIDATES = cands
        try:
            x = x0.clone()
            eng = E.DiLoCoOuter(Collective(), K, n, DEV, torch.float32)
            eng.init_master(x[0])
            for step in range(2):
                eng(x)
                x.add_(drift)
            outs.append((x.clone(), eng.master.clone(), eng.mom.clone(), eng.placement))
        finally:
            E.PLACEMENT_CANDIDATES = old
    assert outs[0][3] is not None and outs[0][3]["candidates"] >= 2
    for a, b2 in zip(outs[0][:3], outs[1][:3]):
        assert torch.equal(a, b2)


def test_replica_loop_placements_bit_exact_under_allocation_churn():
    """The replica loop's two physical placements (the fused AdamW moments,
    fused_optim.ArenaAdam._place; the DiLoCo master/momentum, DiLoCoOuter._place)
    against the same loop with placement disabled, with ordinary allocations made,
    written and freed between every step: every replica, the master, the momentum
    and both moments bit-identical after each outer step
    (tools/dbg_product_placement.py; profiles/r04u_vmm_alias.txt: hipMemCreate
    allocations interleaved with ordinary ones were seen corrupted in other
    patterns, so the product's pattern is pinned here)."""
    from gym_amd import engine as E
    from gym_amd import fused_optim as F
    from gym_amd.arena import ReplicaArena
    from gym_amd.comm import Collective
    from gym_amd.fused_optim import ArenaAdam
    torch.manual_seed(0)
    base = torch.nn.Sequential(*[torch.nn.Linear(2048, 2048) for _ in range(3)]).to(DEV)  # 12.6M params

    def run(placed):
        oc, oa = E.PLACEMENT_CANDIDATES, F.PLACEMENT_CANDIDATES
        if not placed:
            E.PLACEMENT_CANDIDATES = F.PLACEMENT_CANDIDATES = 1
        try:
            ra = ReplicaArena([copy.deepcopy(base) for _ in range(4)])
            opt = ArenaAdam(ra.params, ra, lr=1e-3, weight_decay=0.01)
            eng = E.DiLoCoOuter(Collective(), 4, ra.ld, DEV, torch.float32)
            eng.init_master(ra.flat_set[0])
            g = torch.Generator(device=DEV)
            g.manual_seed(5)
            hist = []
            for _ in range(3):
                for _ in range(3):
                    for p in ra.params:
                        p.grad = torch.randn(p.shape, device=DEV, generator=g) * 1e-2
                    opt.step()
                    junk = [torch.empty(1 << 22, device=DEV).fill_(7.0) for _ in range(8)]
                    del junk
                eng(ra.flat_set)
                hist.append([t.clone() for t in (ra.flat_set, eng.master, eng.mom, opt.M, opt.V)])
            return hist, opt._placed is not None, eng.placement
        finally:
            E.PLACEMENT_CANDIDATES, F.PLACEMENT_CANDIDATES = oc, oa
    a, adam_placed, dil = run(True)
    b, _, _ = run(False)
    assert dil is not None
    for sa, sb in zip(a, b):
        for x, y in zip(sa, sb):
            assert torch.equal(x, y)


def test_adam_moments_searched_again_after_relocation():
    """ArenaAdam at K > 1 places each replica's moment rows against that
    replica's parameter / gradient rows; when the parameter set moves (the
    outer step's relocation at step H), the next step searches again, so the
    record describes the rows the step streams with.  The budget holds (the
    record's search_s), and the trajectory is bit-identical to placement off."""
    from gym_amd import fused_optim as F
    from gym_amd.arena import ReplicaArena
    from gym_amd.fused_optim import ArenaAdam
    torch.manual_seed(0)
    base = torch.nn.Sequential(*[torch.nn.Linear(2048, 2048) for _ in range(3)]).to(DEV)

    def run(placed):
        ra = ReplicaArena([copy.deepcopy(base) for _ in range(4)])
        opt = ArenaAdam(ra.params, ra, lr=1e-3, weight_decay=0.01, placement=placed)
        g = torch.Generator(device=DEV)
        g.manual_seed(5)
        recs = []
        for step in range(4):
            if step == 2:
                ra.relocate_params(ra.flat_set.clone())  # as DiLoCoOuter._place_replicas does
            for p in ra.params:
                p.grad = torch.randn(p.shape, device=DEV, generator=g) * 1e-2
            opt.step()
            recs.append(dict(opt.placement or {}))
        return ra.flat_set.clone(), opt.M.clone(), opt.V.clone(), recs
    a = run(True)
    b = run(False)
    for x, y in zip(a[:3], b[:3]):
        assert torch.equal(x, y)
    recs = a[3]
    assert recs[0]["searches"] == 1 and recs[2]["searches"] == 2 and recs[3]["searches"] == 2
    for r in (recs[0], recs[2]):
        assert r["per_replica"] and len(r["probe_ms"]) == 4
        assert r["search_s"] < F.PLACEMENT_ROW_BUDGET_S + 1.0, r["search_s"]


def test_demo_step_placement_leaves_the_step_unchanged():
    """The DeMo optimizer moves its gradient, parameter and delta arenas into the
    device allocations its step runs fastest on, once, after the first step
    (engine.place_demo_step): the probe decodes at lr = 0, encodes into a scratch
    payload and restores P, G and D, so three steps give bit-identical parameters
    to an optimizer that kept its ordinary allocations, and after the move the
    parameters, their .grad (autograd still writes it) and the deltas live in
    the chosen buffers."""
    from gym_amd import engine as E
    from gym_amd.strategy.demo_impl.demo import DeMo
    torch.manual_seed(0)
    base = torch.nn.Sequential(*[torch.nn.Linear(2048, 2048) for _ in range(3)]).to(DEV)  # 12.6M params
    x = torch.randn(64, 2048, device=DEV)
    # fixed per-step gradients (the backward's GEMMs may pick other kernels for other
    # addresses; the step under test is the optimizer's)
    grads = [[torch.randn_like(p) * 1e-2 for p in base.parameters()] for _ in range(3)]
    outs = []
    for min_bytes in (E.DEMO_PLACEMENT_MIN_BYTES, 1 << 62):
        old = E.DEMO_PLACEMENT_MIN_BYTES
        E.DEMO_PLACEMENT_MIN_BYTES = min_bytes
        try:
            model = copy.deepcopy(base)
            opt = DeMo(model.parameters(), lr=1e-3, compression_topk=32, compression_chunk=64)
            for s in range(3):
                opt.zero_grad()
                model(x).square().mean().backward()  # autograd writes .grad (in the moved arena after step 1)
                for p, g in zip(model.parameters(), grads[s]):
                    p.grad.copy_(g)
                opt.step()
            outs.append(([p.detach().clone() for p in model.parameters()], opt))
        finally:
            E.DEMO_PLACEMENT_MIN_BYTES = old
    opt = outs[0][1]
    assert opt.placement is not None and "grad_placed_ms" in opt.placement
    assert outs[1][1].placement == {"placed": False}

    def inside(buf, ptr):
        if buf is None:
            return False
        t = buf.tensor(torch.uint8)
        return t.data_ptr() <= ptr < t.data_ptr() + t.numel()
    if opt._placed is not None:
        bp, bg, bd = opt._placed
        for p in opt.arena.params:
            assert inside(bp, p.data_ptr()) == (bp is not None)
            assert inside(bg, p.grad.data_ptr()) == (bg is not None)
            assert inside(bd, opt.demo_state[p]["delta"].data_ptr()) == (bd is not None)
    for a, b in zip(outs[0][0], outs[1][0]):
        assert torch.equal(a, b)


def test_pipelined_demo_codec_placement_restores_and_matches():
    """PipelinedDeMoCodec.place (the multi-GPU DeMo codec's placement; here over
    two tensor groups without an exchange): P, G, D come back bit-identical, the
    moved buffers hold the same contents, and the next step on them equals the
    step on the ordinary buffers."""
    from gym_amd.arena import ArenaLayout
    from gym_amd.comm import Collective
    from gym_amd.engine import PipelinedDeMoCodec
    shapes = [(2048, 2048), (2048,), (4096, 1024), (1024,)] * 2
    layout = ArenaLayout(shapes)
    g = torch.Generator(device=DEV)
    g.manual_seed(11)
    n = layout.n
    P = (torch.randn(1, n, device=DEV, generator=g) * 0.02)
    G = torch.randn(1, n, device=DEV, generator=g) * 1e-3
    D = torch.zeros(1, n, device=DEV)
    codec = PipelinedDeMoCodec(Collective(), 1, layout, DEV, pieces=2)
    assert len(codec.codecs) == 2
    codec(P, G, D, 1e-3)
    snap = [t.clone() for t in (P, G, D)]
    bufs, moved, rec = codec.place(P, G, D, 1e-3)
    assert rec is not None and len(rec["placed"]) == 3
    for t, s in zip((P, G, D), snap):
        assert torch.equal(t, s)
    for t, s in zip(moved, snap):
        assert torch.equal(t, s)
    G2 = torch.randn(1, n, device=DEV, generator=g) * 1e-3
    P1, G1, D1 = P.clone(), G2.clone(), D.clone()
    Pm, Gm, Dm = moved
    Gm.copy_(G2)
    codec(P1, G1, D1, 1e-3)
    codec(Pm, Gm, Dm, 1e-3)
    for a, b in zip((P1, G1, D1), (Pm, Gm, Dm)):
        assert torch.equal(a, b)


def test_placement_false_bit_identical_without_probe_launches(monkeypatch):
    """placement=False on the DiLoCo engine, the fused AdamW and the DeMo
    optimizer: no probe kernel is launched and no candidate is allocated (the
    probes and the candidate search raise if called), the records say why, and
    the steps are bit-identical to the placed run."""
    from gym_amd import ops, placement
    from gym_amd import engine as E
    from gym_amd.arena import ReplicaArena
    from gym_amd.comm import Collective
    from gym_amd.fused_optim import ArenaAdam
    from gym_amd.strategy.demo_impl.demo import DeMo
    torch.manual_seed(0)
    base = torch.nn.Sequential(*[torch.nn.Linear(2048, 2048) for _ in range(3)]).to(DEV)  # 12.6M params
    x = torch.randn(64, 2048, device=DEV)

    def run(placed):
        ra = ReplicaArena([copy.deepcopy(base) for _ in range(4)])
        opt = ArenaAdam(ra.params, ra, lr=1e-3, weight_decay=0.01, placement=placed)
        eng = E.DiLoCoOuter(Collective(), 4, ra.ld, DEV, torch.float32, placement=placed)
        eng.init_master(ra.flat_set[0])
        eng.relocate_replicas = ra.relocate_params  # as ReplicaRunner: the step may move the replica set
        g = torch.Generator(device=DEV)
        g.manual_seed(5)
        for _ in range(2):
            for _ in range(2):
                for p in ra.params:
                    p.grad = torch.randn(p.shape, device=DEV, generator=g) * 1e-2
                opt.step()
            eng(ra.flat_set)
        model = copy.deepcopy(base)
        dm = DeMo(model.parameters(), lr=1e-3, compression_topk=32, compression_chunk=64, placement=placed)
        for s in range(2):
            dm.zero_grad()
            model(x).square().mean().backward()
            for p in model.parameters():
                p.grad.copy_(torch.randn(p.shape, device=DEV, generator=g) * 1e-2)
            dm.step()
        ra.check_bound()  # every model still reads its row of the (possibly moved) parameter set
        lo, hi = ra.flat_set.data_ptr(), ra.flat_set.data_ptr() + 4 * ra.flat_set.numel()
        assert all(lo <= p.data_ptr() < hi for p in ra.params)
        out = [t.clone() for t in (ra.flat_set, eng.master, eng.mom, opt.M, opt.V)]
        out += [p.detach().clone() for p in model.parameters()]
        return out, (opt.placement, eng.placement, dm.placement)

    placed, recs_on = run(True)
    assert recs_on[1] is not None and recs_on[1].get("candidates", 0) >= 2
    assert recs_on[1]["replica_set"]["candidates"] >= 2, recs_on[1]

    def boom(*a, **k):
        raise AssertionError("placement probe launched with placement=False")
    for name in ("probe_diloco_placement", "probe_adam_placement"):
        monkeypatch.setattr(ops, name, boom)
    monkeypatch.setattr(placement, "choose", boom)
    monkeypatch.setattr(placement, "place_each", boom)
    plain, recs_off = run(False)
    assert all(r == {"placed": False, "why": "placement=False"} for r in recs_off), recs_off
    for a, b in zip(placed, plain):
        assert torch.equal(a, b)
