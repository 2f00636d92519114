"""CPU stand-ins for gym_amd.ops, built on the oracle — TEST INFRASTRUCTURE.

Only the CPU (`-m "not gpu"`) multi-process tests install these, to exercise
the strategies' host orchestration (arenas, collectives, sharding, gating)
over gloo without a GPU.  Each function has the signature and in-place
semantics of its gym_amd.ops counterpart; the GPU tests run the real kernels.
"""
import numpy as np
import torch

from oracle import demo as odemo
from oracle import diloco as odiloco
from oracle import reduce as oreduce
from oracle import sparta as osparta


def _np(t):
    return t.detach().cpu().float().numpy()


def _2d(t):
    return t if t.dim() == 2 else t.view(1, -1)


def replica_mean(src, dst, n=None, divisor=None, rows=None):
    s2, d2 = _2d(src), _2d(dst)
    n = min(s2.shape[1], d2.shape[1]) if n is None else int(n)
    xs = _np(s2)[:, :n]
    rws = [int(r) for r in rows.tolist()] if rows is not None else None
    K = len(rws) if rws is not None else xs.shape[0]
    out = oreduce.mean_reduce(list(xs), divisor=K if divisor is None else divisor, rows=rws)
    o = torch.from_numpy(out).to(d2.dtype)
    for j in range(d2.shape[0]):
        d2[j, :n].copy_(o)


def diloco_outer(src, master, mom, dst, n, divisor, lr, momentum, dampening, weight_decay, nesterov, first_step):
    xs = list(_np(_2d(src))[:, :n])
    prev = None if (first_step or mom is None) else _np(mom)[:n]
    nm, nb, _ = odiloco.outer_step(_np(master)[:n], prev, xs, lr, momentum, nesterov, dampening, weight_decay,
                                   divisor)
    master[:n].copy_(torch.from_numpy(nm))
    if mom is not None and nb is not None:
        mom[:n].copy_(torch.from_numpy(nb))
    if dst is not None:
        d2 = _2d(dst)
        for j in range(d2.shape[0]):
            d2[j, :n].copy_(torch.from_numpy(nm).to(d2.dtype))


def sparta_gap_table(p):
    return [int(v) for v in osparta.gap_table(p)]


def sparta_workspace(n, device):
    return torch.empty(16, dtype=torch.uint8, device=device)


def sparta_mask_words(n):
    return (int(n) + 63) // 64


def sparta_pack_mask(mask, n, bits):
    bits[:sparta_mask_words(n)] = torch.from_numpy(osparta.pack_mask(_np(mask)[:n]))


def _mask_bits(mask, n):
    """bool numpy mask of n elements from a uint8/bool arena or packed int64 words."""
    if mask.dtype == torch.int64:
        return osparta.unpack_mask(mask.cpu().numpy(), n)
    return _np(mask)[:n] != 0


def _skip_list(skip):
    return None if skip is None else [tuple(r) for r in skip.cpu().tolist()]


def _rows_view(t, layout):
    return t.t() if layout == "elem" else _2d(t)


def sparta_select(src, n, cap, idx, vals, count, work, mask=None, seed=0, iteration=0, p=0.0, skip=None,
                  layout="rows"):
    src = _rows_view(src, layout)
    m = _mask_bits(mask, n) if mask is not None else osparta.philox_mask(n, seed, iteration, p,
                                                                         skip=_skip_list(skip))
    sel = np.flatnonzero(m)
    count[0] = len(sel)
    count[1] = int(len(sel) > cap)
    sel = sel[:cap]
    idx[: len(sel)] = torch.from_numpy(sel.astype(np.int32))
    vals[: len(sel)] = torch.from_numpy(oreduce.mean_reduce(list(_np(_2d(src))[:, sel]), divisor=1)).to(vals.dtype)


def sparta_scatter(vals, idx, count, cap, divisor, dst, layout="rows"):
    dst = _rows_view(dst, layout)
    m = min(int(count[0]), int(cap))
    ii = idx[:m].long()
    v = (vals[:m].float() / np.float32(divisor)).to(dst.dtype)
    d2 = _2d(dst)
    for r in range(d2.shape[0]):
        d2[r, ii] = v


def sparta_average_local(reps, n, divisor, mask=None, seed=0, iteration=0, p=0.0, idx=None, vals=None, cap=0,
                         count=None, work=None, skip=None, layout="rows"):
    reps = _rows_view(reps, layout)
    m = _mask_bits(mask, n) if mask is not None else osparta.philox_mask(n, seed, iteration, p,
                                                                         skip=_skip_list(skip))
    r2 = _2d(reps)
    out = osparta.sparse_average(list(_np(r2)[:, :n]), m, divisor)
    for k in range(r2.shape[0]):
        r2[k, :n].copy_(torch.from_numpy(out[k]).to(r2.dtype))


def _tensor_slices(plan):
    e = 0
    for shape, off, nel, ne in zip(plan.layout.shapes, plan.layout.offsets, plan.layout.numels,
                                   plan.entries_per_tensor):
        yield shape, off, nel, e, ne
        e += ne


def demo_encode(plan, param, grad, delta, payload, lr, decay, wd_factor):
    P, G, D, PL = _2d(param), _2d(grad), _2d(delta), _2d(payload)
    M = plan.M
    for k in range(P.shape[0]):
        for shape, off, nel, e0, ne in _tensor_slices(plan):
            if wd_factor != 1.0:
                P[k, off:off + nel] = P[k, off:off + nel] * np.float32(wd_factor)
            d = _np(D[k, off:off + nel]).astype(np.float64)
            if decay != 1.0:
                d = d * decay
            d = d + lr * _np(G[k, off:off + nel])
            Y = odemo.encode(d.reshape(shape), shape, plan.chunk)
            idx, val = odemo.topk_chunks(Y, plan.topk)
            _, _, n1, n2 = odemo.tensor_view(shape, plan.chunk)
            tx = odemo.decode(odemo.scatter_mean([idx], [val], n1, n2), shape, plan.chunk)
            D[k, off:off + nel] = torch.from_numpy((d - tx.reshape(-1)).astype(np.float32))
            PL[k, e0:e0 + ne] = torch.from_numpy(idx.reshape(-1).astype(np.int32))
            PL[k, M + e0:M + e0 + ne] = torch.from_numpy(val.reshape(-1).astype(np.float32).view(np.int32))


def demo_decode(plan, gathered, param, grad, lr):
    P = _2d(param)
    G = _2d(grad) if grad is not None else None
    GA = gathered.view(gathered.shape[0], -1) if gathered.dim() == 2 else gathered.view(1, -1)
    M = plan.M
    for shape, off, nel, e0, ne in _tensor_slices(plan):
        R, C, n1, n2 = odemo.tensor_view(shape, plan.chunk)
        kk = max(1, min(plan.topk, n1 * n2))
        grid = (R // n1, C // n2, kk)
        idxs = [GA[s, e0:e0 + ne].numpy().reshape(grid) for s in range(GA.shape[0])]
        vals = [GA[s, M + e0:M + e0 + ne].numpy().view(np.float32).reshape(grid) for s in range(GA.shape[0])]
        g = odemo.decode(odemo.scatter_mean(idxs, vals, n1, n2), shape, plan.chunk).reshape(-1)
        sgn = torch.from_numpy(np.sign(g).astype(np.float32))
        for k in range(P.shape[0]):
            P[k, off:off + nel] = (P[k, off:off + nel].double() - lr * sgn.double()).float()
            if G is not None:
                G[k, off:off + nel] = sgn


def sumsq_partials(device, K=1):
    return torch.zeros(1024 * K, dtype=torch.float32, device=device)


def grad_clip_coef(grad, n, max_norm, partials, out):
    from oracle import optim as ooptim
    g2 = _2d(grad)
    for k in range(g2.shape[0]):
        c, total = ooptim.clip_coef([_np(g2[k])[:n]], max_norm)
        out[2 * k] = c
        out[2 * k + 1] = total


def adam_step(param, grad, exp_avg, exp_avg_sq, lerp_w, beta2, one_m_beta2, eps, wd_factor, l2_wd, step_size,
              bc2_sqrt, clip_coef=None, n=None):
    """The fused step's arithmetic on CPU tensors (oracle/optim.py order)."""
    P2, G2, M2, V2 = (_2d(t) for t in (param, grad, exp_avg, exp_avg_sq))
    n = P2.shape[1] if n is None else int(n)
    for k in range(P2.shape[0]):
        c = None if clip_coef is None else float(clip_coef[2 * k])
        _adam_one(P2[k, :n], G2[k, :n], M2[k, :n], V2[k, :n], lerp_w, beta2, one_m_beta2, eps, wd_factor, l2_wd,
                  step_size, bc2_sqrt, c)


def _adam_one(param, grad, exp_avg, exp_avg_sq, lerp_w, beta2, one_m_beta2, eps, wd_factor, l2_wd, step_size,
              bc2_sqrt, coef):
    f = np.float32
    p, g, m, v = _np(param).copy(), _np(grad).copy(), _np(exp_avg).copy(), _np(exp_avg_sq).copy()
    if coef is not None and coef < 1.0:
        g = (g * f(coef)).astype(f)
        grad.copy_(torch.from_numpy(g))
    if wd_factor != 1.0:
        p = (p * f(wd_factor)).astype(f)
    if l2_wd != 0.0:
        g = (g.astype(np.float64) + float(f(l2_wd)) * p.astype(np.float64)).astype(f)
    m = (m.astype(np.float64) + float(f(lerp_w)) * (g - m).astype(f).astype(np.float64)).astype(f)
    v = (v * f(beta2)).astype(f)
    v = (v.astype(np.float64) + (f(one_m_beta2) * g).astype(f).astype(np.float64) * g).astype(f)
    denom = ((np.sqrt(v).astype(f) / f(bc2_sqrt)).astype(f) + f(eps)).astype(f)
    p = (p.astype(np.float64) + float(f(step_size)) * (m / denom).astype(f).astype(np.float64)).astype(f)
    param.copy_(torch.from_numpy(p))
    exp_avg.copy_(torch.from_numpy(m))
    exp_avg_sq.copy_(torch.from_numpy(v))


def install(monkeypatch_target_modules=None):
    """Point every gym_amd module that imported `ops` at these stand-ins and
    let CPU models through the GPU check."""
    import gym_amd.engine as engine
    import gym_amd.fused_optim as fused_optim
    import gym_amd.replica as replica
    import gym_amd.strategy.diloco as diloco
    import gym_amd.strategy.federated_averaging as fedavg
    import gym_amd.strategy.strategy as strategy
    import gym_amd.train_node as train_node
    import gym_amd.trainer as trainer
    import sys
    me = sys.modules[__name__]
    for mod in (engine, diloco, fedavg, fused_optim, replica, train_node, trainer):
        mod.ops = me
    strategy.require_gpu = lambda device: None
    import gym_amd.strategy.demo_impl.demo as demo_mod
    demo_mod._REQUIRE_GPU = False
