"""Shared cases for the fused inner optimizer tests (CPU stand-ins and GPU):
ArenaAdam vs torch.optim.AdamW / Adam (+ clip_grad_norm_) on the same model,
gradients and steps.  torch's optimizer is the reference's inner optimizer
(exogym/strategy/optim.py:11, strategy.py:135-140)."""
import numpy as np
import torch

SHAPES = [(66, 32), (128,), (96, 64), (3, 7), (10,)]


def make_model(dev, seed=3):
    g = torch.Generator().manual_seed(seed)
    m = torch.nn.Module()
    m.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(*s, generator=g) * 0.02) for s in SHAPES])
    return m.to(dev)


def grads_for(step, seed=7):
    g = torch.Generator().manual_seed(seed + 31 * step)
    return [torch.randn(*s, generator=g) * (0.05 if step % 2 else 0.5) for s in SHAPES]


def run_pair(dev, cls, kw, max_norm=None, steps=5, skip=None):
    """Returns (ours, torch's) parameter lists after `steps` steps; `skip` =
    index of a parameter whose grad is None from step 2 on."""
    from gym_amd.arena import ParamArena
    from gym_amd.fused_optim import ArenaAdam
    a, b = make_model(dev), make_model(dev)
    arena = ParamArena(list(a.parameters()))
    ours = ArenaAdam(a.parameters(), arena, decoupled=cls is torch.optim.AdamW, **kw)
    ref = cls(b.parameters(), **kw)
    for step in range(steps):
        gs = grads_for(step)
        arena.zero_grad()
        for i, (pa, pb, g) in enumerate(zip(a.parameters(), b.parameters(), gs)):
            if skip is not None and i == skip and step >= 2:
                pa.grad = None
                pb.grad = None
                continue
            pa.grad.copy_(g.to(dev)) if pa.grad is not None else setattr(pa, "grad", g.to(dev).clone())
            pb.grad = g.to(dev).clone()
        ours.step(max_norm=max_norm)
        if max_norm:
            torch.nn.utils.clip_grad_norm_([p for p in b.parameters() if p.grad is not None], max_norm)
        ref.step()
    return ([p.detach().cpu().numpy() for p in a.parameters()], [p.detach().cpu().numpy() for p in b.parameters()])


CASES = [
    ("adamw-default", torch.optim.AdamW, {}, None, None),
    ("adamw-wd-lr", torch.optim.AdamW, {"lr": 3e-3, "weight_decay": 0.1, "betas": (0.8, 0.95)}, None, None),
    ("adamw-clip", torch.optim.AdamW, {"lr": 1e-3}, 0.5, None),
    ("adam-l2", torch.optim.Adam, {"lr": 2e-3, "weight_decay": 0.05}, None, None),
    ("adamw-unused-param", torch.optim.AdamW, {"lr": 1e-3}, None, 1),
]


def assert_close(ours, ref, rtol=1e-5, atol=1e-7):
    for x, y in zip(ours, ref):
        np.testing.assert_allclose(x, y, rtol=rtol, atol=atol)
