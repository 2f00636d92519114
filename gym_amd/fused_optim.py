"""Inner optimizer on the flat arena.

The reference's strategies run `clip_grad_norm_(model.parameters(), max_norm)`
and `self.optim.step()` with the default inner optimizer torch.optim.AdamW
(exogym/strategy/strategy.py:135-140, diloco.py:52-59,
communicate_optimize_strategy.py:69-74; OptimSpec default optim.py:11).
ArenaAdam is a torch.optim.Optimizer (schedulers such as LambdaLR drive its
param_groups[0]["lr"] as usual) whose step() is ONE fused kernel over the
node's parameter arena (ga_adam_step: read p, g, m, v; write p, m, v) and,
with clipping, one norm reduction (ga_grad_clip_coef) whose coefficient the
step kernel applies on the device -- no host synchronisation.

Exactness: parameters whose .grad is None at step time are skipped, as torch
does (the kernel runs over the contiguous arena ranges that have gradients).
The per-parameter state (exp_avg, exp_avg_sq, step) are views of the flat
state buffers, so state_dict() has torch's layout.
"""
import math

import torch

from . import ops

_UNSUPPORTED = ("amsgrad", "maximize", "capturable", "differentiable")


def fusable(spec_cls, kwargs, arena):
    """True when OptimSpec(spec_cls, **kwargs) can run as ArenaAdam on this arena."""
    if spec_cls not in (torch.optim.AdamW, torch.optim.Adam):
        return False
    if arena is None or arena.grad_flat is None or arena.dtype != torch.float32:
        return False
    kw = dict(kwargs or {})
    if any(kw.get(k) for k in _UNSUPPORTED):
        return False
    if spec_cls is torch.optim.Adam and kw.get("decoupled_weight_decay"):
        return False
    allowed = {"lr", "betas", "eps", "weight_decay", "foreach", "fused"} | set(_UNSUPPORTED)
    if set(kw) - allowed:
        return False
    lr = kw.get("lr", 1e-3)
    return not isinstance(lr, torch.Tensor)


class ArenaAdam(torch.optim.Optimizer):
    def __init__(self, params, arena, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=None, decoupled=True,
                 **ignored):
        if weight_decay is None:
            weight_decay = 1e-2 if decoupled else 0.0  # torch's AdamW / Adam defaults
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        for i, b in enumerate(betas):
            if not 0.0 <= b < 1.0:
                raise ValueError(f"Invalid beta parameter at index {i}: {b}")
        if not 0.0 <= weight_decay:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=None, capturable=False, differentiable=False, fused=None,
                        decoupled_weight_decay=bool(decoupled))
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("ArenaAdam: one parameter group (the node's arena)")
        self.arena = arena
        dev = arena.flat.device
        self.exp_avg = torch.zeros(arena.n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(arena.n, dtype=torch.float32, device=dev)
        self._step_t = torch.tensor(0.0)
        index = {id(p): i for i, p in enumerate(arena.params)}
        self._spans = []  # (param, arena offset, numel) in arena order
        for p in self.param_groups[0]["params"]:
            if id(p) not in index:
                raise ValueError("ArenaAdam: every parameter must live in the arena")
            i = index[id(p)]
            o, n = arena.layout.offsets[i], arena.layout.numels[i]
            self._spans.append((p, o, n))
            self.state[p] = {"step": self._step_t, "exp_avg": self.exp_avg[o:o + n].view(p.shape),
                             "exp_avg_sq": self.exp_avg_sq[o:o + n].view(p.shape)}
        self._spans.sort(key=lambda s: s[1])
        self._partials = ops.sumsq_partials(dev)
        self._clip = torch.ones(2, dtype=torch.float32, device=dev)

    def _ranges(self):
        """Contiguous arena ranges [a, b) of the parameters that have a gradient
        now (a whole-arena range when all do, padding included: it stays 0)."""
        live = [(o, n) for p, o, n in self._spans if p.grad is not None]
        if len(live) == len(self._spans):
            return [(0, self.arena.n)]
        out = []
        for o, n in live:
            if out and o - out[-1][1] < 64:  # adjacent tensors (the alignment gap is zero padding)
                out[-1][1] = o + n
            else:
                out.append([o, o + n])
        return [(a, b) for a, b in out]

    @torch.no_grad()
    def step(self, closure=None, max_norm=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        ranges = self._ranges()
        self.arena.sync_grads()
        g = self.param_groups[0]
        lr, (b1, b2), eps, wd = float(g["lr"]), g["betas"], float(g["eps"]), float(g["weight_decay"])
        decoupled = g["decoupled_weight_decay"]
        self._step_t += 1
        t = float(self._step_t)
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        step_size = -(lr / bc1)
        bc2_sqrt = math.sqrt(bc2)
        wd_factor = (1 - lr * wd) if (decoupled and wd != 0) else 1.0
        l2 = wd if (not decoupled and wd != 0) else 0.0
        clip = None
        if max_norm:
            ops.grad_clip_coef(self.arena.grad_flat, self.arena.n, max_norm, self._partials, self._clip)
            clip = self._clip
        for a, b in ranges:
            ops.adam_step(self.arena.flat[a:b], self.arena.grad_flat[a:b], self.exp_avg[a:b], self.exp_avg_sq[a:b],
                          1 - b1, b2, 1 - b2, eps, wd_factor, l2, step_size, bc2_sqrt, clip)
        return loss
