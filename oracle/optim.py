"""Inner optimizer step (oracle; test infrastructure only).

Reference: the strategies' `clip_grad_norm_(model.parameters(), max_norm)` +
`self.optim.step()` with the default torch.optim.AdamW
(exogym/strategy/strategy.py:135-140, diloco.py:52-59,
communicate_optimize_strategy.py:69-74; OptimSpec default optim.py:11).
The arithmetic lives in torch (third party, torch 2.10 here):
torch/optim/adam.py `_multi_tensor_adam` (AdamW = decoupled weight decay)
and torch/nn/utils/clip_grad.py.  Restated in numpy fp32 in torch's op order;
`a + s*b` forms that ATen evaluates with a fused multiply-add are evaluated
exactly and rounded once.  Pinned against torch.optim.AdamW / clip_grad_norm_
run here (tests/test_oracle_golden.py).
"""
import numpy as np

f32 = np.float32


def _fma(a, b, c):
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(f32)


def clip_coef(grads, max_norm):
    """(coef, total_norm) of clip_grad_norm_ (norm type 2, eps 1e-6, clamped to 1)."""
    total = np.sqrt(sum(float(np.sum(np.asarray(g, np.float64) ** 2)) for g in grads))
    coef = min(1.0, float(f32(max_norm) / (f32(total) + f32(1e-6))))
    return coef, total


def adam_step(p, g, m, v, step, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, decoupled=True,
              clip=None):
    """One Adam(W) step on fp32 arrays; step = the step count after increment.
    Returns (p, g_used, m, v)."""
    b1, b2 = betas
    p, g, m, v = (np.asarray(x, f32).copy() for x in (p, g, m, v))
    if clip is not None and clip < 1.0:
        g = (g * f32(clip)).astype(f32)
    if weight_decay != 0:
        if decoupled:
            p = (p * f32(1 - lr * weight_decay)).astype(f32)
        else:
            g = _fma(f32(weight_decay), p, g)
    w = f32(1 - b1)
    m = _fma(w, (g - m).astype(f32), m)  # lerp, weight < 0.5
    v = (v * f32(b2)).astype(f32)
    v = _fma((f32(1 - b2) * g).astype(f32), g, v)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    step_size = f32(-(lr / bc1))
    denom = ((np.sqrt(v).astype(f32) / f32(bc2 ** 0.5)).astype(f32) + f32(eps)).astype(f32)
    p = _fma(step_size, (m / denom).astype(f32), p)
    return p, g, m, v
