"""DiLoCo outer step (oracle; test infrastructure only).

Reference: DiLoCoStrategy.step (exogym/strategy/diloco.py:51-76):
  _average_models (:34-37)      avg = sum_k theta_k / K
  _set_master_grad (:43-45)     g = master - avg
  outer SGD (:26-28, :70)       torch.optim.SGD(lr=0.7, momentum=0.9, nesterov=True),
                                single-tensor path of torch/optim/sgd.py:
                                  g += wd*p; buf = g (first) | buf = mu*buf + (1-damp)*g
                                  g = g + mu*buf (nesterov) | buf;  p -= lr*g
  _synchronize_master_model + _broadcast_model_params (:47-49, :39-41)
                                every node's params = master (GPU semantics; quirk Q1)
The gate: the outer step runs when local_step % H == 0 and local_step > 0, with
local_step counted before Strategy.step increments it (:62).
"""
import numpy as np

from .reduce import mean_reduce


def outer_step(master, mom, node_params, lr=0.7, momentum=0.9, nesterov=True, dampening=0.0,
               weight_decay=0.0, divisor=None):
    """Returns (new_master, new_mom, params_for_every_node).  mom=None means the
    momentum buffer does not exist yet (first outer step).  fp32 arithmetic in
    torch's op order; `a + alpha*b` (torch's add with alpha, a fused multiply-add
    in ATen's vectorised CPU kernel) is evaluated exactly and rounded once."""
    f32 = np.float32
    avg = mean_reduce(node_params, divisor)
    m = np.asarray(master, dtype=f32)
    g = (m - avg).astype(f32)
    if weight_decay != 0.0:
        g = (g.astype(np.float64) + float(f32(weight_decay)) * m.astype(np.float64)).astype(f32)
    new_mom = None
    if momentum != 0.0:
        if mom is None:
            buf = g.copy()
        else:
            t = (np.asarray(mom, dtype=f32) * f32(momentum)).astype(f32)
            buf = (t.astype(np.float64) + float(f32(1.0 - dampening)) * g.astype(np.float64)).astype(f32)
        new_mom = buf
        if nesterov:
            g = (g.astype(np.float64) + float(f32(momentum)) * buf.astype(np.float64)).astype(f32)
        else:
            g = buf
    new_master = (m.astype(np.float64) - float(f32(lr)) * g.astype(np.float64)).astype(f32)
    return new_master, new_mom, new_master.copy()


def is_outer_step(local_step, H):
    """diloco.py:62 gate (local_step before increment)."""
    return local_step % H == 0 and local_step > 0
