"""DiLoCo: local inner optimizer steps, an outer step every H steps.

API of exogym/strategy/diloco.py:14-89 (optim_spec = inner optimizer,
outer_optim_spec default SGD(lr=0.7, nesterov=True, momentum=0.9), H=100;
gradient clipping when "max_norm" is passed; outer step when
local_step % H == 0 and local_step > 0).

The reference's outer step is 148 per-tensor all-reduces, a GPU->CPU copy of
every tensor on rank 0, a CPU SGD step, a CPU->GPU copy and 148 broadcasts.
Here, for an SGD-family outer optimizer, it is ONE fused kernel per node
(ga_diloco_outer: average, pseudo-gradient master - avg, momentum/Nesterov,
master update, parameter write-back) around one reduce-scatter + one
all-gather over RCCL; the master copy and momentum are fp32 and sharded over
the ranks.  Any other outer optimizer class runs torch's optimizer on a GPU
master copy (replicated on every rank) fed by the same averaging kernel.
"""
from typing import Optional, Union

import torch

from .. import ops
from ..engine import DiLoCoOuter
from .optim import OptimSpec, ensure_optim_spec
from .strategy import Strategy, build_inner_optimizer, clip_and_step


def fused_sgd_hparams(spec: OptimSpec):
    """Hyper-parameters for the fused kernel if `spec` is plain torch SGD."""
    if spec.cls is not torch.optim.SGD:
        return None
    kw = dict(spec.kwargs or {})
    if kw.pop("maximize", False):
        return None
    for k in ("foreach", "fused", "differentiable"):
        kw.pop(k, None)
    defaults = torch.optim.SGD([torch.zeros(1, requires_grad=True)]).defaults
    hp = dict(lr=float(kw.pop("lr", defaults["lr"])), momentum=float(kw.pop("momentum", 0.0)),
              dampening=float(kw.pop("dampening", 0.0)), weight_decay=float(kw.pop("weight_decay", 0.0)),
              nesterov=bool(kw.pop("nesterov", False)))
    if kw:
        return None
    if hp["nesterov"] and (hp["momentum"] <= 0 or hp["dampening"] != 0):
        raise ValueError("Nesterov momentum requires a momentum and zero dampening")
    return hp


class DiLoCoStrategy(Strategy):
    def __init__(self, optim_spec: Optional[Union[str, OptimSpec]] = None,
                 outer_optim_spec: Optional[Union[str, OptimSpec]] = None, H: int = 100, **kwargs):
        self.inner_optim_spec = ensure_optim_spec(optim_spec, OptimSpec(torch.optim.AdamW))
        self.outer_optim_spec = ensure_optim_spec(
            outer_optim_spec, OptimSpec(torch.optim.SGD, lr=0.7, nesterov=True, momentum=0.9))
        self.H = H
        super().__init__(**kwargs)

    def _init_node(self, model, rank, num_nodes):
        super()._init_node(model, rank, num_nodes)
        arena = self._bind_arena(model)
        # the reference's master copy is rank 0's initial model (diloco.py:81-82)
        self.coll.broadcast_(arena.flat, 0)
        hp = fused_sgd_hparams(self.outer_optim_spec)
        self.outer_optimizer = None
        if hp is not None:
            self.engine = DiLoCoOuter(self.coll, 1, arena.n, arena.device, arena.dtype, placement=self.placement_opt,
                                      **hp)
            self.engine.init_master(arena.flat)
        else:
            self.engine = None
            self.master = torch.nn.Parameter(arena.flat.detach().float().clone())
            self.outer_optimizer = self.outer_optim_spec.build([self.master])
            self._avg = torch.empty_like(arena.flat)
        self.optim = build_inner_optimizer(self.inner_optim_spec, model, arena, self.placement_opt)
        self._setup_scheduler()

    def _outer_step(self):
        self.arena.check_bound()
        if self.engine is not None:
            self.engine(self.arena.flat.view(1, -1))
            return
        self._avg.copy_(self.arena.flat)
        self.coll.all_reduce_(self._avg)
        ops.replica_mean(self._avg, self._avg, divisor=self.coll.world)
        self.outer_optimizer.zero_grad()
        self.master.grad = self.master.detach() - self._avg.float()
        self.outer_optimizer.step()
        with torch.no_grad():
            self.arena.flat.copy_(self.master)

    def step(self):
        clip_and_step(self, self.kwargs.get("max_norm"))  # diloco.py:52-59
        if self.local_step % self.H == 0 and self.local_step > 0:
            self._outer_step()
        super().step()
