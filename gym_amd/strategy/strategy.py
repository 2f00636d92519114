"""Strategy base class and SimpleReduceStrategy on a flat parameter arena.

API kept from exogym/strategy/strategy.py:18-142 (constructor kwargs become
attributes, lr scheduler "lambda_cosine", lr_callbacks, max_steps, step(),
zero_grad(), __config__()).  What changes underneath:

- `_init_node` binds the model's parameters and gradients to one flat arena
  per node (gym_amd.arena.ParamArena) on the node's MI355X;
- SimpleReduce's per-parameter `all_reduce(grad); grad.div_(K)` loop
  (strategy.py:130-133) becomes ONE RCCL all-reduce over the gradient arena
  plus ONE division kernel (ga_replica_mean);
- gradient clipping + the default AdamW step run over the arena as one norm
  reduction and one fused kernel (gym_amd.fused_optim.ArenaAdam);
- zero_grad() zeroes the gradient arena in place (grads stay bound to it)
  instead of setting them to None.
"""
import math
from abc import ABC, abstractmethod
from typing import Any, Dict

import torch
from torch.optim.lr_scheduler import LambdaLR

from ..arena import ParamArena
from ..comm import Collective
from ..engine import MeanReduce
from ..utils import LogModule
from .optim import OptimSpec, ensure_optim_spec


def require_gpu(device):
    """gym_amd's step kernels run on the GPU only; a CPU model is an error, not
    a silent fallback."""
    if torch.device(device).type != "cuda":
        raise RuntimeError(f"gym_amd strategies run on MI355X GPUs; the model is on {device}. "
                           "Move it to a cuda device (one process per GPU).")


def build_inner_optimizer(spec, model, arena, placement=True):
    """The node's inner optimizer: torch's AdamW/Adam become ArenaAdam (one fused
    kernel over the arena per step, gym_amd.fused_optim); any other OptimSpec is
    built as in the reference (OptimSpec.build, optim.py:38-39).  GA_FUSED_OPTIM=0
    keeps torch's optimizer."""
    import os
    from ..fused_optim import ArenaAdam, fusable
    if os.environ.get("GA_FUSED_OPTIM", "1") != "0" and fusable(spec.cls, spec.kwargs, arena):
        kw = {k: v for k, v in (spec.kwargs or {}).items() if k in ("lr", "betas", "eps", "weight_decay")}
        return ArenaAdam(model.parameters(), arena, decoupled=spec.cls is torch.optim.AdamW, placement=placement, **kw)
    return spec.build(model)


def clip_and_step(strategy, max_norm):
    """clip_grad_norm_(max_norm) (if set) then the inner optimizer step; fused
    into the ArenaAdam step (norm reduction + device-side coefficient)."""
    from ..fused_optim import ArenaAdam
    if isinstance(strategy.optim, ArenaAdam):
        strategy.optim.step(max_norm=max_norm or None)
        return
    if max_norm:
        strategy.arena.sync_grads()
        clip_arena_grad_norm_(strategy.arena.grad_flat, max_norm)
    strategy.optim.step()


def clip_arena_grad_norm_(grad_flat, max_norm):
    """clip_grad_norm_ over the whole gradient arena (the padding between
    tensors is zero, so the arena norm is the global norm).  Same rule as
    torch.nn.utils.clip_grad_norm_: scale by max_norm / (norm + 1e-6) if < 1."""
    total = torch.linalg.vector_norm(grad_flat.float(), 2.0)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    grad_flat.mul_(coef.to(grad_flat.dtype))
    return total


class Strategy(ABC, LogModule):
    def __init__(self, lr_scheduler: str = None, lr_scheduler_kwargs: Dict[str, Any] = None, **kwargs: Any):
        self.lr_scheduler = lr_scheduler
        self.lr_scheduler_kwargs = lr_scheduler_kwargs
        self.kwargs = kwargs
        for k, v in kwargs.items():
            setattr(self, k, v)  # unknown kwargs are kept, as in the reference
        self.scheduler = None
        self.lr_callbacks = []
        self.max_steps = 1  # read by lr_lambda before TrainNode sets it

    # -- node setup -------------------------------------------------------------
    def _init_node(self, model, rank, num_nodes):
        self.model = model
        self.rank = rank
        self.num_nodes = num_nodes
        self.local_step = 0

    def _bind_arena(self, model, with_grad=True):
        """One flat arena for this node's parameters (and gradients)."""
        params = list(model.parameters())
        require_gpu(params[0].device)
        self.coll = Collective()
        if self.coll.world not in (1, self.num_nodes):
            raise RuntimeError(f"process group has {self.coll.world} ranks but num_nodes={self.num_nodes}: "
                               "gym_amd runs one simulated node per process")
        self.arena = ParamArena(params, world=self.coll.world, with_grad=with_grad)
        return self.arena

    # -- per step ---------------------------------------------------------------
    @abstractmethod
    def step(self):
        self.nbytes = 0
        if self.scheduler is not None:
            self.scheduler.step()
            if self.rank == 0:
                for cb in self.lr_callbacks:
                    cb(self.scheduler.get_last_lr()[0])
        self.local_step += 1

    def finish(self):
        """End of training (called by TrainNode.train after the last step):
        surface any deferred device-side error of the step kernels (SPARTA's
        capacity flag is read back asynchronously)."""

    def zero_grad(self):
        arena = getattr(self, "arena", None)
        if arena is not None and arena.grad_flat is not None:
            arena.zero_grad()
        else:
            self.optim.zero_grad()

    def _setup_scheduler(self):
        kw = self.lr_scheduler_kwargs

        def lr_lambda(step):
            warmup = kw.get("warmup_steps", 1)
            max_steps = min(kw["max_steps"], self.max_steps) if "max_steps" in kw else self.max_steps
            if step < warmup:
                return float(step) / float(max(warmup, 1))
            if kw.get("cosine_anneal", False):
                floor = 0.1
                progress = (step - warmup) / float(max(1, max_steps - warmup))
                return (1 - floor) * 0.5 * (1.0 + math.cos(math.pi * progress)) + floor
            return 1.0

        if self.lr_scheduler == "lambda_cosine":
            self.scheduler = LambdaLR(self.optim, lr_lambda)
        elif self.lr_scheduler is not None:
            self.scheduler = self.lr_scheduler(self.optim, **(kw or {}))
        else:
            self.scheduler = None

    @property
    def placement_opt(self):
        """The `placement` kwarg (default True): False keeps every buffer of the
        step where it was allocated -- no probe launches, no relocation
        (gym_amd.placement.policy)."""
        return self.kwargs.get("placement", True)

    def placement_records(self):
        """What each placement-capable part of this node's step decided: probe
        times and the chosen candidate, or why it was skipped (None: not yet
        run or not applicable)."""
        out = {}
        for name in ("engine", "optim"):
            rec = getattr(getattr(self, name, None), "placement", None)
            if rec is not None and not isinstance(rec, bool):
                out[name] = rec
        return out

    def __config__(self):
        cfg = super().__config__(["iteration", "local_step", "lr_callbacks", "model", "optim", "scheduler",
                                  "arena", "coll", "engine"])
        cfg["strategy"] = self.__class__.__name__
        cfg["placement"] = {"enabled": self.placement_opt is not False, "records": self.placement_records()}
        return cfg


class SimpleReduceStrategy(Strategy):
    """DDP-like: average the gradients over all nodes, then the optimizer step
    (strategy.py:114-142)."""

    def __init__(self, optim_spec=None, max_norm=None, **kwargs):
        super().__init__(**kwargs)
        self.optim_spec = ensure_optim_spec(optim_spec) or OptimSpec(torch.optim.AdamW)
        self.max_norm = max_norm

    def _init_node(self, model, rank, num_nodes):
        super()._init_node(model, rank, num_nodes)
        arena = self._bind_arena(model)
        self.engine = MeanReduce(self.coll, 1, arena.n, arena.device, arena.dtype)
        self.optim = build_inner_optimizer(self.optim_spec, model, arena, self.placement_opt)
        self._setup_scheduler()

    def step(self):
        self.arena.sync_grads()
        self.engine(self.arena.grad_flat.view(1, -1))
        clip_and_step(self, self.max_norm)
        super().step()
