"""Strategies that interleave a local optimizer step with communication modules.

API of exogym/strategy/communicate_optimize_strategy.py:10-94:
CommunicationModule (communicate(model, rank, num_nodes, local_step),
_init_node(model, rank, num_nodes)) and CommunicateOptimizeStrategy
(communication_modules, inner_optim=None, max_norm=None, **kwargs) whose step
is clip -> inner optimizer step -> modules in order -> base step.  Here the
node's parameters live in a flat arena (bound in _init_node before the modules
and the optimizer are built), which the modules reach via `self.strategy`.
"""
from abc import ABC, abstractmethod
from typing import List, Optional, Union

import torch

from .optim import OptimSpec, ensure_optim_spec
from .strategy import Strategy, build_inner_optimizer, clip_and_step


class CommunicationModule(ABC):
    @abstractmethod
    def __init__(self):
        pass

    @abstractmethod
    def communicate(self, model, rank: int, num_nodes: int, local_step: int) -> None:
        """Communicate the model's state for this step."""

    @abstractmethod
    def _init_node(self, model, rank: int, num_nodes: int) -> None:
        """Per-node setup."""


class CommunicateOptimizeStrategy(Strategy):
    def __init__(self, communication_modules: List[CommunicationModule],
                 inner_optim: Optional[Union[str, OptimSpec]] = None, max_norm: Optional[float] = None, **kwargs):
        super().__init__(**kwargs)
        self.inner_optim_spec = ensure_optim_spec(inner_optim) or OptimSpec(torch.optim.AdamW)
        self.communication_modules = communication_modules
        self.max_norm = max_norm
        for m in self.communication_modules:
            m.strategy = self

    def step(self):
        clip_and_step(self, self.max_norm)
        self._communicate()
        super().step()

    def _communicate(self):
        for m in self.communication_modules:
            m.communicate(self.model, self.rank, self.num_nodes, self.local_step)

    def finish(self):
        for m in self.communication_modules:
            fin = getattr(m, "finish", None)
            if fin is not None:
                fin()

    def _init_node(self, model, rank, num_nodes):
        super()._init_node(model, rank, num_nodes)
        self._bind_arena(model)
        for m in self.communication_modules:
            m._init_node(model, rank, num_nodes)
        self.optim = build_inner_optimizer(self.inner_optim_spec, model, self.arena, self.placement_opt)
        self._setup_scheduler()
