"""FedAvg: average the parameters across nodes every H steps (optionally
within random islands).

API of exogym/strategy/federated_averaging.py:16-117:
AveragingCommunicator(island_size=None) and FedAvgStrategy(inner_optim=None,
island_size=None, H=1, max_norm=None, **kwargs); communication when
local_step % H == 0 and local_step > 0.

Full averaging is one RCCL all-reduce over the parameter arena plus one
division kernel (the reference: a per-tensor all-reduce + divide).  Island
averaging keeps the reference's algorithm — rank 0 shuffles the ranks with
Python's `random` and broadcasts the permutation (:27-51), every node
all-gathers the parameters and averages its island's members in ascending
rank order (:61-69) — as ONE all-gather of the arena and one
ga_replica_mean over the member rows.
"""
import random
from typing import Optional, Set, Union

import torch
import torch.distributed as dist

from .. import ops
from ..engine import MeanReduce
from .communicate_optimize_strategy import CommunicateOptimizeStrategy, CommunicationModule
from .optim import OptimSpec


class AveragingCommunicator(CommunicationModule):
    def __init__(self, island_size: Optional[int] = None, **kwargs):
        super().__init__(**kwargs)
        self.island_size = island_size
        self._mean = None
        self._gathered = None

    def _select_partners(self, rank: int, num_nodes: int) -> Set[int]:
        ranks = list(range(num_nodes)) if rank == 0 else [None] * num_nodes
        if rank == 0:
            random.shuffle(ranks)
        dist.broadcast_object_list(ranks, src=0)
        size = self.island_size if self.island_size is not None else num_nodes
        for i in range(0, len(ranks), size):
            island = set(ranks[i:i + size])
            if rank in island:
                return island
        return None

    def _average_models(self, model, island_members: Set[int], num_nodes: int) -> None:
        s = self.strategy
        a = s.arena
        a.check_bound()
        if len(island_members) == num_nodes:
            if self._mean is None:
                self._mean = MeanReduce(s.coll, 1, a.n, a.device, a.dtype)
            self._mean(a.flat.view(1, -1))
            return
        if self._gathered is None:
            self._gathered = torch.empty(s.coll.world, a.n, device=a.device, dtype=a.dtype)
        s.coll.all_gather_into(self._gathered.view(-1), a.flat)
        rows = torch.tensor(sorted(island_members), dtype=torch.int32, device=a.device)
        ops.replica_mean(self._gathered, a.flat, n=a.n, rows=rows)

    def communicate(self, model, rank: int, num_nodes: int, local_step: int) -> None:
        if num_nodes > 1:
            if self.island_size is not None and self.island_size < num_nodes:
                members = self._select_partners(rank, num_nodes)
            else:
                members = set(range(num_nodes))
            with torch.no_grad():
                self._average_models(model, members, num_nodes)

    def _init_node(self, model, rank, num_nodes):
        pass


class FedAvgStrategy(CommunicateOptimizeStrategy):
    def __init__(self, inner_optim: Optional[Union[str, OptimSpec]] = None, island_size: Optional[int] = None,
                 H: int = 1, max_norm: float = None, **kwargs):
        averaging = AveragingCommunicator(island_size=island_size)
        super().__init__(inner_optim=inner_optim, communication_modules=[averaging], max_norm=max_norm, **kwargs)
        self.island_size = island_size
        self.H = H

    def _communicate(self):
        if self.local_step % self.H == 0 and self.local_step > 0:
            super()._communicate()

    def _init_node(self, model, rank, num_nodes):
        super()._init_node(model, rank, num_nodes)
        if self.island_size is None:
            self.island_size = num_nodes
