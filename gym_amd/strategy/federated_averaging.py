"""FedAvg: average the parameters across nodes every H steps (optionally
within random islands).

API of exogym/strategy/federated_averaging.py:16-117:
AveragingCommunicator(island_size=None) and FedAvgStrategy(inner_optim=None,
island_size=None, H=1, max_norm=None, **kwargs); communication when
local_step % H == 0 and local_step > 0.

Full averaging is one RCCL all-reduce over the parameter arena plus one
division kernel (the reference: a per-tensor all-reduce + divide).  Island
averaging keeps the reference's partner draw — rank 0 shuffles the ranks with
Python's `random` and broadcasts the permutation (:27-51) — and its
arithmetic, the island's members summed in ascending rank order and divided
(:61-69), but moves only the island's arenas: each island is a sub-
communicator (`dist.new_group`, created once per distinct member set, by
every rank in permutation order, and cached), the members all-gather their
arenas within it ((s-1)·N received per rank instead of the reference's
(K-1)·N per-tensor all-gather over the world), and one ga_replica_mean over
the gathered rows averages them.  With a caller-supplied process group the
island step falls back to one all-gather over that group + the same mean over
the member rows.

Sub-communicators are bounded: each costs a store barrier over the world to
create and, under RCCL, a communicator with its own GPU buffers, and rank 0
reshuffles every round, so up to C(K, s) (+ C(K, K mod s)) member sets appear.
They are used only when EVERY set the shuffles can produce fits under
MAX_ISLAND_GROUPS (created lazily, as they first appear, and cached); when
that count exceeds the cap (e.g. 1820 sets at K = 16, s = 4) no group is ever
created and every round takes the world all-gather + member-row mean.  The
choice depends only on K, s and the cap, so every rank makes the same one.
"""
import math
import random
from typing import Optional, Set, Union

import torch
import torch.distributed as dist

from .. import ops
from ..comm import Collective
from ..engine import MeanReduce
from .communicate_optimize_strategy import CommunicateOptimizeStrategy, CommunicationModule
from .optim import OptimSpec

# cached island sub-communicators per process (bounded, no per-round growth)
MAX_ISLAND_GROUPS = 32


class AveragingCommunicator(CommunicationModule):
    def __init__(self, island_size: Optional[int] = None, **kwargs):
        super().__init__(**kwargs)
        self.island_size = island_size
        self._mean = None
        self._gathered = None
        self._islands = []     # this communication's islands, in permutation order
        self._groups = {}      # sorted member tuple -> (process group, Collective or None)

    def _select_partners(self, rank: int, num_nodes: int) -> Set[int]:
        ranks = list(range(num_nodes)) if rank == 0 else [None] * num_nodes
        if rank == 0:
            random.shuffle(ranks)
        dist.broadcast_object_list(ranks, src=0)
        size = self.island_size if self.island_size is not None else num_nodes
        self._islands = [set(ranks[i:i + size]) for i in range(0, len(ranks), size)]
        for island in self._islands:
            if rank in island:
                return island
        return None

    def _groups_possible(self, num_nodes: int) -> int:
        """Distinct multi-member island sets rank 0's shuffles can produce."""
        s = self.island_size if self.island_size is not None else num_nodes
        n = math.comb(num_nodes, s) if s > 1 else 0
        r = num_nodes % s
        return n + (math.comb(num_nodes, r) if r > 1 else 0)

    def _island_collective(self, members: Set[int], num_nodes: int):
        """(True, Collective over `members` or None for an island of one) when
        this round's islands use sub-communicators; (False, None) for the
        world all-gather path, which every rank then joins (islands of one
        included).  Every island of this communication that is new gets its
        group here, on every rank, in the permutation order rank 0 broadcast:
        dist.new_group is collective over the world, so all ranks create the
        same groups in the same order.  Sub-communicators are used only when
        every possible island set fits under MAX_ISLAND_GROUPS (module
        docstring)."""
        if self._groups_possible(num_nodes) > MAX_ISLAND_GROUPS:
            return False, None
        keys = [tuple(sorted(i)) for i in self._islands]
        new = [k for k in dict.fromkeys(keys) if len(k) > 1 and k not in self._groups]
        # every possible set fits under the cap (checked above), so the cache cannot outgrow it
        assert len(self._groups) + len(new) <= MAX_ISLAND_GROUPS
        me = dist.get_rank()
        for key in new:
            g = dist.new_group(list(key))
            self._groups[key] = (g, Collective(g) if me in key else None)
        key = tuple(sorted(members))
        return True, (self._groups[key][1] if len(key) > 1 else None)

    def _average_models(self, model, island_members: Set[int], num_nodes: int) -> None:
        s = self.strategy
        a = s.arena
        a.check_bound()
        if len(island_members) == num_nodes:
            if self._mean is None:
                self._mean = MeanReduce(s.coll, 1, a.n, a.device, a.dtype)
            self._mean(a.flat.view(1, -1))
            return
        members = sorted(island_members)
        sub, coll = (self._island_collective(island_members, num_nodes)
                     if s.coll.group is None and self._islands else (False, None))
        if sub and len(members) == 1:  # (0 + x) / 1, as the reference's sum([x]) / 1
            ops.replica_mean(a.flat.view(1, -1), a.flat, n=a.n)
            return
        if sub:
            rows_all = len(members)
            rows = None  # every gathered row is a member, in ascending rank order
        else:  # every rank joins the world all-gather, islands of one too
            coll, rows_all = s.coll, s.coll.world
            rows = torch.tensor(members, dtype=torch.int32, device=a.device)
        if self._gathered is None or self._gathered.shape[0] < rows_all:
            self._gathered = torch.empty(rows_all, a.n, device=a.device, dtype=a.dtype)
        buf = self._gathered[:rows_all]
        coll.all_gather_into(buf.view(-1), a.flat)
        ops.replica_mean(buf, a.flat, n=a.n, rows=rows)

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
