"""SPARTA: after every inner step, average a random sparse subset of the
parameters across nodes.

API of exogym/strategy/sparta.py:14-193: SparseCommunicator(index_selector)
(:14-47), SPARTAStrategy(inner_optim=None, p_sparta=0.005, **kwargs) (:50-66),
IndexSelector (:69-77), RandomIndexSelector (:80-85),
ShuffledSequentialIndexSelector (:88-136), PartitionedIndexSelector (:139-193).

The reference loops over every tensor that has a gradient (:28-30): draw the
mask, broadcast the bool mask from rank 0, gather, all-reduce, divide,
masked_scatter (:32-42).  Here one select+gather kernel runs over the whole
arena, ONE all-reduce moves the packed values (about p*N elements), one
scatter kernel writes them back.

Mask sources (RandomIndexSelector(p, mask_source=...), SPARTAStrategy(...,
mask_source=...)):
  "torch" (default) — the reference's exact draw,
      torch.bernoulli(torch.full(shape, p, device=param.device)) per tensor in
      parameter order (same generator calls, so the same selections and the
      same global RNG state afterwards), rank 0's masks broadcast as one mask
      arena packed to a bit per element (n/8 bytes instead of the reference's
      n bool bytes).  Bit-identical to the reference given the same generator.
  "philox" (opt-in fast mode) — each element is selected independently with
      probability p, drawn in-kernel as the Geometric(p) gaps between selected
      elements from Philox4x32-10 keyed by a per-run seed (rank 0's
      torch.initial_seed(), broadcast once) and the iteration (include/gym_amd.h,
      ga_sparta_gap_table); every rank computes the identical mask in-kernel, so the per-step N-byte mask broadcast and the per-tensor
      draws disappear.  Same distribution, a DIFFERENT random stream: selections
      are not the reference's, and the global torch RNG is not consumed.
      Tensors without a gradient are skipped as in the reference (a skip-range
      table passed to the kernel).
The ShuffledSequential / Partitioned selectors are the reference's algorithms
(the same torch draws on the device) feeding the mask-mode kernels.
"""
import math
from typing import Optional, Union

import torch

from ..engine import Sparta
from .communicate_optimize_strategy import CommunicateOptimizeStrategy, CommunicationModule
from .optim import OptimSpec


class IndexSelector:
    def __init__(self, p):
        self.state = {}
        self.p = p

    def get_indices(self, param, iteration):
        return torch.ones_like(param, dtype=torch.bool)


class RandomIndexSelector(IndexSelector):
    def __init__(self, p, mask_source="torch"):
        super().__init__(p)
        if mask_source not in ("philox", "torch"):
            raise ValueError(f"mask_source must be 'philox' or 'torch', got {mask_source!r}")
        self.mask_source = mask_source

    def get_indices(self, param, iteration):
        return torch.bernoulli(torch.full(param.shape, self.p, device=param.device)).bool()


def draw_masks(selector, params, views, skip, iteration, pfull):
    """Every tensor's selector mask into its view of a uint8 mask arena, in
    parameter order (sparta.py:28-33); tensors in `skip` stay 0.

    RandomIndexSelector: `view.bernoulli_(P)` with P = the cached
    torch.full(shape, p) of the tensor -- the same bernoulli kernel on the same
    probabilities as the reference's torch.bernoulli(torch.full(shape, p))
    (so the same bits and the same generator offsets), written straight into
    the arena: no per-step fill of 4 B/element, no float mask, no copy.
    pfull: the per-tensor cache (a list, filled here).  Other selectors: their
    get_indices, copied in."""
    fast = type(selector) is RandomIndexSelector
    if fast and len(pfull) != len(params):
        pfull[:] = [None] * len(params)
    for i, (p, v) in enumerate(zip(params, views)):
        if i in skip:
            v.zero_()
        elif fast:
            P = pfull[i]
            if P is None or P.shape != p.shape or P.device != p.device:
                P = pfull[i] = torch.full(p.shape, selector.p, device=p.device)
            v.bernoulli_(P)
        else:
            v.copy_(selector.get_indices(p, iteration))


class ShuffledSequentialIndexSelector(IndexSelector):
    """Cycles through a per-tensor random permutation in ceil(1/p) chunks."""

    def get_indices(self, param, iteration):
        n = param.numel()
        if n == 0:
            return torch.zeros_like(param, dtype=torch.bool)
        st = self.state.get(param)
        if st is None:
            st = self.state[param] = {"num_partitions": max(1, math.ceil(1.0 / self.p)),
                                      "shuffled_indices": torch.randperm(n, device=param.device)}
        parts = st["num_partitions"]
        c = iteration % parts
        size, rem = divmod(n, parts)
        lo = c * size + min(c, rem)
        hi = lo + size + (1 if c < rem else 0)
        mask = torch.zeros(n, dtype=torch.bool, device=param.device)
        sel = st["shuffled_indices"][lo:hi]
        if sel.numel() > 0:
            mask[sel] = True
        return mask.view(param.shape)


class PartitionedIndexSelector(IndexSelector):
    """Random partition of each tensor into ceil(1/p) parts, visited in turn,
    re-drawn when a cycle ends."""

    def _set_partition(self, param):
        st = self.state[param]
        st["curr_partition"] = 0
        parts = max(1, min(math.ceil(1.0 / self.p), param.numel()))
        st["num_partitions"] = parts
        if param.numel() > 0:
            st["partitions"] = torch.rand(param.numel(), device=param.device).argsort() % parts
        else:
            st["partitions"] = torch.empty(0, dtype=torch.long, device=param.device)

    def get_indices(self, param, iteration):
        if param.numel() == 0:
            return torch.zeros_like(param, dtype=torch.bool)
        if param not in self.state:
            self.state[param] = {}
            self._set_partition(param)
        elif self.state[param]["curr_partition"] >= self.state[param]["num_partitions"]:
            self._set_partition(param)
        st = self.state[param]
        if st["num_partitions"] == 0:
            return torch.zeros_like(param, dtype=torch.bool)
        mask = (st["partitions"] == st["curr_partition"]).view(param.shape).bool()
        st["curr_partition"] += 1
        return mask


class SparseCommunicator(CommunicationModule):
    def __init__(self, index_selector, **kwargs):
        super().__init__(**kwargs)
        self.index_selector = index_selector
        self.iteration = 0
        self._engine = None
        self._seed = None
        self._mask = None
        self._skip_key = None
        self._skip = None
        self._pfull = []

    def _init_node(self, model, rank, num_nodes):
        pass

    def _setup(self):
        s = self.strategy
        a = s.arena
        self._engine = Sparta(s.coll, 1, a.n, a.device, a.dtype, self.index_selector.p)

    def _philox_mode(self):
        sel = self.index_selector
        return isinstance(sel, RandomIndexSelector) and sel.mask_source == "philox"

    def _shared_seed(self):
        if self._seed is None:
            s = self.strategy
            t = torch.tensor([torch.initial_seed() & (2**63 - 1)], dtype=torch.int64, device=s.arena.device)
            s.coll.broadcast_(t, 0)
            self._seed = int(t.item())
        return self._seed

    def _skip_table(self):
        """[lo, hi) arena ranges of the tensors that are skipped this step
        (`not requires_grad or grad is None`, sparta.py:29-30), merged; None
        when every tensor takes part.  Cached on the device while unchanged."""
        a = self.strategy.arena
        key = tuple(i for i, p in enumerate(a.params) if not p.requires_grad or p.grad is None)
        if key != self._skip_key:
            rng = []
            for i in key:
                lo, hi = a.layout.offsets[i], a.layout.offsets[i] + a.layout.numels[i]
                if rng and rng[-1][1] == lo:
                    rng[-1][1] = hi
                else:
                    rng.append([lo, hi])
            self._skip = torch.tensor(rng, dtype=torch.int64, device=a.device).view(-1, 2) if rng else None
            self._skip_key = key
        return self._skip

    def _build_mask(self, model):
        """Reference mask path: per-tensor selector draws into one uint8 mask
        arena (frozen / grad-less tensors stay 0); the engine packs rank 0's
        and broadcasts it."""
        s = self.strategy
        a = s.arena
        if self._mask is None:
            self._mask = torch.zeros(a.n, dtype=torch.uint8, device=a.device)
        skip = {i for i, p in enumerate(a.params) if not p.requires_grad or p.grad is None}
        draw_masks(self.index_selector, a.params, a.layout.views(self._mask), skip, self.iteration, self._pfull)
        return self._mask

    def _mask_cap(self):
        """Selected-count bound for Bernoulli masks (no host sync per step);
        None (exact count read back) for the deterministic-cycle and custom
        selectors."""
        if type(self.index_selector) is RandomIndexSelector:
            return self._engine.cap
        return None

    def finish(self):
        if self._engine is not None:
            self._engine.check()

    def communicate(self, model, rank: int, num_nodes: int, local_step: int) -> None:
        if num_nodes > 1:
            if self._engine is None:
                self._setup()
            s = self.strategy
            s.arena.check_bound()
            with torch.no_grad():
                reps = s.arena.flat.view(1, -1)
                if self._philox_mode():
                    self._engine(reps, seed=self._shared_seed(), iteration=self.iteration, skip=self._skip_table())
                else:
                    self._engine(reps, mask=self._build_mask(model), mask_cap=self._mask_cap())
        self.iteration += 1


class SPARTAStrategy(CommunicateOptimizeStrategy):
    def __init__(self, inner_optim: Optional[Union[str, OptimSpec]] = None, p_sparta=0.005,
                 mask_source="torch", **kwargs):
        index_selector = RandomIndexSelector(p_sparta, mask_source=mask_source)
        sparse_comm = SparseCommunicator(index_selector)
        super().__init__(inner_optim=inner_optim, communication_modules=[sparse_comm], **kwargs)
        self.index_selector = index_selector
