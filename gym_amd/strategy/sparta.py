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
import warnings
from typing import Optional, Union

import torch
import torch.distributed as dist

from .. import ops
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


class MaskDraw:
    """State of draw_masks for one mask arena: the fused kernel's tensor table;
    for the per-tensor torch path the cached probability tensors and the HIP
    graph of the draw sequence."""

    fused = True       # one ga_sparta_torch_bernoulli launch for every tensor (GPU)
    use_graphs = True  # otherwise: the per-tensor torch draws, as one HIP graph replay
    offset_step = 12   # generator offset per bernoulli_ call (philox_cuda_state(10), rounded up to 4)

    def __init__(self):
        self.pfull = []
        self.key = None
        self.graph = None
        self.calls = 0
        self.table = None
        self.mode = None  # "fused" | "torch": which draw ran last (recorded in __config__ and the bench line)


def draw_masks(selector, params, views, skip, iteration, state, bits=None, coll=None, defer=False):
    """Every tensor's selector mask into its view of a uint8 mask arena, in
    parameter order (sparta.py:28-33); tensors in `skip` stay 0.  Returns the
    mask to select with: `bits` (int64 packed words of the same arena,
    ga_sparta_pack_mask layout) when the fused GPU draw wrote them there
    instead of the bytes, else None (the uint8 arena holds the masks).
    coll (a Collective with an exchange): the fused draw uses rank 0's
    generator state, broadcast (16 bytes), so the returned packed mask is
    already rank 0's on every rank (the reference broadcasts the masks,
    sparta.py:32-37); every rank's own generator still advances as its own
    draws would advance it.
    defer (no exchange): the fused path returns an ops.TorchDraw instead of
    drawing -- the SPARTA kernel then draws the same masks in-kernel
    (GA_MASK_TORCH); the generator is advanced here all the same.

    RandomIndexSelector on a GPU: one ga_sparta_torch_bernoulli launch draws
    every tensor's mask exactly as the per-tensor torch.bernoulli calls would
    (same bits, generator advanced by the same amount; _draw_fused).  With
    MaskDraw.fused off: `view.bernoulli_(P)` with P = the cached
    torch.full(shape, p) of the tensor -- the same bernoulli kernel on the same
    probabilities as the reference's torch.bernoulli(torch.full(shape, p))
    (so the same bits and the same generator offsets), written straight into
    the arena: no per-step fill of 4 B/element, no float mask, no copy.  The
    sequence is launch-bound (one small kernel per tensor), so from its second
    call on a GPU it runs as one captured HIP graph: a replay reads the
    generator's seed/offset at replay time and advances it by the captured
    total, i.e. draws exactly what the eager sequence would.  Other
    selectors: their get_indices, copied in (eager)."""
    fast = type(selector) is RandomIndexSelector
    if not fast:
        state.mode = "torch"
        for i, (p, v) in enumerate(zip(params, views)):
            if i in skip:
                v.zero_()
            else:
                v.copy_(selector.get_indices(p, iteration))
        return
    key = (tuple(v.data_ptr() for v in views), tuple(tuple(p.shape) for p in params), frozenset(skip),
           float(selector.p), str(params[0].device) if params else "")
    if key != state.key:
        state.key, state.graph, state.calls, state.table = key, None, 0, None
        state.pfull = [None] * len(params)

    def body():
        for i, (p, v) in enumerate(zip(params, views)):
            if i in skip:
                v.zero_()
            else:
                v.bernoulli_(state.pfull[i])

    on_gpu = _on_gpu(params)
    if on_gpu and MaskDraw.fused and coll is not None and coll.exchange and _capturing():
        # the fused and the torch draws exchange different things (16 B of generator state vs the
        # packed masks), and the choice is agreed across ranks by a collective: a rank inside a
        # graph capture would take the torch path alone and the ranks' collectives would not match
        raise RuntimeError("SPARTA: a multi-rank mask draw cannot run inside a graph capture (the ranks "
                           "must agree on the draw path); capture the single-process step only")
    # inside a user's graph capture the generator offsets are graph-relative: torch's own kernels then
    if (on_gpu and MaskDraw.fused and not _capturing()
            and fused_draw_matches_torch(params[0].device, coll)):
        out = _draw_fused(selector, params, views, skip, state, bits, coll, defer)
        state.calls += 1
        state.mode = "fused"
        return out
    state.mode = "torch"
    for i, p in enumerate(params):
        if i not in skip and state.pfull[i] is None:
            state.pfull[i] = torch.full(p.shape, selector.p, device=p.device)
    if (on_gpu and MaskDraw.use_graphs and state.graph is None and state.calls >= 1
            and not _capturing()):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            body()
        state.graph = g
    if state.graph is not None:
        state.graph.replay()
    else:
        body()
    state.calls += 1


def _on_gpu(params):
    return bool(params) and params[0].device.type == "cuda"


def _capturing():
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


_FUSED_OK = {}      # device -> this process's probe result
_FUSED_AGREED = {}  # (device, process group) -> the result every rank of the group uses
_FUSED_WARNED = set()


def _probe_fused(device):
    """One-time check per device that ga_sparta_torch_bernoulli still restates
    this torch build's bernoulli kernel: a 3-tensor probe drawn both ways from
    the same generator state (bits, and the state torch leaves behind), the
    caller's generator state restored afterwards."""
    dev = torch.device(device)
    gen = torch.cuda.default_generators[dev.index if dev.index is not None else torch.cuda.current_device()]
    state = torch.cuda.get_rng_state(dev)
    try:
        shapes = [(4099,), (64, 65), (1,)]
        p = 0.3
        want = [torch.bernoulli(torch.full(s, p, device=dev)).bool().reshape(-1) for s in shapes]
        after = torch.cuda.get_rng_state(dev)
        torch.cuda.set_rng_state(state, dev)
        numels = [w.numel() for w in want]
        offs = [sum(-(-m // 64) * 64 for m in numels[:i]) for i in range(len(numels))]
        table, nb = ops.sparta_bernoulli_table(offs, numels, dev)
        mask = torch.zeros(offs[-1] + numels[-1], dtype=torch.uint8, device=dev)
        off0 = gen.get_offset()
        ops.sparta_torch_bernoulli(table, nb, p, gen.initial_seed(), off0, MaskDraw.offset_step, mask)
        same_bits = all(torch.equal(mask[a:a + m].bool(), w) for a, m, w in zip(offs, numels, want))
        gen.set_offset(off0 + MaskDraw.offset_step * len(shapes))
        same_state = torch.equal(torch.cuda.get_rng_state(dev), after)
        return bool(same_bits and same_state)
    finally:
        torch.cuda.set_rng_state(state, dev)


def fused_draw_matches_torch(device, coll=None):
    """Whether draw_masks may use the fused kernel (_probe_fused, once per
    device).  With an exchange every rank must take the same path (the fused
    one broadcasts 16 bytes of generator state, the torch one the packed
    masks), so the probe results are combined once per group with a MIN
    all-reduce.  False -> torch's own kernels (same bits, ~10x slower), with
    a one-time warning; the draw that ran is recorded as MaskDraw.mode."""
    key = str(device)
    if key not in _FUSED_OK:
        _FUSED_OK[key] = bool(_probe_fused(device))
    ok = _FUSED_OK[key]
    if coll is not None and coll.exchange:
        gk = (key, id(coll.group))
        if gk not in _FUSED_AGREED:
            t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=coll.group)
            _FUSED_AGREED[gk] = bool(int(t.item()))
        ok = _FUSED_AGREED[gk]
    if not ok and key not in _FUSED_WARNED:
        _FUSED_WARNED.add(key)
        warnings.warn(f"SPARTA: the fused reference draw (ga_sparta_torch_bernoulli) does not match this torch "
                      f"build's bernoulli kernel on {key} (or on another rank); drawing with torch's per-tensor "
                      f"kernels instead (same masks, ~0.75 ms instead of ~0.07 ms per step at 124M)",
                      RuntimeWarning, stacklevel=2)
    return ok


def _i64(v):
    v = int(v) & (2**64 - 1)
    return v - 2**64 if v >= 2**63 else v


def _draw_fused(selector, params, views, skip, state, bits=None, coll=None, defer=False):
    """Every drawn tensor's torch.bernoulli(torch.full(shape, p)) in ONE launch
    (ga_sparta_torch_bernoulli: ATen's HIP kernel for it restated, bit for
    bit), with the default generator of the device read and advanced exactly
    as the per-tensor calls would (offset_step per drawn tensor).  With `bits`
    (int64 words covering the arena, the arena's trailing words zero) the
    masks are written packed, one bit per element, and `bits` is returned."""
    if state.table is None:
        base = views[0]._base if views[0]._base is not None else views[0]
        if base.dtype != torch.uint8 or not base.is_contiguous():
            raise ValueError("draw_masks: views must be views of one contiguous uint8 mask arena")
        drawn = [i for i in range(len(params)) if i not in skip]
        offs = [views[i].storage_offset() - base.storage_offset() for i in drawn]
        state.table = ops.sparta_bernoulli_table(offs, [views[i].numel() for i in drawn], base.device)
        state.base, state.ndrawn = base, len(drawn)
        # packed words of the skipped tensors (their offsets are multiples of 64)
        state.skip_words = [((views[i].storage_offset() - base.storage_offset()) // 64,
                             -(-(views[i].storage_offset() - base.storage_offset() + views[i].numel()) // 64))
                            for i in sorted(skip)]
    table, nblocks = state.table
    dev = state.base.device
    gen = torch.cuda.default_generators[dev.index if dev.index is not None else torch.cuda.current_device()]
    if defer and not (coll is not None and coll.exchange) and state.ndrawn > 0:
        off0 = gen.get_offset()
        gen.set_offset(off0 + MaskDraw.offset_step * state.ndrawn)
        return ops.TorchDraw(table, selector.p, gen.initial_seed(), off0, MaskDraw.offset_step)
    out = state.base
    if bits is not None:
        if bits.dtype != torch.int64 or bits.numel() < ops.sparta_mask_words(state.base.numel()):
            raise ValueError("draw_masks: bits must be int64 words covering the mask arena")
        for a, b in state.skip_words:
            bits[a:b].zero_()
        out = bits
    else:
        for i in skip:
            views[i].zero_()
    off0 = gen.get_offset()
    seedoff = None
    if coll is not None and coll.exchange:  # rank 0's generator state, 16 bytes on the wire
        if getattr(state, "seedoff", None) is None:
            state.seedoff = torch.zeros(2, dtype=torch.int64, device=dev)
        state.seedoff[0].fill_(_i64(gen.initial_seed()))
        state.seedoff[1].fill_(_i64(off0))
        coll.broadcast_(state.seedoff, 0)
        seedoff = state.seedoff
    ops.sparta_torch_bernoulli(table, nblocks, float(selector.p), gen.initial_seed(), off0, MaskDraw.offset_step, out,
                               seedoff=seedoff)
    gen.set_offset(off0 + MaskDraw.offset_step * state.ndrawn)
    return bits


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
        self._draw = MaskDraw()
        self.mask_draw = None  # "philox" | "fused" | "torch" once a step has drawn (read by __config__)

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
            self._bits = torch.zeros(ops.sparta_mask_words(a.n), dtype=torch.int64, device=a.device)
        skip = {i for i, p in enumerate(a.params) if not p.requires_grad or p.grad is None}
        packed = draw_masks(self.index_selector, a.params, a.layout.views(self._mask), skip, self.iteration,
                            self._draw, bits=self._bits, coll=s.coll)
        self._shared = packed is not None
        return self._mask if packed is None else packed

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
                    self.mask_draw = "philox"
                else:
                    m = self._build_mask(model)
                    self._engine(reps, mask=m, mask_cap=self._mask_cap(), mask_shared=self._shared)
                    self.mask_draw = self._draw.mode
                s.mask_draw = self.mask_draw
        self.iteration += 1


class SPARTAStrategy(CommunicateOptimizeStrategy):
    def __init__(self, inner_optim: Optional[Union[str, OptimSpec]] = None, p_sparta=0.005,
                 mask_source="torch", **kwargs):
        index_selector = RandomIndexSelector(p_sparta, mask_source=mask_source)
        sparse_comm = SparseCommunicator(index_selector)
        super().__init__(inner_optim=inner_optim, communication_modules=[sparse_comm], **kwargs)
        self.index_selector = index_selector
        self.mask_draw = None  # which mask draw the last step ran ("philox" | "fused" | "torch")
