"""Flat parameter arenas.

One simulated node's parameters live in ONE contiguous buffer so a single
kernel launch (and a single RCCL call) covers every tensor, instead of the
reference's per-tensor loops (e.g. strategy.py:130-133, diloco.py:34-41,
sparta.py:28-42).  Tensor offsets are aligned to 64 elements (256 B for
fp32) so every tensor starts on a cache line and 16-byte vector loads stay
aligned; the padding between tensors is kept at zero, so elementwise kernels
may run over the whole arena.

ArenaLayout   offsets of an ordered shape list (+ the padded arena length)
ReplicaSet    K replicas of a layout as one [K, ld] tensor (batched-replica mode)
ParamArena    re-points an nn.Module's parameters (and their .grad) at views
              of a flat buffer, keeping `model.parameters()` / `state_dict()`
              keys and shapes unchanged
"""
import math

import torch

ALIGN = 64  # elements


def _round_up(x, m):
    return (x + m - 1) // m * m


class ArenaLayout:
    def __init__(self, shapes, align=ALIGN, shard_multiple=8):
        self.shapes = [tuple(int(d) for d in s) for s in shapes]
        self.numels = [int(math.prod(s)) for s in self.shapes]
        self.offsets = []
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off = _round_up(off + n, align)
        self.n_params = sum(self.numels)
        # padded so [n] splits into `shard_multiple` aligned shards (reduce-scatter)
        self.n = max(_round_up(off, align * shard_multiple), align * shard_multiple)

    def __len__(self):
        return len(self.shapes)

    def subset(self, indices):
        """The tensors `indices` of this layout at their offsets in the SAME
        arena (n unchanged): e.g. the trainable tensors a codec covers while
        frozen ones stay in the arena untouched."""
        sub = object.__new__(ArenaLayout)
        sub.shapes = [self.shapes[i] for i in indices]
        sub.numels = [self.numels[i] for i in indices]
        sub.offsets = [self.offsets[i] for i in indices]
        sub.n_params = sum(sub.numels)
        sub.n = self.n
        return sub

    def views(self, flat):
        """Per-tensor views of a flat [>= n] buffer."""
        return [flat[o:o + n].view(s) for o, n, s in zip(self.offsets, self.numels, self.shapes)]

    def shard(self, rank, world):
        """[begin, end) of rank's shard for a world-size split (aligned)."""
        per = _round_up(-(-self.n // world), ALIGN)
        b = min(rank * per, self.n)
        return b, min(b + per, self.n)

    def padded_to(self, world):
        per = _round_up(-(-self.n // world), ALIGN)
        return per * world


class ReplicaSet:
    """K simulated-node replicas of one arena: data[k] is replica k."""

    def __init__(self, layout, K, device, dtype=torch.float32, ld=None, fill=None):
        self.layout = layout
        self.K = int(K)
        self.ld = int(ld or layout.n)
        self.data = torch.zeros(self.K, self.ld, device=device, dtype=dtype) if fill is None else fill
        assert self.data.shape == (self.K, self.ld)

    def replica(self, k):
        return self.data[k]

    def relocate(self, data):
        """Move the replicas into another [K, ld] buffer (contents copied)."""
        if data.shape != self.data.shape or data.dtype != self.data.dtype:
            raise ValueError("ReplicaSet.relocate: a buffer of the set's shape and dtype")
        if data.data_ptr() != self.data.data_ptr():
            data.copy_(self.data)
        self.data = data

    def views(self, k):
        return self.layout.views(self.data[k])


class ParamArena:
    """Binds the parameters of a module (or a parameter list) to one flat
    buffer and their gradients to another.  Parameters without
    requires_grad are still placed (they keep their values) but get no grad."""

    def __init__(self, params, device=None, dtype=None, world=1, with_grad=True, flat=None, grad_flat=None):
        self.params = [p for p in params]
        if not self.params:
            raise ValueError("ParamArena: empty parameter list")
        self.device = device or self.params[0].device
        self.dtype = dtype or self.params[0].dtype
        for p in self.params:
            if p.dtype != self.dtype:
                raise TypeError(f"ParamArena: mixed parameter dtypes ({p.dtype} vs {self.dtype})")
        self.layout = ArenaLayout([p.shape for p in self.params])
        n = self.layout.padded_to(world)
        self.external = flat is not None
        if flat is not None:  # a row of a ReplicaArena (zeroed by its owner)
            if flat.numel() != n or (with_grad and (grad_flat is None or grad_flat.numel() != n)):
                raise ValueError(f"ParamArena: external buffers must hold {n} elements")
            self.flat, self.grad_flat = flat, (grad_flat if with_grad else None)
        else:
            self.flat = torch.zeros(n, device=self.device, dtype=self.dtype)
            self.grad_flat = torch.zeros(n, device=self.device, dtype=self.dtype) if with_grad else None
        with torch.no_grad():
            for p, v in zip(self.params, self.layout.views(self.flat)):
                v.copy_(p.data)
                p.data = v
        self._data_ptrs = [p.data_ptr() for p in self.params]
        self._grad_views = None
        if with_grad:
            self._grad_views = self.layout.views(self.grad_flat)
            for p, g in zip(self.params, self._grad_views):
                if p.requires_grad:
                    if p.grad is not None:
                        g.copy_(p.grad)
                    p.grad = g

    @property
    def n(self):
        return self.flat.numel()

    def check_bound(self):
        """Raise if something re-pointed a parameter away from the arena
        (e.g. `param.data = ...`), which would silently desynchronise it."""
        if [p.data_ptr() for p in self.params] != self._data_ptrs:
            raise RuntimeError("ParamArena: a parameter's storage was replaced outside the arena; "
                               "update parameters in place (param.data.copy_) instead")

    def sync_grads(self):
        """Make sure every .grad is the arena view (autograd allocates a fresh
        tensor when .grad was None, e.g. after zero_grad(set_to_none=True)):
        copy such grads into the arena and re-point them."""
        if self._grad_views is None:
            return
        for p, g in zip(self.params, self._grad_views):
            if not p.requires_grad:
                continue
            cur = p.grad
            if cur is g:
                continue
            if cur is None:
                g.zero_()
            elif cur.data_ptr() != g.data_ptr():
                g.copy_(cur)
            p.grad = g

    def zero_grad(self):
        if self.grad_flat is not None:
            self.grad_flat.zero_()
            self.rebind_grads()

    def relocate(self, flat, grad_flat):
        """Move the parameters and gradients into new buffers of the same size
        (contents copied; every parameter's .data and .grad re-pointed): how the
        DeMo optimizer moves them into the memory its step runs fastest on."""
        if self.external:
            raise RuntimeError("ParamArena.relocate: the buffers belong to a ReplicaArena")
        if flat.numel() != self.n or (self.grad_flat is not None and grad_flat.numel() != self.n):
            raise ValueError("ParamArena.relocate: buffers of the arena's size")
        with torch.no_grad():
            if flat.data_ptr() != self.flat.data_ptr():
                flat.copy_(self.flat)
            self._bind(flat)
            if self.grad_flat is not None:
                if grad_flat.data_ptr() != self.grad_flat.data_ptr():
                    grad_flat.copy_(self.grad_flat)
                self.grad_flat = grad_flat
                self._grad_views = self.layout.views(grad_flat)
                self.rebind_grads()

    def _bind(self, flat):
        """Point every parameter's .data at its view of `flat` (contents already there)."""
        self.flat = flat
        for p, v in zip(self.params, self.layout.views(flat)):
            p.data = v
        self._data_ptrs = [p.data_ptr() for p in self.params]

    def rebind_grads(self):
        """Point every trainable parameter's .grad back at its arena view."""
        if self._grad_views is not None:
            for p, g in zip(self.params, self._grad_views):
                if p.requires_grad:
                    p.grad = g


class ReplicaArena:
    """K simulated nodes hosted by one process (batched-replica mode,
    SURVEY §8(f) row 1): K model copies whose parameters and gradients are the
    rows of one [K, ld] parameter set and one [K, ld] gradient set, so every
    strategy kernel covers all K nodes in one launch.  arenas[k] is node k's
    ParamArena (row views; model k's param.data / .grad point into them)."""

    def __init__(self, models, world=1, with_grad=True):
        self.models = list(models)
        if not self.models:
            raise ValueError("ReplicaArena: no models")
        p0 = list(self.models[0].parameters())
        self.layout = ArenaLayout([p.shape for p in p0])
        self.K = len(self.models)
        self.ld = self.layout.padded_to(world)
        self.device, self.dtype = p0[0].device, p0[0].dtype
        self.flat_set = torch.zeros(self.K, self.ld, device=self.device, dtype=self.dtype)
        self.grad_set = torch.zeros(self.K, self.ld, device=self.device, dtype=self.dtype) if with_grad else None
        self.arenas = []
        for k, m in enumerate(self.models):
            ps = list(m.parameters())
            if [tuple(p.shape) for p in ps] != self.layout.shapes:
                raise ValueError("ReplicaArena: the replicas must share one parameter layout")
            self.arenas.append(ParamArena(ps, world=world, with_grad=with_grad, flat=self.flat_set[k],
                                          grad_flat=self.grad_set[k] if with_grad else None))
        self.params = [p for a in self.arenas for p in a.params]

    @property
    def n(self):
        return self.ld

    def sync_grads(self):
        for a in self.arenas:
            a.sync_grads()

    def relocate_grads(self, grad_set):
        """Move the K gradient rows into another [K, ld] buffer (contents copied;
        every model's .grad re-pointed at its view of the new rows): how the
        SimpleReduce step moves the gradient set into the memory its mean runs
        fastest on (engine.MeanReduce._place)."""
        if self.grad_set is None or grad_set.shape != self.grad_set.shape or grad_set.dtype != self.grad_set.dtype:
            raise ValueError("ReplicaArena.relocate_grads: a buffer of the gradient set's shape and dtype")
        with torch.no_grad():
            if grad_set.data_ptr() != self.grad_set.data_ptr():
                grad_set.copy_(self.grad_set)
            self.grad_set = grad_set
            for k, a in enumerate(self.arenas):
                a.grad_flat = grad_set[k]
                a._grad_views = a.layout.views(grad_set[k])
                a.rebind_grads()

    def relocate_params(self, flat_set):
        """Move the K parameter rows into another [K, ld] buffer (contents copied;
        every model's parameters re-pointed at their views of the new rows;
        gradients stay): how the DiLoCo outer step moves the replica set into
        the memory its step runs fastest on (engine.DiLoCoOuter._place)."""
        if flat_set.shape != self.flat_set.shape or flat_set.dtype != self.flat_set.dtype:
            raise ValueError("ReplicaArena.relocate_params: a buffer of the parameter set's shape and dtype")
        with torch.no_grad():
            if flat_set.data_ptr() != self.flat_set.data_ptr():
                flat_set.copy_(self.flat_set)
            self.flat_set = flat_set
            for k, a in enumerate(self.arenas):
                a._bind(flat_set[k])

    def zero_grad(self):
        if self.grad_set is not None:
            self.grad_set.zero_()
            for a in self.arenas:
                a.rebind_grads()

    def check_bound(self):
        for a in self.arenas:
            a.check_bound()
