"""Batched-replica node loop.

The reference runs one OS process per simulated node and, with more nodes than
GPUs, puts several processes on one GPU over gloo (exogym/trainer.py:310-351).
Here one process per GPU hosts K_local = num_nodes / processes simulated nodes:
K model copies whose parameters and gradients are the rows of one [K, ld]
ReplicaArena, so the strategy's communication step is the batched engine
(gym_amd.engine: in-kernel reduction over the K local nodes, RCCL across the
processes) and the inner optimizer is one fused launch over all K nodes.

Each node keeps the reference's per-node semantics (train_node.py:145-175):
its own data shard (DistributedSampler(num_replicas=num_nodes, rank=node) or
the dataset factory called with the node's rank), gradient accumulation over
batch_size // minibatch_size minibatches with `grad /= batch_size /
minibatch_size`, its own clip_grad_norm_, then the strategy step.  Supported
strategies: SimpleReduce, DiLoCo (any outer optimizer: the fused kernel for
SGD-family, torch's optimizer on an fp32 master otherwise), SPARTA (every
selector: the torch-drawn masks of node 0 -- the reference uses rank 0's --
or the Philox stream), FedAvg (full or island averaging), DeMo.  Anything else runs on
the process-per-node path (ReplicaRunner.supports).

The K nodes' forward/backward passes run one node after the other by default
(replica_forward="loop": each node's gradients bit-identical to its own
process).  replica_forward="vmap" runs them as one torch.func.vmap over the
rows of the replica arena instead (BatchedForward: batched GEMMs instead of K
sets of small launches; gradients equal to the loop's up to fp32 rounding).
"""
import contextlib
import copy
import random
import warnings

import numpy as np
import torch
import torch.distributed as dist
from torch.func import functional_call, vmap
from torch.utils.data import DataLoader

from . import ops
from .arena import ReplicaArena
from .comm import Collective
from .engine import DiLoCoOuter, MeanReduce, Sparta, demo_codec
from .fused_optim import ArenaAdam, fusable
from .strategy.demo import DeMoStrategy
from .strategy.diloco import DiLoCoStrategy, fused_sgd_hparams
from .strategy.federated_averaging import FedAvgStrategy
from .strategy.sparta import MaskDraw, RandomIndexSelector, SPARTAStrategy, draw_masks
from .strategy.strategy import SimpleReduceStrategy, clip_arena_grad_norm_


def consecutive_runs(xs):
    """[(first, last)] of the runs of consecutive integers in ascending xs."""
    runs = []
    for x in xs:
        if runs and x == runs[-1][1] + 1:
            runs[-1][1] = x
        else:
            runs.append([x, x])
    return [tuple(r) for r in runs]


class _LRGroup(torch.optim.Optimizer):
    """Holds the learning rate a scheduler drives when the step itself is a
    kernel (DeMo): one group with one placeholder parameter, no state."""

    def __init__(self, lr):
        super().__init__([torch.zeros(1, requires_grad=True)], {"lr": lr})

    def step(self, closure=None):
        return None


class _PerNodeOptim:
    """K torch optimizers (a non-fusable inner OptimSpec), one per local node,
    each clipped by its own gradient norm (clip_grad_norm_ per node)."""

    def __init__(self, spec, models, arenas):
        self.opts = [spec.build(m) for m in models]
        self.arenas = arenas
        self.param_groups = self.opts[0].param_groups

    def step(self, max_norm=None):
        for a, o in zip(self.arenas, self.opts):
            if max_norm:
                a.sync_grads()
                clip_arena_grad_norm_(a.grad_flat, max_norm)
            o.step()


class ReplicaRunner:
    """The strategy step for the K_local nodes of one process."""

    @staticmethod
    def supports(strategy):
        if isinstance(strategy, SPARTAStrategy):
            return True
        if isinstance(strategy, FedAvgStrategy):
            return True
        if isinstance(strategy, DiLoCoStrategy):
            return True  # any outer OptimSpec: fused kernel for SGD, torch's optimizer on a master otherwise
        return isinstance(strategy, (SimpleReduceStrategy, DeMoStrategy))

    def __init__(self, strategy, models, rank, num_nodes):
        if not self.supports(strategy):
            raise NotImplementedError(f"{type(strategy).__name__} with these options has no batched-replica path")
        self.s = strategy
        self.coll = Collective()
        self.K = len(models)
        self.rank, self.num_nodes = rank, num_nodes
        self.first_node = rank * self.K
        if self.coll.world * self.K != num_nodes:
            raise ValueError(f"{self.coll.world} processes x {self.K} replicas != {num_nodes} nodes")
        self.models = models
        self.ra = ReplicaArena(models, world=self.coll.world)
        dev, dt, ld = self.ra.device, self.ra.dtype, self.ra.ld
        # every node starts from node 0's parameters (train_node.py:86-92)
        with torch.no_grad():
            self.coll.broadcast_(self.ra.flat_set[0], 0)
            if self.K > 1:
                ops.replica_mean(self.ra.flat_set[0:1], self.ra.flat_set[1:], divisor=1.0)
        s = strategy
        s.local_step = 0
        s.max_steps = getattr(s, "max_steps", 1)
        s.rank, s.num_nodes = rank, num_nodes
        self.max_norm = None
        self.lr_scheds = []
        if isinstance(s, DeMoStrategy):
            kw = s.optimizer_kwargs()
            self.demo_kw = kw
            self.optim = _LRGroup(kw.get("lr", 0.001))
            self.delta = torch.zeros_like(self.ra.flat_set)
            # the codec covers the trainable tensors only, as DeMo's param list (demo.py:99-117)
            live = [i for i, p in enumerate(self.ra.arenas[0].params) if p.requires_grad]
            self.codec = demo_codec(self.coll, self.K, self.ra.layout.subset(live), dev,
                                    chunk=kw["compression_chunk"], topk=kw["compression_topk"],
                                    bf16_transform=kw.get("bf16_transform", "fp32") if dt == torch.bfloat16
                                    else "fp32")
            # after the first step the [K, ld] parameter, gradient and delta sets may move into
            # the memory the K-row encode + decode run fastest on, as the DeMo optimizer's own
            # (_place_demo; placement=False keeps them where they are)
            self.placement, self._placed = None, None
        else:
            spec = s.optim_spec if isinstance(s, SimpleReduceStrategy) else s.inner_optim_spec
            if fusable(spec.cls, spec.kwargs, self.ra):
                kw = {k: v for k, v in (spec.kwargs or {}).items() if k in ("lr", "betas", "eps", "weight_decay")}
                self.optim = ArenaAdam(self.ra.params, self.ra, decoupled=spec.cls is torch.optim.AdamW,
                                       placement=s.placement_opt, **kw)
            else:
                self.optim = _PerNodeOptim(spec, models, self.ra.arenas)
            if isinstance(s, DiLoCoStrategy):
                self.max_norm = s.kwargs.get("max_norm")
                hp = fused_sgd_hparams(s.outer_optim_spec)
                if hp is not None:
                    self.outer = DiLoCoOuter(self.coll, self.K, ld, dev, dt, placement=s.placement_opt, **hp)
                    self.outer.init_master(self.ra.flat_set[0])
                    # the step may move the replica set itself (every model re-pointed)
                    self.outer.relocate_replicas = self.ra.relocate_params
                else:
                    # any other outer OptimSpec (diloco.py:26-28): torch's optimizer on an fp32
                    # master of node 0's start (diloco.py:81-89), fed the node average
                    self.outer = self._generic_outer
                    self.master = torch.nn.Parameter(self.ra.flat_set[0].detach().float().clone())
                    self.outer_optimizer = s.outer_optim_spec.build([self.master])
                    self._avg = torch.empty(ld, device=dev, dtype=dt)
            else:
                self.max_norm = s.max_norm
            self.islands = (isinstance(s, FedAvgStrategy) and s.island_size is not None
                            and s.island_size < num_nodes)
            if isinstance(s, (SimpleReduceStrategy, FedAvgStrategy)) and not self.islands:
                self.mean = MeanReduce(self.coll, self.K, ld, dev, dt, placement=s.placement_opt)
                # the mean may move the set it averages (gradients for SimpleReduce, parameters for
                # FedAvg) into the memory it runs fastest on, once (MeanReduce._place)
                self.mean.relocate_replicas = (self.ra.relocate_grads if isinstance(s, SimpleReduceStrategy)
                                               else self.ra.relocate_params)
            if self.islands:
                self._isl_row = torch.empty(1, ld, device=dev, dtype=dt)
                self._isl_all = None  # [num_nodes, ld]: every node's parameters, gathered (processes > 1)
            elif isinstance(s, SPARTAStrategy):
                self.sparta = Sparta(self.coll, self.K, ld, dev, dt, s.index_selector.p)
                sel = s.index_selector
                self.philox = isinstance(sel, RandomIndexSelector) and sel.mask_source == "philox"
                if self.philox:
                    t = torch.tensor([torch.initial_seed() & (2**63 - 1)], dtype=torch.int64, device=dev)
                    self.coll.broadcast_(t, 0)
                    self.seed = int(t.item())
                else:
                    self.mask = torch.zeros(ld, dtype=torch.uint8, device=dev)
                    self.bits = torch.zeros(ops.sparta_mask_words(ld), dtype=torch.int64, device=dev)
                    self.draw = MaskDraw()
                self.iteration = 0
        # the strategy's LR schedule on every optimizer (strategy.py:75-112)
        for o in (self.optim.opts if isinstance(self.optim, _PerNodeOptim) else [self.optim]):
            s.optim = o
            s._setup_scheduler()
            if s.scheduler is not None:
                self.lr_scheds.append(s.scheduler)
        s.optim = self.optim

    def zero_grad(self):
        self.ra.zero_grad()

    @torch.no_grad()
    def step(self):
        s = self.s
        self.ra.check_bound()
        P, G = self.ra.flat_set, self.ra.grad_set
        if isinstance(s, DeMoStrategy):
            self.ra.sync_grads()
            lr = self.optim.param_groups[0]["lr"]
            kw = self.demo_kw
            self.codec(P, G, self.delta, lr, kw["compression_decay"], kw["weight_decay"])
            if self.placement is None:
                self._place_demo(P, G, lr)
        elif isinstance(s, SimpleReduceStrategy):
            self.ra.sync_grads()
            self.mean(G)
            self._inner()
        elif isinstance(s, DiLoCoStrategy):
            self._inner()
            if s.local_step % s.H == 0 and s.local_step > 0:
                self.outer(P)
        elif isinstance(s, SPARTAStrategy):
            self._inner()
            if self.philox:
                self.sparta(P, seed=self.seed, iteration=self.iteration, skip=self._skip_table())
            else:
                sel = s.index_selector
                m = self._build_mask()
                self.sparta(P, mask=m, mask_cap=self.sparta.cap if type(sel) is RandomIndexSelector else None,
                            mask_shared=self.mask_shared)
            self.iteration += 1
        elif isinstance(s, FedAvgStrategy):
            self._inner()
            if s.local_step % s.H == 0 and s.local_step > 0:
                if self.islands:
                    self._island_average(P)
                else:
                    self.mean(P)
        for sch in self.lr_scheds:
            sch.step()
        if self.rank == 0 and self.lr_scheds:
            for cb in s.lr_callbacks:
                cb(self.lr_scheds[0].get_last_lr()[0])
        s.local_step += 1

    def _place_demo(self, P, G, lr):
        """Once, after the first DeMo step: the K nodes' parameter, gradient and
        delta sets into the fresh device allocations the step's encode + decode
        run fastest on (engine.place_demo_step over [K, ld] sets, as
        demo_impl.demo.DeMo._place does for one node; the probe restores all
        three, so the nodes' steps are unchanged).  Every model's parameters and
        gradients are re-pointed at their rows of the moved sets
        (ReplicaArena.relocate_params / relocate_grads; the caller contract of
        INTEGRATION.md applies)."""
        from .placement import policy
        ok, why = policy(self.demo_kw.get("placement", True))
        if not ok:
            self.placement = {"placed": False, "why": why}
            return
        bufs, tens, rec = self.codec.place(P, G, self.delta, lr, self.demo_kw["compression_decay"])
        self.placement = rec or {"placed": False}
        if bufs is None or tens is None or not any(b is not None for b in bufs):
            return
        if tens[0].data_ptr() != P.data_ptr():
            self.ra.relocate_params(tens[0])
        if tens[1].data_ptr() != G.data_ptr():
            self.ra.relocate_grads(tens[1])
        self.delta = tens[2]
        self._placed = bufs  # own the memory the sets now live in

    def _generic_outer(self, P):
        """DiLoCo's outer step for a non-SGD outer optimizer (diloco.py:34-49,
        66-74) over the K local nodes: the ascending fp32 sum of the rows
        (ga_replica_mean), an all-reduce across processes, true division by
        num_nodes (the reference's `/= num_nodes`), master.grad = master - avg,
        the torch optimizer's step, and the master written to every row -- the
        arithmetic of DiLoCoStrategy._outer_step on each process-per-node rank."""
        ops.replica_mean(P, self._avg, divisor=1.0)
        self.coll.all_reduce_(self._avg)
        ops.replica_mean(self._avg, self._avg, divisor=float(self.num_nodes))
        self.outer_optimizer.zero_grad()
        self.master.grad = self.master.detach() - self._avg.float()
        self.outer_optimizer.step()
        P.copy_(self.master.detach().to(P.dtype).unsqueeze(0).expand_as(P))

    def _island_average(self, P):
        """FedAvg islands (federated_averaging.py:26-69) over the nodes of this
        process: the first process shuffles the node ids with Python's `random`
        (the reference's rank 0 draw) and broadcasts them; every island is the
        ascending-node fp32 sum of its members over its size (ga_replica_mean
        through a row table, one launch per island), written to the members this
        process hosts.  With several processes each first all-gathers every
        node's parameters (the reference's all_gather), so islands may span them."""
        N, s = self.num_nodes, self.s.island_size
        ranks = list(range(N)) if self.rank == 0 else [None] * N
        if self.rank == 0:
            random.shuffle(ranks)
        if self.coll.world > 1:
            dist.broadcast_object_list(ranks, src=0)
        src = P
        if self.coll.exchange:
            if self._isl_all is None:
                self._isl_all = torch.empty(N, self.ra.ld, device=P.device, dtype=P.dtype)
            self.coll.all_gather_into(self._isl_all.view(-1), P.reshape(-1))
            src = self._isl_all
        lo, hi = self.first_node, self.first_node + self.K
        islands = [sorted(ranks[i:i + s]) for i in range(0, N, s)]
        # every island's ascending member list in ONE host-to-device copy per round
        table = torch.tensor([m for isl in islands for m in isl], dtype=torch.int32).to(P.device, non_blocking=True)
        a = 0
        for members in islands:
            rows = table[a:a + len(members)]
            a += len(members)
            mine = [m for m in members if lo <= m < hi]
            if not mine:
                continue
            ops.replica_mean(src, self._isl_row, rows=rows, divisor=float(len(members)))
            # written back in one launch per run of consecutive member rows
            for a0, a1 in consecutive_runs(mine):
                ops.replica_mean(self._isl_row, P[a0 - lo:a1 - lo + 1], divisor=1.0)

    def _grad_less(self):
        """Indices of node 0's tensors without a gradient (skipped, sparta.py:29-30)."""
        a0 = self.ra.arenas[0]
        return [i for i, p in enumerate(a0.params) if not p.requires_grad or p.grad is None]

    def _skip_table(self):
        L = self.ra.layout
        rng = []
        for i in self._grad_less():
            lo, hi = L.offsets[i], L.offsets[i] + L.numels[i]
            if rng and rng[-1][1] == lo:
                rng[-1][1] = hi
            else:
                rng.append([lo, hi])
        return torch.tensor(rng, dtype=torch.int64, device=self.ra.device).view(-1, 2) if rng else None

    def _build_mask(self):
        """Node 0's selector masks (the reference broadcasts rank 0's,
        sparta.py:32-37) as one uint8 arena; the engine packs the first
        process's and broadcasts it to the others."""
        a0 = self.ra.arenas[0]
        packed = draw_masks(self.s.index_selector, a0.params, self.ra.layout.views(self.mask), set(self._grad_less()),
                            self.iteration, self.draw, bits=self.bits, coll=self.coll, defer=True)
        self.mask_shared = packed is not None
        return self.mask if packed is None else packed

    def _inner(self):
        if isinstance(self.optim, ArenaAdam):
            self.optim.step(max_norm=self.max_norm or None)
        else:
            self.optim.step(max_norm=self.max_norm)

    def averaged_flat(self):
        """The mean over all num_nodes nodes' parameters (a new [ld] buffer)."""
        avg = torch.empty(self.ra.ld, device=self.ra.device, dtype=self.ra.dtype)
        ops.replica_mean(self.ra.flat_set, avg, divisor=1.0)
        self.coll.all_reduce_(avg)
        ops.replica_mean(avg, avg, divisor=float(self.num_nodes))
        return avg


_SDPA = torch.nn.functional.scaled_dot_product_attention


class _FoldedSDPA(torch.autograd.Function):
    """scaled_dot_product_attention (no mask, no dropout) whose vmap rule folds
    the vmapped node dim into the batch dim, so the K nodes' attention runs as
    one call of the fused kernel; backward recomputes the attention (the fused
    kernels' own backward has no batching rule on this stack)."""

    @staticmethod
    def forward(q, k, v, is_causal, scale):
        return _SDPA(q, k, v, is_causal=is_causal, scale=scale)

    @staticmethod
    def setup_context(ctx, inputs, output):
        q, k, v, is_causal, scale = inputs
        ctx.save_for_backward(q, k, v)
        ctx.is_causal, ctx.scale = is_causal, scale
        dt = q.device.type
        ctx.amp = (dt, torch.is_autocast_enabled(dt), torch.get_autocast_dtype(dt))

    @staticmethod
    def backward(ctx, grad_out):
        q, k, v = ctx.saved_tensors
        dt, enabled, dtype = ctx.amp
        want = ctx.needs_input_grad[:3]
        with torch.enable_grad(), torch.autocast(device_type=dt, dtype=dtype, enabled=enabled):
            qq, kk, vv = (t.detach().requires_grad_(w) for t, w in zip((q, k, v), want))
            out = _SDPA(qq, kk, vv, is_causal=ctx.is_causal, scale=ctx.scale)
            got = iter(torch.autograd.grad(out, [t for t, w in zip((qq, kk, vv), want) if w], grad_out))
        return tuple(next(got) if w else None for w in want) + (None, None)

    @staticmethod
    def vmap(info, in_dims, q, k, v, is_causal, scale):
        B = info.batch_size

        def fold(t, d):
            t = t.movedim(d, 0) if d is not None else t.unsqueeze(0).expand(B, *t.shape)
            return t.reshape(B * t.shape[1], *t.shape[2:])

        n = q.movedim(in_dims[0], 0).shape[1] if in_dims[0] is not None else q.shape[0]  # SDPA's own batch
        out = _FoldedSDPA.apply(fold(q, in_dims[0]), fold(k, in_dims[1]), fold(v, in_dims[2]), is_causal, scale)
        return out.reshape(B, n, *out.shape[1:]), 0


def _foldable(q, k, v):
    """True when the folded call is exact: every operand carries the same
    per-node leading dims (SDPA's own batch / heads), so node b's tokens stay in
    node b's slice of the folded batch.  Unbatched (L, E) operands or k / v
    broadcast over batch (a leading 1) are not foldable."""
    return q.dim() >= 3 and k.dim() == q.dim() and v.dim() == q.dim() and \
        q.shape[:-2] == k.shape[:-2] == v.shape[:-2]


def _sdpa_vmappable(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, scale=None, enable_gqa=False):
    if attn_mask is None and dropout_p == 0.0 and not enable_gqa and _foldable(query, key, value):
        return _FoldedSDPA.apply(query, key, value, is_causal, scale)
    from torch.nn.attention import SDPBackend, sdpa_kernel
    with sdpa_kernel([SDPBackend.MATH]):  # masks / dropout / broadcasts: the math backend batches under vmap
        return _SDPA(query, key, value, attn_mask=attn_mask, dropout_p=dropout_p, is_causal=is_causal, scale=scale,
                     enable_gqa=enable_gqa)


class _VmappableAttention(torch.overrides.TorchFunctionMode):
    """Routes torch.nn.functional.scaled_dot_product_attention to
    _sdpa_vmappable while the batched forward runs; every other torch function
    passes through.  A torch-function mode lives on the calling thread's mode
    stack, so only the batched forward sees it: the module attribute is never
    swapped and another thread calling SDPA meanwhile (a data-loader worker, an
    eval thread) gets torch's own function."""

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func is _SDPA:
            return _sdpa_vmappable(*args, **kwargs)
        return func(*args, **kwargs)


def _stack(batches):
    """K minibatches (tensors, or tuples / dicts of tensors) -> one with a leading K dim."""
    if isinstance(batches[0], dict):
        return {key: torch.stack([b[key] for b in batches]) for key in batches[0]}
    if isinstance(batches[0], (tuple, list)):
        return tuple(torch.stack(parts) for parts in zip(*batches))
    return torch.stack(batches)


class BatchedForward:
    """The forward + backward of K local nodes as ONE torch.func.vmap over the
    rows of their ReplicaArena (replica_forward="vmap").

    Each parameter's [K_c, *shape] view of the parameter set (a chunk of K_c
    nodes at a time, `chunk`, default all K) is a leaf whose .grad is the same
    view of the gradient set, so backward accumulates every node's gradient in
    place into its arena row, as the per-node loop does (gradient accumulation
    over minibatches included).  Buffers (BatchNorm statistics) go in stacked
    per node and are written back after the forward.  The model's forward must
    return the loss, as exogym's TrainNode expects (train_node.py:145-175);
    dropout draws differ per node (randomness="different").  Scaled dot-product
    attention without mask or dropout runs as ONE fused-kernel call over the
    nodes folded into its batch dim (_FoldedSDPA; the fused kernels' backward
    has no batching rule on this stack), with a mask, dropout or operands
    that do not fold (_foldable) on the math backend; the override is a
    torch-function mode active only around this forward, on this thread
    (_VmappableAttention).  The copy runs in the models' current train()/eval()
    mode.  BatchNorm under bf16 autocast does not batch (torch's vmap rule
    for batch_norm rejects autocast's mixed dtypes): such models keep the loop.

    Measured on MI355X (tools/exp_replica_vmap.py, profiles/r05k_replica_vmap.txt),
    32 nodes: the reference's char-level nanoGPT preset (4 layers, d 128, 16 x
    1024 tokens per node) 1.47x faster than the loop, at 16 x 256 tokens 4.5x;
    GPT-2 124M at 2 x 256 tokens 1.56x, at 8 x 1024 tokens 0.97x (compute-bound).
    The loop stays the default: its gradients are bit-identical to a process
    per node."""

    def __init__(self, models, ra, chunk=None):
        self.models = list(models)
        self.ra = ra
        self.K = len(self.models)
        self.chunk = int(chunk) if chunk else self.K
        if self.chunk < 1:
            raise ValueError(f"replica_vmap_chunk must be >= 1, got {chunk}")
        m0 = self.models[0]
        self.names = [n for n, _ in m0.named_parameters()]
        self.trainable = [p.requires_grad for p in m0.parameters()]
        if len(self.names) != len(ra.layout.shapes):
            raise ValueError("BatchedForward: the model's parameters do not match the arena layout")
        self.buf_names = [n for n, _ in m0.named_buffers()]
        # a storage-free copy of the module (functional_call supplies every tensor)
        memo = {id(p): torch.nn.Parameter(torch.empty_like(p, device="meta"), requires_grad=p.requires_grad)
                for p in m0.parameters()}
        memo.update({id(b): torch.empty_like(b, device="meta") for b in m0.buffers()})
        self.meta = copy.deepcopy(m0, memo)

        def loss_of(params, bufs, batch):
            return functional_call(self.meta, (dict(zip(self.names, params)), bufs), (batch,))

        self.vloss = vmap(loss_of, in_dims=(0, 0, 0), randomness="different")

    def _leaves(self, c0, c1):
        ra, L = self.ra, self.ra.layout
        P, G = ra.flat_set, ra.grad_set
        leaves = []
        for o, n, shape, train in zip(L.offsets, L.numels, L.shapes, self.trainable):
            w = P[c0:c1, o:o + n].view(c1 - c0, *shape).detach()
            if train:
                w.requires_grad_(True)
                w.grad = G[c0:c1, o:o + n].view(c1 - c0, *shape)
            leaves.append(w)
        return leaves

    def __call__(self, batches, autocast=contextlib.nullcontext):
        """batches[k]: node k's minibatch; returns the K losses (detached)."""
        # the storage-free copy follows the models' current mode (dropout, BatchNorm), as
        # the per-node loop does: model.train()/eval() calls on the real models never reach it
        self.meta.train(self.models[0].training)
        losses = []
        for c0 in range(0, self.K, self.chunk):
            c1 = min(self.K, c0 + self.chunk)
            leaves = self._leaves(c0, c1)
            per_node = [dict(m.named_buffers()) for m in self.models[c0:c1]]
            bufs = {n: torch.stack([b[n] for b in per_node]) for n in self.buf_names}
            with autocast(), _VmappableAttention():
                loss = self.vloss(leaves, bufs, _stack(batches[c0:c1]))
            with warnings.catch_warnings():  # views of [K, ld] rows: strided, never the layout autograd prefers
                warnings.filterwarnings("ignore", message=".*gradient layout contract.*")
                loss.sum().backward()
            G = self.ra.grad_set
            for w, o, n, train in zip(leaves, self.ra.layout.offsets, self.ra.layout.numels, self.trainable):
                if train and w.grad.data_ptr() != G[c0, o:o + n].data_ptr():
                    raise RuntimeError("BatchedForward: a gradient left the arena")
            with torch.no_grad():
                for k, b in enumerate(per_node):
                    for n in self.buf_names:
                        b[n].copy_(bufs[n][k])
            losses.append(loss.detach())
        return torch.cat(losses)


class ReplicaTrainNode:
    """TrainNode (train_node.py:19-626) for the K_local nodes of one process."""

    def __init__(self, model, train_dataset, val_dataset, strategy, device, rank, num_nodes, K, num_epochs,
                 max_steps=None, batch_size=16, minibatch_size=16, val_size=64, val_interval=100, shuffle=True,
                 autocast=False, replica_forward="loop", replica_vmap_chunk=None, **kwargs):
        from .train_node import RunLog
        seed = kwargs.get("seed", 42)
        torch.manual_seed(seed)
        torch.cuda.manual_seed(seed)
        np.random.seed(seed)
        self.device, self.rank, self.num_nodes, self.K = device, rank, num_nodes, K
        self.models = [copy.deepcopy(model).to(device) for _ in range(K)]
        self.nodes = [rank * K + k for k in range(K)]
        self.batch_size, self.minibatch_size = batch_size, minibatch_size
        self.val_size, self.val_interval, self.autocast = val_size, val_interval, autocast
        self.loaders, self.iters, self.epoch = [], [], 0
        for node in self.nodes:
            if callable(train_dataset):
                ds, sampler = train_dataset(node, num_nodes, False), None
            else:
                ds = train_dataset
                sampler = torch.utils.data.DistributedSampler(ds, num_replicas=num_nodes, rank=node, shuffle=shuffle)
            dl = DataLoader(ds, batch_size=minibatch_size, sampler=sampler, shuffle=(sampler is None))
            self.loaders.append(dl)
            self.iters.append(iter(dl))
        vds = val_dataset(self.nodes[0], num_nodes, True) if callable(val_dataset) else val_dataset
        self.val_loader = DataLoader(vds, batch_size=minibatch_size, shuffle=True)
        self.val_iter = iter(self.val_loader)
        torch.manual_seed(42)
        torch.cuda.manual_seed(42)
        self.runner = ReplicaRunner(strategy, self.models, rank, num_nodes)
        self.strategy = strategy
        if replica_forward not in ("loop", "vmap"):
            raise ValueError(f"replica_forward must be 'loop' or 'vmap', got {replica_forward!r}")
        self.batched = (BatchedForward(self.models, self.runner.ra, replica_vmap_chunk)
                        if replica_forward == "vmap" else None)
        if max_steps is None:
            max_steps = num_epochs * len(self.loaders[0]) / (batch_size // minibatch_size)
        self.max_steps = max_steps
        strategy.max_steps = max_steps
        self.local_step = 0
        self.logger = RunLog(strategy, max_steps) if rank == 0 else None

    def _next(self, k):
        try:
            batch = next(self.iters[k])
        except StopIteration:
            if k == 0:
                self.epoch += 1
            self.iters[k] = iter(self.loaders[k])
            batch = next(self.iters[k])
        return self._to(batch)

    def _next_val(self):
        try:
            batch = next(self.val_iter)
        except StopIteration:
            self.val_iter = iter(self.val_loader)
            batch = next(self.val_iter)
        return self._to(batch)

    def _to(self, batch):
        if isinstance(batch, (tuple, list)):
            return tuple(x.to(self.device) for x in batch)
        return batch.to(self.device)

    def _autocast(self):
        if self.autocast:
            return torch.autocast(device_type=torch.device(self.device).type, dtype=torch.bfloat16)
        return contextlib.nullcontext()

    def _forward(self, model, minibatch):
        with self._autocast():
            return model(minibatch)

    def _train_step(self):
        self.runner.zero_grad()
        accum = self.batch_size // self.minibatch_size
        loss0 = None
        if self.batched is not None:
            for _ in range(accum):  # each node's loader in node order, as the loop draws them
                loss0 = self.batched([self._next(k) for k in range(self.K)], self._autocast)[0]
        else:
            for k, m in enumerate(self.models):
                for _ in range(accum):
                    loss = self._forward(m, self._next(k))
                    loss.backward()
                    if k == 0:
                        loss0 = loss
        self.runner.ra.sync_grads()
        self.runner.ra.grad_set.div_(self.batch_size / self.minibatch_size)
        self.runner.step()
        if self.logger is not None:
            self.logger.log_train(loss=loss0.item())

    def _eval_loss(self, model):
        model.eval()
        total = 0.0
        accum = self.batch_size // self.minibatch_size
        with torch.no_grad():
            for _ in range(int(self.val_size / self.batch_size)):
                for _ in range(accum):
                    total += self._forward(model, self._next_val()).item() / accum
        model.train()
        return total / max(1, int(self.val_size / self.batch_size))

    def _evaluate(self):
        if self.val_size == 0:
            return
        avg = self.runner.averaged_flat() if self.num_nodes > 1 else None
        if self.rank != 0:
            return
        self.logger.log_loss(loss=self._eval_loss(self.models[0]), name="local")
        if avg is not None:
            clone = copy.deepcopy(self.models[0])
            with torch.no_grad():
                for p, v in zip(clone.parameters(), self.runner.ra.layout.views(avg)):
                    p.copy_(v)
            self.logger.log_loss(loss=self._eval_loss(clone), name="global")

    def train(self):
        world = self.runner.coll.world
        while self.local_step < self.max_steps:
            if self.local_step % self.val_interval == 0:
                self._evaluate()
            self._train_step()
            self.local_step += 1
            if self.logger is not None:
                self.logger.increment_step()
            if world > 1:
                dist.barrier()
        if hasattr(self.runner, "sparta"):
            self.runner.sparta.check()
        self._evaluate()
        return [m.state_dict() for m in self.models]


def replica_layout(num_nodes, devices, replicas_per_process, strategy):
    """(processes, K_local) for Trainer.fit, or None for the process-per-node
    path.  replicas_per_process: None/"auto" = batch the nodes when there are
    more nodes than GPUs; an int forces K_local (1 = process per node)."""
    if replicas_per_process in (None, "auto"):
        G = len(devices)
        if num_nodes <= G or num_nodes % G != 0 or not ReplicaRunner.supports(strategy):
            return None
        return G, num_nodes // G
    K = int(replicas_per_process)
    if K <= 1:
        return None
    if num_nodes % K != 0:
        raise ValueError(f"num_nodes={num_nodes} is not a multiple of replicas_per_process={K}")
    if not ReplicaRunner.supports(strategy):
        raise NotImplementedError(f"{type(strategy).__name__} with these options has no batched-replica path")
    G = num_nodes // K
    if G > len(devices):
        raise ValueError(f"{G} processes need {G} GPUs, {len(devices)} given")
    return G, K
