"""DeMo (Decoupled Momentum Optimization, Peng, Quesnelle & Kingma 2024,
arXiv:2411.19870) as a torch.optim.SGD subclass whose step runs on the gfx950
DCT codec kernels.

Constructor API of exogym/strategy/demo_impl/demo.py:39-90:
DeMo(params, compression_decay=0.999, compression_topk=32,
compression_chunk=64, weight_decay=0.0, process_group=None,
custom_all_gather=None, **sgd_kwargs) with the same argument checks, the
per-parameter `demo_state[p]` ({"step", "delta"}), and `data_transmit` /
`data_receive` byte counters reporting the reference's numbers (int64 index +
parameter-dtype value per transmitted coefficient, demo.py:188-190).

step() (demo.py:142-209): for every parameter, decoupled weight decay, delta
= decay*delta + lr*grad, chunked DCT-II, top-k per chunk, residual update,
all-gather of (idx, val), scatter-mean, inverse DCT, sign, SGD step.  Here:
the parameters, gradients and deltas are flat arenas, the whole model is one
encode launch, ONE all-gather of a packed payload (int32 idx + fp32 val per
coefficient; a wire format of our own, half the reference's int64 index
bytes), and one decode launch that also applies p -= lr*sign(g) and leaves
sign(g) in p.grad.
"""
from typing import Callable, Optional

import torch
import torch.distributed as dist

from ...arena import ParamArena
from ...comm import Collective
from ...demo_codec import smaller_split as _get_smaller_split  # noqa: F401  (demo.py:489-498, same name)
from ...engine import DeMoCodec, PipelinedDeMoCodec, demo_codec

_REQUIRE_GPU = True  # the CPU orchestration tests swap the kernels for oracle stand-ins


class DeMo(torch.optim.SGD):
    def __init__(self, params, compression_decay: float = 0.999, compression_topk: int = 32,
                 compression_chunk: int = 64, weight_decay: float = 0.0,
                 process_group: Optional[dist.ProcessGroup] = None, custom_all_gather=None, placement: bool = True,
                 bf16_transform: str = "fp32", **kwargs):
        super().__init__(params, foreach=False, momentum=0.0, dampening=0.0, nesterov=False, maximize=False,
                         weight_decay=0.0, **kwargs)
        if compression_topk <= 0:
            raise ValueError("topk_size has to be positive")
        if compression_chunk <= 0:
            raise ValueError("chunk_size has to be positive")
        if compression_decay < 0:
            raise ValueError("Negative compression_decay is currently not supported")
        if compression_decay >= 1:
            raise ValueError("Values of compression_decay bigger or equal to 1.0 is currently not supported")
        self.compression_decay = compression_decay
        self.compression_chunk = compression_chunk
        self.compression_topk = compression_topk
        self.process_group = process_group
        self.weight_decay = weight_decay
        self.custom_all_gather = custom_all_gather
        self.data_transmit = 0
        self.data_receive = 0

        if len(self.param_groups) != 1:
            raise NotImplementedError("gym_amd DeMo: one parameter group (the codec runs over one arena)")
        trainable = [p for p in self.param_groups[0]["params"] if p.requires_grad]
        if not trainable:
            raise ValueError("DeMo: no trainable parameters")
        if _REQUIRE_GPU and trainable[0].device.type != "cuda":
            raise RuntimeError("gym_amd DeMo runs on MI355X GPUs (no CPU fallback)")
        self.default_dtype = trainable[0].dtype
        self.coll = Collective(process_group)
        self.arena = ParamArena(trainable, world=self.coll.world)
        self.delta_flat = torch.zeros_like(self.arena.flat)
        # pipelined over tensor groups when the all-gather is async RCCL (engine.demo_codec);
        # a user-supplied custom_all_gather gets the one-exchange codec
        # bf16 parameters: "fp32" bases and arithmetic (default) or the reference's own bf16
        # transform ("reference": bf16 bases, every einsum stage rounded, demo.py:235-252)
        if bf16_transform not in ("fp32", "reference"):
            raise ValueError(f"bf16_transform must be 'fp32' or 'reference', got {bf16_transform!r}")
        self.bf16_transform = bf16_transform
        self._codec_kw = dict(chunk=compression_chunk, topk=compression_topk,
                              bf16_transform=bf16_transform if self.default_dtype == torch.bfloat16 else "fp32")
        self.codec = (demo_codec(self.coll, 1, self.arena.layout, self.arena.device, **self._codec_kw)
                      if self._gather_fn() is None else
                      DeMoCodec(self.coll, 1, self.arena.layout, self.arena.device, **self._codec_kw))
        self.demo_state = {}
        for p, d in zip(trainable, self.arena.layout.views(self.delta_flat)):
            self.demo_state[p] = {"step": 0, "delta": d}
        # placement=False: the parameters, gradients and deltas stay where they are
        # (no probe launches, no relocation); see _place
        self.place_opt = placement
        self.placement, self._placed = None, None
        itemsize = torch.finfo(self.default_dtype).bits // 8
        ref = self.codec.reference_bytes if isinstance(self.codec, PipelinedDeMoCodec) else self.codec.plan.reference_bytes
        self._tx = ref(itemsize)

    def _place(self, P, G, D, lr):
        """Once, after the first step: move the gradient, parameter and delta
        arenas into the device allocations the step's kernels run fastest on
        (engine.place_demo_step; the probe decodes at lr = 0, encodes into a
        scratch payload and restores P, G and D, so the results are unchanged).

        This RE-POINTS every trainable parameter's storage (`p.data`) and its
        `.grad` at views of the new buffers (the values are identical).  A
        caller that captured the old storage -- a CUDA/HIP graph of the forward
        and backward, a tensor alias, an EMA keyed by data_ptr -- must take it
        again after the first step, or pass placement=False (INTEGRATION.md,
        caller contract)."""
        from ...placement import policy
        ok, why = policy(self.place_opt)
        if not ok:
            self.placement = {"placed": False, "why": why}
            return
        bufs, tens, rec = self.codec.place(P, G, D, lr, self.compression_decay)
        self.placement = rec or {"placed": False}
        if bufs is not None and tens is not None and any(b is not None for b in bufs):
            self.arena.relocate(tens[0].view(-1), tens[1].view(-1))
            if tens[2].data_ptr() != self.delta_flat.data_ptr():
                self.delta_flat = tens[2].view(-1)
                for st, d in zip(self.demo_state.values(), self.arena.layout.views(self.delta_flat)):
                    st["delta"] = d
            self._placed = bufs  # own the memory the parameters / gradients / deltas now live in

    def _gather_fn(self):
        from ..communicate import all_gather as ours
        fn = self.custom_all_gather
        if fn is None or fn is ours or fn is dist.all_gather:
            return None  # one flat all_gather_into_tensor
        return fn

    @torch.no_grad()
    def step(self, closure: Optional[Callable] = None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        a = self.arena
        a.check_bound()
        a.sync_grads()
        for st in self.demo_state.values():
            st["step"] += 1
        lr = self.param_groups[0]["lr"]
        P = a.flat.view(1, -1)
        G = a.grad_flat.view(1, -1)
        D = self.delta_flat.view(1, -1)
        if isinstance(self.codec, PipelinedDeMoCodec):
            self.codec(P, G, D, lr, self.compression_decay, self.weight_decay)
        else:
            self.codec.encode(P, G, D, lr, self.compression_decay, self.weight_decay)
            self.codec.exchange(self._gather_fn())
            self.codec.decode(P, G, lr)
        if self.placement is None:
            self._place(P, G, D, lr)
        self.data_transmit = self._tx
        self.data_receive = self._tx * self.coll.world
        return loss
