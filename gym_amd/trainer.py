"""Trainer.fit: one OS process per simulated node, MI355X-first process groups.

API of exogym/trainer.py:122-351 (Trainer(model, train_dataset, val_dataset,
start_port=None, **kwargs); fit(num_epochs, strategy, num_nodes, max_steps,
device, devices, batch_size, minibatch_size, shuffle, val_size, val_interval,
autocast, checkpoint_interval, **kwargs) returning the node-averaged model;
LocalTrainer._build_connection).

Process-group setup (the north star's "process-group setup in trainer.py"):
  - one process per simulated node, `spawn` start method;
  - when every node has a GPU of its own (num_nodes <= len(devices)) the group
    is "nccl", i.e. RCCL over xGMI on ROCm, node i on devices[i]; the strategies
    then run their flat-arena collectives (reduce-scatter / all-gather /
    all-reduce) over RCCL;
  - more nodes than GPUs (and a multiple of them): one process per GPU hosts
    num_nodes / GPUs simulated nodes on a [K, ld] replica arena
    (gym_amd.replica, replicas_per_process="auto"), RCCL across the GPUs;
    their forward/backward passes run node by node (replica_forward="loop",
    the default) or as one torch.func.vmap over the arena rows
    (replica_forward="vmap", replica_vmap_chunk=nodes per vmap);
  - otherwise (or replicas_per_process=1) nodes share GPUs round-robin over a
    gloo group (RCCL cannot put two ranks on one GPU).
  - MASTER_ADDR is 127.0.0.1; device "cpu"/"mps" is refused (the step kernels
    are MI355X kernels, there is no CPU path).
The final average of the nodes' state dicts (trainer.py:95-119) runs on the GPU
through ga_replica_mean for floating tensors.
"""
import copy
import os
from abc import abstractmethod
from collections import OrderedDict
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional, Union

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from . import ops
from .strategy import Strategy
from .train_node import TrainNode


@dataclass
class TrainingConfig:
    model: torch.nn.Module
    train_dataset: Union[torch.utils.data.Dataset, Callable[[int, int, bool], torch.utils.data.Dataset]]
    val_dataset: Union[torch.utils.data.Dataset, Callable[[int, int, bool], torch.utils.data.Dataset]]
    strategy: Strategy
    num_epochs: int
    num_nodes: int
    max_steps: Optional[int] = None
    device: Optional[str] = None
    devices: Optional[List[int]] = None
    batch_size: int = 16
    minibatch_size: int = 16
    shuffle: bool = True
    val_size: int = 64
    val_interval: int = 100
    autocast: bool = False
    checkpoint_interval: int = 100
    trainer_class: type = None
    kwargs: Dict[str, Any] = None

    def __post_init__(self):
        if self.kwargs is None:
            self.kwargs = {}


_FIELDS = ("num_epochs", "max_steps", "strategy", "num_nodes", "device", "devices", "batch_size",
           "minibatch_size", "shuffle", "val_size", "val_interval", "autocast", "checkpoint_interval")


def _worker(rank: int, config: TrainingConfig, result_queue):
    trainer = config.trainer_class(model=config.model, train_dataset=config.train_dataset,
                                   val_dataset=config.val_dataset, **config.kwargs)
    for f in _FIELDS:
        setattr(trainer, f, getattr(config, f))
    state = trainer._fit_process(rank)
    log = trainer.run_log.summary() if getattr(trainer, "run_log", None) is not None else None
    result_queue.put((rank, OrderedDict((k, v.detach().cpu()) for k, v in state.items()), log))


def _replica_worker(rank: int, config: TrainingConfig, procs: int, K: int, result_queue):
    """One process per GPU hosting K simulated nodes (gym_amd.replica)."""
    from .replica import ReplicaTrainNode
    trainer = config.trainer_class(model=config.model, train_dataset=config.train_dataset,
                                   val_dataset=config.val_dataset, **config.kwargs)
    for f in _FIELDS:
        setattr(trainer, f, getattr(config, f))
    trainer.rank = rank
    trainer.world_size = procs
    trainer._build_connection()
    strategy = copy.deepcopy(trainer.strategy)
    node = ReplicaTrainNode(trainer.model_orig, trainer.train_dataset, trainer.val_dataset, strategy, trainer.device,
                            rank, trainer.num_nodes, K, num_epochs=trainer.num_epochs, max_steps=trainer.max_steps,
                            batch_size=trainer.batch_size, minibatch_size=trainer.minibatch_size,
                            val_size=trainer.val_size, val_interval=trainer.val_interval, shuffle=trainer.shuffle,
                            autocast=trainer.autocast, **trainer.kwargs)
    states = node.train()
    trainer._process_cleanup()
    log = node.logger.summary() if node.logger is not None else None
    for k, sd in enumerate(states):
        result_queue.put((rank * K + k, OrderedDict((n, v.detach().cpu()) for n, v in sd.items()),
                          log if k == 0 else None))


def _average_model_states(model_states: Dict[int, OrderedDict]) -> Optional[OrderedDict]:
    """Mean over nodes of every state-dict entry; integer entries are averaged
    in float and cast back (trainer.py:95-119)."""
    if not model_states:
        return None
    states = list(model_states.values())
    out = OrderedDict()
    for name in states[0].keys():
        stack = torch.stack([s[name] for s in states])
        if stack.dtype in (torch.float32, torch.bfloat16) and torch.cuda.is_available() and stack[0].numel() > 0:
            src = stack.reshape(len(states), -1).cuda()
            dst = torch.empty(src.shape[1], device=src.device, dtype=src.dtype)
            ops.replica_mean(src, dst)
            out[name] = dst.view(stack.shape[1:]).cpu()
        elif stack.dtype.is_floating_point or stack.dtype.is_complex:
            out[name] = torch.mean(stack, dim=0)
        else:
            out[name] = torch.mean(stack.float(), dim=0).to(stack.dtype)
    return out


class Trainer:
    def __init__(self, model: torch.nn.Module, train_dataset, val_dataset, start_port: Optional[int] = None,
                 **kwargs):
        self.model_orig = model
        self.train_dataset = train_dataset
        self.val_dataset = val_dataset
        self.kwargs = kwargs
        self.port = start_port if start_port is not None else 12355

    def fit(self, num_epochs: int, strategy: Strategy, num_nodes: int, max_steps: int = None, device: str = None,
            devices: List[int] = None, batch_size: int = 16, minibatch_size: int = 16, shuffle: bool = True,
            val_size: int = 64, val_interval: int = 100, autocast: bool = False, checkpoint_interval: int = 100,
            **kwargs):
        self.num_epochs, self.max_steps, self.strategy, self.num_nodes = num_epochs, max_steps, strategy, num_nodes
        self.device, self.devices, self.batch_size, self.minibatch_size = device, devices, batch_size, minibatch_size
        self.shuffle, self.val_size, self.val_interval = shuffle, val_size, val_interval
        self.autocast, self.checkpoint_interval = autocast, checkpoint_interval
        assert self.val_size // self.batch_size > 0, "val_size must be geq batch_size"
        self.kwargs.update(kwargs)
        self.port += 1
        config = TrainingConfig(model=copy.deepcopy(self.model_orig).cpu(), train_dataset=self.train_dataset,
                                val_dataset=self.val_dataset, strategy=strategy, num_epochs=num_epochs,
                                num_nodes=num_nodes, max_steps=max_steps, device=device, devices=devices,
                                batch_size=batch_size, minibatch_size=minibatch_size, shuffle=shuffle,
                                val_size=val_size, val_interval=val_interval, autocast=autocast,
                                checkpoint_interval=checkpoint_interval, trainer_class=self.__class__,
                                kwargs=self.kwargs)
        from .replica import replica_layout
        devs = devices if devices is not None else list(range(max(1, torch.cuda.device_count())))
        layout = replica_layout(num_nodes, devs, self.kwargs.pop("replicas_per_process", "auto"), strategy)
        # every node's final CPU state dict, kept on the trainer only when asked (K x model size of host memory)
        keep_node_states = bool(self.kwargs.pop("keep_node_states", False))
        config.kwargs = self.kwargs
        manager = mp.Manager()
        queue = manager.Queue()
        if layout is None:  # one process per simulated node (trainer.py:222-228)
            mp.spawn(_worker, args=(config, queue), nprocs=num_nodes, start_method="spawn", join=True)
        else:  # one process per GPU, K simulated nodes each on a [K, ld] replica arena
            procs, K = layout
            mp.spawn(_replica_worker, args=(config, procs, K, queue), nprocs=procs, start_method="spawn", join=True)
        states = {}
        self.run_log = None  # rank 0's record: train losses, evaluation losses, learning rates
        for _ in range(num_nodes):
            r, sd, log = queue.get()
            states[r] = sd
            if log is not None:
                self.run_log = log
        self.node_states = [states[r] for r in sorted(states)] if keep_node_states else None
        avg = _average_model_states(states)
        if avg is None:
            return None
        final = copy.deepcopy(self.model_orig)
        final.load_state_dict(avg)
        return final

    def _fit_process(self, rank):
        self.rank = rank
        self._build_connection()
        self.model = copy.deepcopy(self.model_orig).to(self.device)
        self.strategy = copy.deepcopy(self.strategy)
        self.strategy._init_node(self.model, self.rank, self.num_nodes)
        if callable(self.train_dataset):
            self.sampler = None
        else:
            self.sampler = torch.utils.data.DistributedSampler(self.train_dataset, num_replicas=self.num_nodes,
                                                               rank=self.rank, shuffle=self.shuffle)
        node = TrainNode(self.model, self.train_dataset, self.sampler, self.val_dataset, self.strategy, self.device,
                         self.rank, self.num_nodes, num_epochs=self.num_epochs, max_steps=self.max_steps,
                         batch_size=self.batch_size, minibatch_size=self.minibatch_size, val_size=self.val_size,
                         val_interval=self.val_interval, checkpoint_interval=self.checkpoint_interval,
                         autocast=self.autocast, **self.kwargs)
        state = node.train()
        self.run_log = node.logger
        self._process_cleanup()
        return state

    @abstractmethod
    def _build_connection(self):
        raise NotImplementedError

    def _process_cleanup(self):
        dist.destroy_process_group()


def select_backend(num_nodes, devices):
    """RCCL when every node gets its own GPU, else gloo (nodes share GPUs)."""
    return "nccl" if num_nodes <= len(devices) else "gloo"


class LocalTrainer(Trainer):
    def _build_connection(self):
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(self.port)
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if self.device in ("", None):
            self.device = "cuda"
        if self.device != "cuda" and not str(self.device).startswith("cuda"):
            raise ValueError(f"Invalid device type: {self.device} (gym_amd runs its strategy step on MI355X GPUs)")
        if not torch.cuda.is_available():
            raise RuntimeError("LocalTrainer: no GPU visible (gym_amd has no CPU path)")
        if self.devices is None:
            self.devices = list(range(torch.cuda.device_count()))
        world = getattr(self, "world_size", None) or self.num_nodes  # processes (< num_nodes with replicas)
        gpu = self.devices[self.rank % len(self.devices)]
        torch.cuda.set_device(gpu)
        backend = select_backend(world, self.devices)
        kw = {"device_id": torch.device(f"cuda:{gpu}")} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=self.rank, world_size=world, **kw)
        self.device = torch.device(f"cuda:{gpu}")
        from .placement import note_devices
        note_devices()  # placement is skipped on a GPU other ranks of the job share
