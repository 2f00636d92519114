"""One simulated node's training loop (caller of the strategy step).

Constructor and loop semantics of exogym/train_node.py:19-626: seeding (42),
dataset-or-factory handling, rank 0's initial parameters broadcast to every
node, gradient accumulation over batch_size // minibatch_size minibatches
with `grad /= batch_size / minibatch_size`, `strategy.zero_grad()` /
`strategy.step()`, evaluation every val_interval steps (rank 0 evaluates its
local model, rank 1 the node-averaged model), a barrier every step.

MI355X changes: the initial broadcast and the evaluation average run over the
strategy's flat parameter arena (one collective + one ga_replica_mean launch
instead of one per tensor).  Logging is a small in-memory recorder (the
reference's wandb/CSV loggers and its disabled checkpointing are out of scope).
"""
import copy
from typing import Callable, Union

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import DataLoader

from . import ops
from .strategy.communicate import all_reduce, broadcast
from .strategy.strategy import Strategy
from .utils import LogModule


class RunLog:
    """Rank 0's record of the run: train losses, evaluation losses, learning rates."""

    def __init__(self, strategy, max_steps):
        self.step = 0
        self.max_steps = max_steps
        self.train = []
        self.evals = []
        self.lrs = []
        strategy.lr_callbacks.append(self.log_lr)

    def log_train(self, loss):
        self.train.append((self.step, float(loss)))

    def log_loss(self, loss, name):
        self.evals.append((self.step, name, float(loss)))

    def log_lr(self, lr):
        self.lrs.append((self.step, float(lr)))

    def increment_step(self):
        self.step += 1

    def summary(self):
        """Plain lists (picklable through the trainer's result queue)."""
        return {"train": list(self.train), "evals": list(self.evals), "lrs": list(self.lrs)}


class TrainNode(LogModule):
    def __init__(self, model: torch.nn.Module,
                 train_dataset: Union[torch.utils.data.Dataset, Callable[[int, int, bool], torch.utils.data.Dataset]],
                 train_sampler: torch.utils.data.Sampler,
                 val_dataset: Union[torch.utils.data.Dataset, Callable[[int, int, bool], torch.utils.data.Dataset]],
                 strategy: Strategy, device: torch.device, rank: int, num_nodes: int, num_epochs: int,
                 max_steps: int = None, batch_size: int = 16, minibatch_size: int = 16, val_size: int = 64,
                 val_interval: int = 100, checkpoint_interval: int = 100, autocast: bool = False, **kwargs):
        seed = kwargs.get("seed", 42)
        torch.manual_seed(seed)
        torch.cuda.manual_seed(seed)
        np.random.seed(seed)
        self.model = model
        if callable(train_dataset):
            self.train_dataset = train_dataset(rank, num_nodes, False)
            self.train_sampler = None
        else:
            self.train_dataset = train_dataset
            self.train_sampler = train_sampler
        self.val_dataset = val_dataset(rank, num_nodes, True) if callable(val_dataset) else val_dataset
        self.strategy = strategy
        self.device = device
        self.rank = rank
        self.num_nodes = num_nodes
        self.num_epochs = num_epochs
        self.max_steps = max_steps
        self.batch_size = batch_size
        self.minibatch_size = minibatch_size
        self.val_size = val_size
        self.val_interval = val_interval
        self.autocast = autocast
        self.checkpoint_interval = checkpoint_interval
        self.kwargs = kwargs
        self.build_dataloaders()
        torch.manual_seed(42)
        torch.cuda.manual_seed(42)
        if self.num_nodes > 1:  # every node starts from rank 0's parameters
            arena = getattr(strategy, "arena", None)
            if arena is not None:
                broadcast(arena.flat, src=0)
            else:
                for p in self.model.parameters():
                    broadcast(p.data, src=0)
        self.local_step = 0
        self.epoch = 0
        self.logger = None

    def build_dataloaders(self):
        self.train_dataloader = DataLoader(self.train_dataset, batch_size=self.minibatch_size,
                                           sampler=self.train_sampler, shuffle=(self.train_sampler is None))
        self.val_dataloader = DataLoader(self.val_dataset, batch_size=self.minibatch_size, shuffle=True)
        self.train_data_iter = iter(self.train_dataloader)
        self.val_data_iter = iter(self.val_dataloader)

    def _get_batch(self, eval=False):
        if not eval or self.val_data_iter is None:
            try:
                batch = next(self.train_data_iter)
            except StopIteration:
                self.epoch += 1
                self.train_data_iter = iter(self.train_dataloader)
                batch = next(self.train_data_iter)
        else:
            try:
                batch = next(self.val_data_iter)
            except StopIteration:
                self.val_data_iter = iter(self.val_dataloader)
                batch = next(self.val_data_iter)
        if isinstance(batch, (tuple, list)):
            return tuple(x.to(self.device) for x in batch)
        return batch.to(self.device)

    def _forward(self, model, minibatch):
        if self.autocast:
            with torch.autocast(device_type=torch.device(self.device).type, dtype=torch.bfloat16):
                return model(minibatch)
        return model(minibatch)

    def _train_step(self):
        self.strategy.zero_grad()
        accum = self.batch_size // self.minibatch_size
        loss = None
        for _ in range(accum):
            loss = self._forward(self.model, self._get_batch())
            loss.backward()
        for p in self.model.parameters():
            if p.requires_grad and p.grad is not None:
                p.grad /= self.batch_size / self.minibatch_size
        self.strategy.step()
        if self.rank == 0 and self.logger is not None:
            self.logger.log_train(loss=loss.item())

    def _averaged_model(self):
        """A copy of the model holding the node-averaged parameters
        (train_node.py:183-189): one all-reduce of the arena + one division launch."""
        clone = copy.deepcopy(self.model)
        arena = getattr(self.strategy, "arena", None)
        if arena is None:
            for p in clone.parameters():
                all_reduce(p.data, op=dist.ReduceOp.SUM)
                p.data = p.data / dist.get_world_size()
            return clone
        avg = arena.flat.detach().clone()
        dist.all_reduce(avg, op=dist.ReduceOp.SUM)
        ops.replica_mean(avg, avg, divisor=dist.get_world_size())
        with torch.no_grad():
            for p, v in zip(clone.parameters(), arena.layout.views(avg)):
                p.copy_(v)
        return clone

    def _evaluate(self):
        if self.val_size == 0:
            return
        clone = self._averaged_model() if self.num_nodes > 1 else self.model
        this_model = None
        if self.rank == 0:
            this_model = self.model
        if self.rank == 1:
            this_model = clone
        loss_total = 0.0
        if this_model is not None:
            this_model.eval()
            accum = self.batch_size // self.minibatch_size
            with torch.no_grad():
                for _ in range(int(self.val_size / self.batch_size)):
                    for _ in range(accum):
                        loss_total += self._forward(this_model, self._get_batch(eval=True)).item() / accum
            this_model.train()
        n_eval = int(self.val_size / self.batch_size)
        if self.rank == 0 and self.logger is not None:
            self.logger.log_loss(loss=loss_total / n_eval, name="local")
        if self.num_nodes > 1:
            g = torch.empty(1, device=next(self.model.parameters()).device)
            if self.rank == 1:
                g[0] = loss_total / n_eval
            broadcast(g, src=1)
            if self.rank == 0 and self.logger is not None:
                self.logger.log_loss(loss=g.item(), name="global")

    def train(self):
        if self.max_steps is None:
            self.max_steps = self.num_epochs * len(self.train_dataloader) / (self.batch_size // self.minibatch_size)
        self.strategy.max_steps = self.max_steps
        if self.rank == 0:
            self.logger = RunLog(self.strategy, self.max_steps)
        while self.local_step < self.max_steps:
            if self.local_step % self.val_interval == 0:
                self._evaluate()
            self._train_step()
            self.local_step += 1
            if self.rank == 0:
                self.logger.increment_step()
            if self.num_nodes > 1:
                dist.barrier()
        self.strategy.finish()
        self._evaluate()
        return self.model.state_dict()

    def __config__(self):
        return super().__config__(remove_keys=["model", "train_dataloader", "val_dataloader", "strategy"])
