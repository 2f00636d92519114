"""Collectives on flat arenas.

Replaces the per-tensor wrappers of exogym/strategy/communicate.py:63-75: the
strategies here issue ONE collective per step over a whole arena (or a whole
packed payload), on the process group set up one process per GPU with the
"nccl" backend, which is RCCL over xGMI on ROCm.  The gloo backend (CPU tests,
or several nodes sharing a GPU) is supported with the same semantics: gloo has
no reduce-scatter, so those paths fall back to all-reduce.
"""
import torch
import torch.distributed as dist


class _Done:
    """Handle of a collective that already completed (synchronous paths)."""

    def wait(self):
        return True


DONE = _Done()


class Collective:
    """force_exchange=True issues the collectives even at world size 1 (the
    engines then take their multi-rank paths): lets a one-GPU box run the
    RCCL reduce-scatter / all-gather pipeline with its async Work handles
    (tests/test_gpu_rccl.py).  Default: world size 1 is a local no-op."""

    def __init__(self, group=None, force_exchange=False):
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.world = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
            self.backend = str(dist.get_backend(group)).lower()
        else:
            self.world, self.rank, self.backend = 1, 0, "none"
        if force_exchange and self.backend == "none":
            raise RuntimeError("Collective(force_exchange=True) needs an initialised process group")
        self.exchange = self.world > 1 or bool(force_exchange)

    @property
    def rccl(self):
        return self.backend == "nccl"

    # -- collectives (no-ops at world size 1) --------------------------------
    # With async_op=True the RCCL forms return the torch Work handle (its
    # wait() orders the CURRENT stream after the collective, the host does not
    # block); every other case runs synchronously and returns DONE.
    def all_reduce_(self, t, async_op=False):
        if self.exchange:
            w = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op and self.rccl)
            if async_op:
                return w if w is not None else DONE
        return DONE if async_op else t

    def broadcast_(self, t, src=0):
        if self.exchange:
            dist.broadcast(t, src=src, group=self.group)
        return t

    def reduce_scatter(self, shard_out, full, async_op=False):
        """shard_out = rank's shard of sum over ranks of `full` (full is scratch:
        the gloo fallback reduces it in place)."""
        if not self.exchange:
            if shard_out.data_ptr() != full.data_ptr():
                shard_out.copy_(full[: shard_out.numel()])
            return DONE if async_op else shard_out
        if self.rccl:
            w = dist.reduce_scatter_tensor(shard_out, full, op=dist.ReduceOp.SUM, group=self.group,
                                           async_op=async_op)
            if async_op:
                return w
        else:
            dist.all_reduce(full, op=dist.ReduceOp.SUM, group=self.group)
            per = shard_out.numel()
            shard_out.copy_(full[self.rank * per:(self.rank + 1) * per])
        return DONE if async_op else shard_out

    def all_gather_into(self, full, shard, async_op=False):
        """full[r*per:(r+1)*per] = shard of rank r.  `shard` may be the rank's
        own slice of `full` (in place)."""
        if not self.exchange:
            if full.data_ptr() != shard.data_ptr():
                full[: shard.numel()].copy_(shard)
            return DONE if async_op else full
        if self.rccl:
            w = dist.all_gather_into_tensor(full, shard, group=self.group, async_op=async_op)
            if async_op:
                return w
        else:
            per = shard.numel()
            parts = list(full.split(per))
            src = shard.clone() if shard.data_ptr() == parts[self.rank].data_ptr() else shard
            dist.all_gather(parts, src, group=self.group)
        return DONE if async_op else full


def world_and_rank(group=None):
    c = Collective(group)
    return c.world, c.rank
