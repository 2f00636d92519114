"""Per-tensor collective wrappers with the signatures of
exogym/strategy/communicate.py:63-75, for callers outside the strategy step
(TrainNode's initial parameter broadcast and evaluation averaging).

The strategies themselves do not call these per tensor: they run one
collective over a flat arena (gym_amd/comm.py).  The reference's MPS staging
wrapper (communicate.py:4-60) has no MI355X counterpart.
"""
import torch.distributed as dist


def broadcast(tensor, src=0):
    return dist.broadcast(tensor, src=src)


def all_reduce(tensor, op=dist.ReduceOp.SUM):
    return dist.all_reduce(tensor, op=op)


def all_gather(tensor_list, tensor, group=None, async_op=False):
    return dist.all_gather(tensor_list, tensor, group=group, async_op=async_op)
