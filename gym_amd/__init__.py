"""gym_amd — MI355X-native strategy communication step for EXO Gym.

Public surface mirrors the reference package `exogym` (exogym/__init__.py):
TrainNode, Trainer, LocalTrainer, plus `gym_amd.strategy` mirroring
`exogym.strategy`.  Kernels: gym_amd/csrc (gfx950 HIP) behind the C ABI in
include/gym_amd.h; host bindings: gym_amd/_lib.py, gym_amd/ops.py.
"""
__version__ = "0.1.0"


def __getattr__(name):
    # lazy: importing the package must not pull torch.distributed launch code
    if name == "TrainNode":
        from .train_node import TrainNode
        return TrainNode
    if name in ("Trainer", "LocalTrainer"):
        from . import trainer
        return getattr(trainer, name)
    raise AttributeError(name)


__all__ = ["TrainNode", "Trainer", "LocalTrainer"]
