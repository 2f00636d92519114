"""`exogym` import surface over gym_amd (drop-in for the reference package).

The reference's public names (exogym/__init__.py:3-6, exogym/strategy/__init__.py:3-22,
exogym/strategy/demo_impl/__init__.py:2-4) resolve to gym_amd's MI355X
implementation, so `from exogym import LocalTrainer` and
`from exogym.strategy import DiLoCoStrategy` work unchanged.  Every submodule
(exogym.trainer, exogym.strategy.sparta, ...) IS the gym_amd module of the same
name.  Not provided: exogym.logger (wandb/CSV logging, out of scope; gym_amd
records a run in memory) and SPARTADiLoCoStrategy (not importable in the
reference either: sparta_diloco.py:6).
"""
from gym_amd.train_node import TrainNode
from gym_amd.trainer import LocalTrainer, Trainer

__all__ = ["TrainNode", "Trainer", "LocalTrainer"]
