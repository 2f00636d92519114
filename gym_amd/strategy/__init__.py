"""Strategy API — same import surface as exogym.strategy (exogym/strategy/__init__.py:3-21).

SPARTADiLoCoStrategy is not provided: the reference's module cannot be
imported (sparta_diloco.py:6 imports a name that does not exist) and is
commented out of its package (__init__.py:10).
"""
from .communicate_optimize_strategy import CommunicateOptimizeStrategy, CommunicationModule
from .demo import DeMoStrategy
from .diloco import DiLoCoStrategy
from .federated_averaging import FedAvgStrategy
from .optim import OptimSpec, ensure_optim_spec
from .sparta import SPARTAStrategy
from .strategy import SimpleReduceStrategy, Strategy

__all__ = [
    "Strategy",
    "SimpleReduceStrategy",
    "DiLoCoStrategy",
    "OptimSpec",
    "SPARTAStrategy",
    "FedAvgStrategy",
    "CommunicateOptimizeStrategy",
    "DeMoStrategy",
]
