"""exogym.strategy -> gym_amd.strategy (names of exogym/strategy/__init__.py:3-12).

The reference's __all__ also lists "SPARTADiLoCoStrategy", whose import is
commented out (exogym/strategy/__init__.py:10,20), so `from exogym.strategy
import *` raises AttributeError there; here __all__ holds the names that exist.
"""
from gym_amd.strategy import (CommunicateOptimizeStrategy, DeMoStrategy, DiLoCoStrategy, FedAvgStrategy, OptimSpec,
                              SimpleReduceStrategy, SPARTAStrategy, Strategy)

__all__ = [
    "Strategy",
    "DiLoCoStrategy",
    "OptimSpec",
    "SPARTAStrategy",
    "FedAvgStrategy",
    "CommunicateOptimizeStrategy",
    "DeMoStrategy",
]
