"""exogym.strategy.federated_averaging -> gym_amd.strategy.federated_averaging (the same module object: attribute look-ups,
monkeypatching and isinstance checks see gym_amd's implementation)."""
import sys

from gym_amd.strategy import federated_averaging as _impl

sys.modules[__name__] = _impl
