"""exogym.strategy.communicate_optimize_strategy -> gym_amd.strategy.communicate_optimize_strategy (the same module object: attribute look-ups,
monkeypatching and isinstance checks see gym_amd's implementation)."""
import sys

from gym_amd.strategy import communicate_optimize_strategy as _impl

sys.modules[__name__] = _impl
