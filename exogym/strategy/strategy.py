"""exogym.strategy.strategy -> gym_amd.strategy.strategy (the same module object: attribute look-ups,
monkeypatching and isinstance checks see gym_amd's implementation)."""
import sys

from gym_amd.strategy import strategy as _impl

sys.modules[__name__] = _impl
