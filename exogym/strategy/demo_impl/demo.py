"""exogym.strategy.demo_impl.demo -> gym_amd.strategy.demo_impl.demo (the same module object: attribute look-ups,
monkeypatching and isinstance checks see gym_amd's implementation)."""
import sys

from gym_amd.strategy.demo_impl import demo as _impl

sys.modules[__name__] = _impl
