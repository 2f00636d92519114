"""exogym.utils -> gym_amd.utils (the same module object: attribute look-ups,
monkeypatching and isinstance checks see gym_amd's implementation)."""
import sys

from gym_amd import utils as _impl

sys.modules[__name__] = _impl
