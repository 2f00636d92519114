"""exogym.train_node -> gym_amd.train_node (the same module object: attribute look-ups,
monkeypatching and isinstance checks see gym_amd's implementation)."""
import sys

from gym_amd import train_node as _impl

sys.modules[__name__] = _impl
