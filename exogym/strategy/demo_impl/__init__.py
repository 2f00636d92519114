"""exogym.strategy.demo_impl (exogym/strategy/demo_impl/__init__.py:2-4)."""
from gym_amd.strategy.demo_impl.demo import DeMo

__all__ = ["DeMo"]
