from .demo import DeMo

__all__ = ["DeMo"]
