"""Config extraction for logging (`Strategy.__config__`).

Behaviour matches exogym/utils.py:5-99 (LogModule.__config__ / extract_config):
a recursive, depth-limited walk that keeps primitives, lists (first 10
items), dicts (first 50 string keys) and public attributes of plain objects,
and replaces tensors / modules / optimizers / callables by short descriptions.
"""
import torch

_OPAQUE = (torch.Tensor, torch.nn.Module, torch.optim.Optimizer, torch.nn.Parameter, torch.dtype)


def _describe(obj):
    if isinstance(obj, torch.Tensor):
        return f"<Tensor {list(obj.shape)}>"
    if isinstance(obj, torch.nn.Module):
        return f"<Module {type(obj).__name__}>"
    if isinstance(obj, torch.optim.Optimizer):
        return f"<Optimizer {type(obj).__name__}>"
    return f"<{type(obj).__name__}>"


def extract_config(obj, max_depth=10, current_depth=0):
    if current_depth >= max_depth:
        return str(type(obj).__name__)
    if obj is None or isinstance(obj, (int, float, str, bool)):
        return obj
    nxt = current_depth + 1
    if isinstance(obj, (list, tuple)):
        return [extract_config(v, max_depth, nxt) for v in obj[:10]]
    if isinstance(obj, dict):
        out = {}
        for k, v in obj.items():
            if isinstance(k, str) and len(out) < 50:
                out[k] = extract_config(v, max_depth, nxt)
        return out
    if isinstance(obj, torch.device):
        return str(obj)
    if isinstance(obj, _OPAQUE):
        return _describe(obj)
    if callable(obj):
        return f"<function {getattr(obj, '__name__', 'unknown')}>"
    if hasattr(obj, "__dict__"):
        out = {}
        for k, v in obj.__dict__.items():
            if not k.startswith("_") and len(out) < 50:
                out[k] = extract_config(v, max_depth, nxt)
        return out
    return f"<{type(obj).__name__}>"


class LogModule:
    def __config__(self, remove_keys=None):
        cfg = extract_config(self)
        for k in remove_keys or ():
            cfg.pop(k, None)
        return cfg
