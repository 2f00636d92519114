"""Optimizer specs: which torch.optim class to build, with which kwargs.

API and behaviour of exogym/strategy/optim.py:9-60: OptimSpec(cls, **kwargs),
OptimSpec.from_string(name, **kwargs) for adam/adamw/sgd/rmsprop/adagrad
(ValueError otherwise), .build(model), and ensure_optim_spec(optim, default,
**kwargs) which accepts None / str / OptimSpec (TypeError otherwise).
"""
from dataclasses import dataclass
from typing import Any, Dict, Optional, Type, Union

import torch

_BY_NAME = {
    "adam": torch.optim.Adam,
    "adamw": torch.optim.AdamW,
    "sgd": torch.optim.SGD,
    "rmsprop": torch.optim.RMSprop,
    "adagrad": torch.optim.Adagrad,
}


@dataclass(init=False)
class OptimSpec:
    cls: Type[torch.optim.Optimizer] = torch.optim.AdamW
    kwargs: Dict[str, Any] = None

    def __init__(self, cls: Type[torch.optim.Optimizer], **kwargs: Any):
        self.cls = cls
        self.kwargs = kwargs

    @classmethod
    def from_string(cls, name: str, **kwargs) -> "OptimSpec":
        key = name.lower()
        if key not in _BY_NAME:
            raise ValueError(f"Unknown optimizer '{name}'. Available options: {', '.join(_BY_NAME)}")
        return cls(_BY_NAME[key], **kwargs)

    def build(self, model):
        params = model.parameters() if hasattr(model, "parameters") else model
        return self.cls(params, **(self.kwargs or {}))


def ensure_optim_spec(optim: Union[str, OptimSpec, None], default: Optional[OptimSpec] = None,
                      **kwargs) -> OptimSpec:
    if optim is None:
        return default if default is not None else OptimSpec(torch.optim.AdamW, **kwargs)
    if isinstance(optim, str):
        return OptimSpec.from_string(optim, **kwargs)
    if isinstance(optim, OptimSpec):
        if kwargs:
            return OptimSpec(optim.cls, **{**(optim.kwargs or {}), **kwargs})
        return optim
    raise TypeError(f"Expected str, OptimSpec, or None, got {type(optim)}")
