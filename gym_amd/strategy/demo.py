"""DeMoStrategy: the DeMo optimizer as a Strategy.

API of exogym/strategy/demo.py:8-53: DeMoStrategy(compression_decay=0.999,
compression_topk=32, compression_chunk=64, weight_decay=0.0, **kwargs); the
optimizer is built in _init_node with custom_all_gather = communicate.all_gather
and lr = kwargs.get("lr", 0.001); step() = optimizer step + base step (no
clipping).
"""
from .communicate import all_gather
from .demo_impl.demo import DeMo
from .strategy import Strategy


class DeMoStrategy(Strategy):
    def __init__(self, compression_decay: float = 0.999, compression_topk: int = 32, compression_chunk: int = 64,
                 weight_decay: float = 0.0, **kwargs):
        super().__init__(**kwargs)
        self.compression_decay = compression_decay
        self.compression_topk = compression_topk
        self.compression_chunk = compression_chunk
        self.weight_decay = weight_decay

    def optimizer_kwargs(self):
        """DeMo's constructor kwargs as the reference builds them (demo.py:31-46),
        strategy_config.optimizer_kwargs applied last."""
        kw = {
            "compression_decay": self.compression_decay,
            "compression_topk": self.compression_topk,
            "compression_chunk": self.compression_chunk,
            "weight_decay": self.weight_decay,
            "custom_all_gather": all_gather,
            "lr": self.kwargs.get("lr", 0.001),
        }
        for opt in ("placement", "bf16_transform"):  # gym_amd options of the DeMo optimizer
            if opt in self.kwargs:
                kw[opt] = self.kwargs[opt]
        if hasattr(self, "strategy_config") and hasattr(self.strategy_config, "optimizer_kwargs"):
            kw.update(self.strategy_config.optimizer_kwargs)
        return kw

    def _init_node(self, model, rank, num_nodes):
        super()._init_node(model, rank, num_nodes)
        self.optim = DeMo(model.parameters(), **self.optimizer_kwargs())
        self.arena = self.optim.arena  # zero_grad() zeroes the gradient arena in place
        self.coll = self.optim.coll
        self._setup_scheduler()

    def step(self):
        self.optim.step()
        super().step()
