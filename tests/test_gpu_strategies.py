"""The Strategy classes end to end on the MI355X with the real gfx950 kernels:
2-3 node processes share cuda:0 over gloo and replay the reference's golden
harnesses (tests/golden/gen_golden.py).  SPARTA replays the reference's own
masks (a CUDA generator draws different bits than the CPU one the goldens
used); the Philox mode is checked against the oracle's Philox stream."""
import pytest
import torch

import strategy_scenarios as S
from conftest import GOLDEN
from scenario_checks import CHECKS

pytestmark = pytest.mark.gpu

CASES = [
    ("simple", 2, {}), ("simple", 3, {}), ("simple", 3, {"shard": True, "chunks": 3}),
    ("diloco", 3, {}), ("diloco", 3, {"shard": True}), ("diloco", 3, {"shard": True, "chunks": 5}),
    ("simple_adamw", 2, {}), ("simple_adamw", 3, {}),
    ("engine", 3, {}),
    ("sparta", 2, {"replay": True}), ("sparta", 3, {"replay": True}),
    ("sparta_philox", 2, {}),
    ("sparta_sel", 2, {"kind": "random"}), ("sparta_sel", 3, {"kind": "random"}),
    ("sparta_sel", 3, {"kind": "random", "rank_seeds": True}),
    ("sparta_sel", 2, {"kind": "shuffled"}), ("sparta_sel", 2, {"kind": "partitioned"}),
    ("sparta_sel", 3, {"kind": "philox"}),
    ("eval_avg", 2, {}), ("eval_avg", 3, {}),
    ("mnist_diloco", 2, {}),
    ("fedavg", 2, {}), ("fedavg", 3, {"island_size": 2}), ("fedavg", 4, {"island_size": 3}),
    ("demo", 2, {}), ("demo_pipe", 2, {}), ("demo_pipe", 3, {"pieces": 2}),
]


@pytest.mark.parametrize("name,world,kw", CASES, ids=[f"{c[0]}-w{c[1]}-{c[2]}" for c in CASES])
def test_strategy_on_gpu(tmp_path, name, world, kw):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = S.run(name, world, "cuda:0", False, str(tmp_path), GOLDEN, **kw)
    check_kw = {k: kw[k] for k in ("island_size", "kind", "rank_seeds") if k in kw}
    if name == "sparta_sel":
        check_kw["device"] = "cuda:0"
    CHECKS[name](res, world, GOLDEN, **check_kw)
