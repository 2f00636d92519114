"""Multi-process (gloo, world size 2-3) runs of the Strategy classes on CPU,
with the kernels replaced by the oracle-backed stand-ins of tests/fake_ops.py:
checks the host orchestration of every strategy against the reference's
golden fixtures (the GPU twin of this file, test_gpu_strategies.py, runs the
same scenarios on the real kernels)."""
import pytest

import strategy_scenarios as S
from conftest import GOLDEN
from scenario_checks import CHECKS

CASES = [
    ("simple", 2, {}), ("simple", 3, {}), ("simple", 3, {"shard": True, "chunks": 3}),
    ("diloco", 3, {}), ("diloco", 3, {"shard": True}), ("diloco", 3, {"shard": True, "chunks": 5}),
    ("simple_adamw", 2, {}), ("simple_adamw", 3, {}),
    ("engine", 3, {}), ("engine", 2, {"chunks": 1}), ("engine", 1, {"force": True}),
    ("sparta", 2, {"replay": True}), ("sparta", 3, {"replay": False}),
    ("sparta_philox", 2, {}),
    ("sparta_sel", 2, {"kind": "random"}), ("sparta_sel", 3, {"kind": "random"}),
    ("sparta_sel", 3, {"kind": "random", "rank_seeds": True}),
    ("sparta_sel", 2, {"kind": "shuffled"}), ("sparta_sel", 2, {"kind": "partitioned"}),
    ("sparta_sel", 3, {"kind": "philox"}),
    ("eval_avg", 2, {}), ("eval_avg", 3, {}),
    ("mnist_diloco", 2, {}),
    ("fedavg", 2, {}), ("fedavg", 3, {"island_size": 2}), ("fedavg", 4, {"island_size": 2}),
    ("fedavg", 4, {"island_size": 3}),
    # many rounds: C(4, 2) = 6 sets > 2 -> world all-gather every round, no group created;
    # C(5, 2) = 10 sets <= 12: every round on cached sub-communicators (created as they appear);
    # C(5, 2) = 10 sets > 8: the world all-gather every round
    ("fedavg", 4, {"island_size": 2, "rounds": 12, "max_groups": 2}),
    ("fedavg", 5, {"island_size": 2, "rounds": 12, "max_groups": 12}),
    ("fedavg", 5, {"island_size": 2, "rounds": 6, "max_groups": 8}),
    ("demo", 2, {}), ("demo_pipe", 2, {}), ("demo_pipe", 3, {"pieces": 2}),
]


@pytest.mark.parametrize("name,world,kw", CASES, ids=[f"{c[0]}-w{c[1]}-{c[2]}" for c in CASES])
def test_strategy_orchestration_gloo(tmp_path, name, world, kw):
    res = S.run(name, world, "cpu", True, str(tmp_path), GOLDEN, **kw)
    check_kw = {k: kw[k] for k in ("island_size", "kind", "rank_seeds", "max_groups") if k in kw}
    if name == "sparta_sel":
        check_kw["device"] = "cpu"
    CHECKS[name](res, world, GOLDEN, **check_kw)
