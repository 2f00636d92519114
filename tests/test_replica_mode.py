"""Batched-replica node loop (gym_amd.replica) == the process-per-node
strategies, on CPU with the oracle-backed kernel stand-ins (host logic: arena
rows, engines over K local nodes, per-node clipping, fused optimizer over the
replica set, gating); tests/test_gpu_replica.py runs the same with the kernels."""
import numpy as np
import pytest

import replica_scenarios as R

NAMES = ["simple", "diloco", "diloco_adam", "sparta", "sparta_philox", "fedavg", "fedavg_islands", "demo", "demo_frozen",
         "sparta_frozen"]


@pytest.fixture
def fake(monkeypatch):
    import fake_ops
    import gym_amd.engine as engine
    import gym_amd.fused_optim as fused_optim
    import gym_amd.replica as replica
    import gym_amd.strategy.demo_impl.demo as demo_mod
    import gym_amd.strategy.diloco as diloco
    import gym_amd.strategy.federated_averaging as fedavg
    import gym_amd.strategy.strategy as strategy
    for mod in (engine, diloco, fedavg, fused_optim, replica):
        monkeypatch.setattr(mod, "ops", fake_ops)
    monkeypatch.setattr(strategy, "require_gpu", lambda device: None)
    monkeypatch.setattr(demo_mod, "_REQUIRE_GPU", False)
    return fake_ops


@pytest.mark.parametrize("name", NAMES)
def test_replicas_match_process_per_node(tmp_path, fake, name):
    proc = R.run_process_mode(name, 3, "cpu", True, str(tmp_path))
    rep = R.run_replica_mode(name, 3, "cpu", True)
    R.compare(proc, rep)


@pytest.mark.parametrize("name", ["fedavg_islands", "simple"])
def test_replica_processes_match_process_per_node(tmp_path, name):
    """2 processes x 2 local nodes (gloo) == 4 processes of one node: FedAvg
    islands spanning the processes (the all-gather path) and the full average."""
    (tmp_path / "p").mkdir()
    (tmp_path / "r").mkdir()
    proc = R.run_process_mode(name, 4, "cpu", True, str(tmp_path / "p"))
    rep = R.run_replica_processes(name, 2, 2, "cpu", True, str(tmp_path / "r"))
    R.compare(proc, rep)


def test_diloco_outer_adam_replicas_bit_exact(tmp_path, fake):
    """A non-SGD outer optimizer runs in replica mode (ReplicaRunner.supports);
    two nodes: bit-identical to two processes (a sum of two is order-free)."""
    from gym_amd.replica import ReplicaRunner
    assert ReplicaRunner.supports(R.make_strategy("diloco_adam"))
    proc = R.run_process_mode("diloco_adam", 2, "cpu", True, str(tmp_path))
    rep = R.run_replica_mode("diloco_adam", 2, "cpu", True)
    R.compare(proc, rep, rtol=0, atol=0)


def test_replica_layout_rules():
    from gym_amd.replica import replica_layout
    from gym_amd.strategy import SPARTAStrategy
    s = R.make_strategy("simple")
    assert replica_layout(4, [0, 1, 2, 3], "auto", s) is None          # one node per GPU
    assert replica_layout(16, [0, 1, 2, 3], "auto", s) == (4, 4)       # 4 per GPU
    assert replica_layout(6, [0, 1, 2, 3], "auto", s) is None          # not a multiple: gloo path
    assert replica_layout(8, [0, 1], 4, s) == (2, 4)
    assert replica_layout(8, [0, 1], 1, s) is None
    assert replica_layout(8, [0], "auto", SPARTAStrategy()) == (1, 8)  # torch-drawn masks batch too
    assert replica_layout(8, [0], "auto", SPARTAStrategy(mask_source="philox")) == (1, 8)
    with pytest.raises(ValueError):
        replica_layout(8, [0], 4, s)  # 2 processes on 1 GPU


def test_consecutive_runs():
    """FedAvg islands write the island mean back once per run of consecutive member rows."""
    from gym_amd.replica import consecutive_runs
    assert consecutive_runs([]) == []
    assert consecutive_runs([4]) == [(4, 4)]
    assert consecutive_runs([0, 1, 2]) == [(0, 2)]
    assert consecutive_runs([0, 2, 3, 5, 6, 7, 9]) == [(0, 0), (2, 3), (5, 7), (9, 9)]


def test_replica_eval_average(fake):
    from oracle.reduce import mean_reduce
    avg, rows = R.replica_eval_average(3, "cpu", True)
    assert not np.array_equal(rows[0], rows[1])
    assert np.array_equal(avg, mean_reduce(list(rows)))
