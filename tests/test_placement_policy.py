"""gym_amd.placement.policy (CPU): the per-owner opt-out, GA_PLACEMENT=0, and
the shared-GPU rule (more ranks than visible devices -> no placement); the
strategies record the option in __config__()."""
import os
import sys

import pytest
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gym_amd import placement  # noqa: E402
from gym_amd.strategy import DiLoCoStrategy, SimpleReduceStrategy  # noqa: E402


def test_policy_opt_out_and_env(monkeypatch):
    monkeypatch.delenv("GA_PLACEMENT", raising=False)
    assert placement.policy(True) == (True, None)
    assert placement.policy(False) == (False, "placement=False")
    monkeypatch.setenv("GA_PLACEMENT", "0")
    assert placement.policy(True) == (False, "GA_PLACEMENT=0")


def test_policy_skips_a_shared_gpu(monkeypatch, tmp_path):
    monkeypatch.delenv("GA_PLACEMENT", raising=False)
    monkeypatch.delenv("LOCAL_WORLD_SIZE", raising=False)
    assert not placement.device_shared()  # no process group
    dist.init_process_group("gloo", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1)
    try:
        monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
        assert not placement.device_shared()  # one rank on one GPU
        monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")  # four ranks on one card
        assert placement.device_shared()
        assert placement.policy(True) == (False, "GPU shared by several processes of the job")
        monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
        assert placement.policy(True) == (True, None)
    finally:
        dist.destroy_process_group()


def test_strategy_config_records_the_option():
    s = DiLoCoStrategy(placement=False, H=10)
    assert s.placement_opt is False
    cfg = s.__config__()
    assert cfg["placement"] == {"enabled": False, "records": {}}
    assert SimpleReduceStrategy().__config__()["placement"]["enabled"] is True


def test_replica_arena_relocate_params():
    """ReplicaArena.relocate_params (DiLoCoOuter's replica-set stage, through
    ReplicaRunner): the K rows move into the new buffer with their values,
    every model's parameters read the new rows, the gradients stay bound, and
    ArenaAdam (which reads the set from the arena) steps the moved rows."""
    import copy

    from gym_amd.arena import ReplicaArena, ReplicaSet
    torch.manual_seed(0)
    models = [torch.nn.Linear(6, 5) for _ in range(3)]
    for k, m in enumerate(models):
        with torch.no_grad():
            m.weight.add_(k)
    ra = ReplicaArena(models)
    before = [copy.deepcopy(m.state_dict()) for m in models]
    gptr = [p.grad.data_ptr() for p in ra.params]
    new = torch.full_like(ra.flat_set, float("nan"))
    ra.relocate_params(new)
    assert ra.flat_set is new
    ra.check_bound()
    lo, hi = new.data_ptr(), new.data_ptr() + 4 * new.numel()
    assert all(lo <= p.data_ptr() < hi for p in ra.params)
    assert [p.grad.data_ptr() for p in ra.params] == gptr
    for m, b in zip(models, before):
        for key, v in m.state_dict().items():
            assert torch.equal(v, b[key])
    with torch.no_grad():
        models[1].bias.fill_(7.0)  # a write through the model lands in the new set
    assert (new[1, ra.layout.offsets[1]:ra.layout.offsets[1] + 5] == 7.0).all()
    with pytest.raises(ValueError):
        ra.relocate_params(torch.zeros(2, ra.ld))
    rs = ReplicaSet(ra.layout, 2, "cpu")
    rs.data.normal_()
    keep = rs.data.clone()
    other = torch.zeros_like(rs.data)
    rs.relocate(other)
    assert rs.data is other and torch.equal(other, keep)


def test_replica_arena_relocate_grads():
    """ReplicaArena.relocate_grads (MeanReduce's placement through ReplicaRunner
    for SimpleReduce): the gradient rows move with their values and every
    model's .grad is the view of its new row; zero_grad keeps them bound."""
    from gym_amd.arena import ReplicaArena
    torch.manual_seed(1)
    models = [torch.nn.Linear(6, 5) for _ in range(3)]
    ra = ReplicaArena(models)
    for p in ra.params:
        p.grad.normal_()
    keep = ra.grad_set.clone()
    new = torch.full_like(ra.grad_set, float("nan"))
    ra.relocate_grads(new)
    assert ra.grad_set is new and torch.equal(new, keep)
    lo, hi = new.data_ptr(), new.data_ptr() + 4 * new.numel()
    assert all(lo <= p.grad.data_ptr() < hi for p in ra.params)
    ra.zero_grad()
    assert (new == 0).all() and all(lo <= p.grad.data_ptr() < hi for p in ra.params)
    ra.sync_grads()
    assert all(lo <= p.grad.data_ptr() < hi for p in ra.params)
