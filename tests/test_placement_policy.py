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


def test_device_sharing_by_identity(monkeypatch, tmp_path):
    """note_devices(): sharing decided by the physical GPU's identity, not by
    counting ranks against visible devices; a per-rank pinning launcher (one
    visible device, HIP_VISIBLE_DEVICES set) is not taken for sharing by the
    fallback rule either."""
    monkeypatch.delenv("GA_PLACEMENT", raising=False)
    for v in placement._VISIBLE_ENVS:
        monkeypatch.delenv(v, raising=False)
    dist.init_process_group("gloo", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1)
    try:
        monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
        monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
        assert placement.device_shared()  # fallback rule: 4 ranks, 1 device
        monkeypatch.setenv("HIP_VISIBLE_DEVICES", "3")  # pinned per rank by the launcher
        assert not placement.device_shared()
        monkeypatch.delenv("HIP_VISIBLE_DEVICES")
        assert placement.note_devices() is False  # one rank: nobody shares its GPU
        assert not placement.device_shared()  # the identity answer wins over the count
        ids = iter(["h|gpu0"])
        monkeypatch.setattr(placement, "device_identity", lambda: next(ids, "h|gpu0"))
        monkeypatch.setattr(dist, "all_gather_object", lambda out, obj, group=None: out.__setitem__(
            slice(None), [obj, "h|gpu0", "h|gpu1"]))
        assert placement.note_devices() is True  # another rank drives the same card
        assert placement.policy(True) == (False, "GPU shared by several processes of the job")
    finally:
        dist.destroy_process_group()
        placement._SHARING = None
    assert not placement.device_shared()  # no process group


class _FakeBuf:
    made = 0

    def __init__(self, nbytes, dev):
        _FakeBuf.made += 1
        self.i = _FakeBuf.made

    def release(self):
        pass


def _choose(monkeypatch, times, **kw):
    monkeypatch.setattr(torch.cuda, "empty_cache", lambda: None)
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda dev=None: (1 << 40, 1 << 40))
    _FakeBuf.made = 0
    t = iter(times)
    return placement.choose(1 << 20, "cpu", lambda b: next(t), 1.0, 16, 0.3, kind=_FakeBuf, **kw)


def test_choose_budget(monkeypatch):
    """placement.choose's budget: with patience p the search stops after p
    candidates unless the best beats the baseline by > min_gain; a deadline
    in the past creates no candidate; the best found is kept either way."""
    best, times = _choose(monkeypatch, [0.995, 1.01, 0.99] + [0.5] * 20, patience=3)
    assert len(times) == 4 and best.i == 3  # three probed, 1% gain < 2%: stop, keep the best
    best, times = _choose(monkeypatch, [1.1, 0.9, 1.2, 0.95, 0.85] + [2.0] * 20, patience=3)
    assert len(times) == 16 and best.i == 5  # 10% gain: the search runs to max_candidates
    best, times = _choose(monkeypatch, [0.5] * 20, deadline=0.0)
    assert best is None and times == [1.0]
    best, times = _choose(monkeypatch, [1.0 + i / 100 for i in range(20)])
    assert best is None and len(times) == 16  # no budget: every candidate, none faster


def test_stopwatch_stamps_search_time():
    rec = placement.Stopwatch().stamp({"chosen": 0})
    assert rec["search_s"] >= 0.0
    assert placement.Stopwatch().stamp(None) is None
