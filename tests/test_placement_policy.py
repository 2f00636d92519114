"""gym_amd.placement.policy (CPU): the per-owner opt-out, GA_PLACEMENT=0, and
the shared-GPU rule (more ranks than visible devices -> no placement); the
strategies record the option in __config__()."""
import os
import sys

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
