"""The fused reference draw's fallback is visible: when the
probe says ga_sparta_torch_bernoulli no longer matches this torch build's
bernoulli kernel, draw_masks warns once, takes torch's per-tensor kernels
(the same masks as the reference's torch.bernoulli(torch.full(shape, p))
sequence) and records which draw ran; ranks agree on one path."""
import warnings

import pytest
import torch

import gym_amd.strategy.sparta as sp


@pytest.fixture
def failing_probe(monkeypatch):
    monkeypatch.setattr(sp, "_probe_fused", lambda device: False)
    monkeypatch.setattr(sp, "_on_gpu", lambda params: True)  # take the GPU branch with CPU tensors
    monkeypatch.setattr(sp.MaskDraw, "use_graphs", False)
    monkeypatch.setattr(sp, "_FUSED_OK", {})
    monkeypatch.setattr(sp, "_FUSED_AGREED", {})
    monkeypatch.setattr(sp, "_FUSED_WARNED", set())


def _arena(shapes):
    n = sum(-(-int(torch.Size(s).numel()) // 64) * 64 for s in shapes)
    mask = torch.zeros(n, dtype=torch.uint8)
    views, o = [], 0
    for s in shapes:
        m = int(torch.Size(s).numel())
        views.append(mask[o:o + m].view(s))
        o += -(-m // 64) * 64
    return mask, views


def test_fallback_warns_once_and_records_torch(failing_probe):
    shapes = [(5, 7), (13,), (64, 3)]
    params = [torch.zeros(s) for s in shapes]
    mask, views = _arena(shapes)
    sel, state = sp.RandomIndexSelector(0.3), sp.MaskDraw()
    torch.manual_seed(3)
    with pytest.warns(RuntimeWarning, match="fused reference draw"):
        assert sp.draw_masks(sel, params, views, set(), 0, state) is None
    assert state.mode == "torch"
    got = [v.clone().bool() for v in views]
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # no second warning
        sp.draw_masks(sel, params, views, set(), 1, state)
    assert state.mode == "torch"
    torch.manual_seed(3)
    want = [torch.bernoulli(torch.full(s, 0.3)).bool() for s in shapes]
    assert all(torch.equal(g, w) for g, w in zip(got, want))


class _Coll:
    exchange = True
    group = None


def test_ranks_agree_with_min(failing_probe, monkeypatch):
    """A rank whose own probe passes still follows a rank whose probe failed:
    the results are combined with one MIN all-reduce per group."""
    monkeypatch.setattr(sp, "_probe_fused", lambda device: True)
    calls = []

    def fake_all_reduce(t, op=None, group=None):
        calls.append(op)
        t.fill_(0)  # another rank's probe failed

    monkeypatch.setattr(sp.dist, "all_reduce", fake_all_reduce)
    with pytest.warns(RuntimeWarning):
        assert sp.fused_draw_matches_torch("cpu", _Coll()) is False
    assert sp.fused_draw_matches_torch("cpu", _Coll()) is False
    assert calls == [sp.dist.ReduceOp.MIN]  # once per group
    assert sp.fused_draw_matches_torch("cpu") is True  # this rank's own probe, no exchange


def test_strategy_config_records_mask_draw():
    s = sp.SPARTAStrategy(p_sparta=0.01)
    assert "mask_draw" in s.__config__() and s.__config__()["mask_draw"] is None
