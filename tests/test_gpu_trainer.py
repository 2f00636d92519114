"""End to end: LocalTrainer.fit with every strategy on the MI355X (two nodes
share cuda:0 over gloo, the reference's shared-GPU mode), checking that
training runs, the loss goes down and the returned model is the node average."""
import numpy as np
import pytest
import torch

import tiny_models

pytestmark = pytest.mark.gpu


def _strategies():
    from gym_amd.strategy import (DeMoStrategy, DiLoCoStrategy, FedAvgStrategy, OptimSpec, SPARTAStrategy,
                                  SimpleReduceStrategy)
    sgd = OptimSpec(torch.optim.SGD, lr=0.1)
    return {
        "simple": SimpleReduceStrategy(optim_spec=sgd, max_norm=1.0),
        "diloco": DiLoCoStrategy(optim_spec=sgd, H=3),
        "sparta": SPARTAStrategy(inner_optim=sgd, p_sparta=0.05),
        "fedavg": FedAvgStrategy(inner_optim=sgd, H=2),
        "demo": DeMoStrategy(lr=0.01, compression_topk=8, compression_chunk=16),
    }


@pytest.mark.parametrize("name", ["simple", "diloco", "sparta", "fedavg", "demo"])
def test_local_trainer_fit(name):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gym_amd import LocalTrainer
    torch.manual_seed(0)
    model = tiny_models.TinyMLP()
    ds = tiny_models.dataset()
    tr = LocalTrainer(model, ds, ds, start_port=21000 + 7 * ["simple", "diloco", "sparta", "fedavg", "demo"].index(name))
    final = tr.fit(num_epochs=1, strategy=_strategies()[name], num_nodes=2, max_steps=12, device="cuda",
                   batch_size=32, minibatch_size=16, val_size=32, val_interval=6)
    assert final is not None
    x, y = ds.tensors
    with torch.no_grad():
        l0 = model((x, y)).item()
        l1 = final((x, y)).item()
    assert l1 < l0, (name, l0, l1)


def _np_state(sd):
    return {k: v.detach().cpu().numpy() for k, v in sd.items()}


@pytest.mark.parametrize("K", [2, 3, 8])
def test_final_state_average_kernel_matches_oracle(K):
    """Trainer._average_model_states on the kernel (floating entries) vs the
    oracle restatement of exogym/trainer.py:95-119, integer buffers included."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from collections import OrderedDict
    from gym_amd.trainer import _average_model_states
    from oracle.reduce import average_state_dicts
    g = torch.Generator().manual_seed(K)
    states = {}
    for r in range(K):
        m = tiny_models.TinyBN()
        sd = OrderedDict((k, v.clone()) for k, v in m.state_dict().items())
        for k in sd:
            if sd[k].dtype.is_floating_point:
                sd[k] = torch.randn(sd[k].shape, generator=g)
            else:
                sd[k] = torch.tensor(7 * r + 3, dtype=sd[k].dtype)
        states[r] = sd
    got = _average_model_states(states)
    want = average_state_dicts([_np_state(states[r]) for r in range(K)])
    for k, v in got.items():
        assert v.dtype == states[0][k].dtype and v.shape == states[0][k].shape
        if v.dtype.is_floating_point:
            np.testing.assert_allclose(v.numpy(), want[k], rtol=1e-6, atol=0)
            if K == 2:
                assert np.array_equal(v.numpy(), want[k])
        else:
            assert np.array_equal(v.numpy(), want[k]), (k, v, want[k])


@pytest.mark.parametrize("name", ["simple", "diloco"])
def test_fit_returns_the_node_average_with_bn_buffers(name):
    """Trainer.fit's returned model = the mean of the nodes' final state dicts
    (exogym/trainer.py:95-119, 241-243), BatchNorm running stats and the int64
    num_batches_tracked included."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gym_amd import LocalTrainer
    from oracle.reduce import average_state_dicts
    torch.manual_seed(1)
    model = tiny_models.TinyBN()
    ds = tiny_models.dataset()
    tr = LocalTrainer(model, ds, ds, start_port=21100 + 7 * ["simple", "diloco"].index(name))
    final = tr.fit(num_epochs=1, strategy=_strategies()[name], num_nodes=2, max_steps=5, device="cuda",
                   batch_size=32, minibatch_size=16, val_size=32, val_interval=100, keep_node_states=True)
    nodes = [_np_state(sd) for sd in tr.node_states]
    assert len(nodes) == 2
    assert not np.array_equal(nodes[0]["bn.running_mean"], nodes[1]["bn.running_mean"])  # nodes differ
    want = average_state_dicts(nodes)
    got = _np_state(final.state_dict())
    assert set(got) == set(want)
    for k in want:
        assert got[k].dtype == want[k].dtype
        np.testing.assert_allclose(got[k], want[k], rtol=1e-6, atol=0, err_msg=k)
    assert int(got["bn.num_batches_tracked"]) == int(nodes[0]["bn.num_batches_tracked"])
