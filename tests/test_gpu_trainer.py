"""End to end: LocalTrainer.fit with every strategy on the MI355X (two nodes
share cuda:0 over gloo, the reference's shared-GPU mode), checking that
training runs, the loss goes down and the returned model is the node average."""
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
