"""Drop-in under the reference's own caller.

tests/golden/dropin.npz was produced by the REFERENCE's trainer worker and
TrainNode (exogym/trainer.py:56-93,247-296; train_node.py:154-189,575-626)
driving gym_amd strategy objects for all five strategies, two nodes over gloo
(tests/golden/gen_dropin.py).  Here the same schedule runs through this
repository's exogym shim (gym_amd's Trainer worker / TrainNode) with the
kernels as oracle stand-ins: the final node states and rank 0's logged
losses must equal the reference caller's, bit for bit (same CPU model
arithmetic, same strategy objects)."""
import numpy as np
import pytest

import dropin_cases as D
from conftest import GOLDEN
from strategy_scenarios import free_port


@pytest.mark.parametrize("name", D.NAMES)
def test_dropin_replay_matches_reference_caller(name):
    z = np.load(f"{GOLDEN}/dropin.npz")
    assert int(z["steps"]) == D.STEPS and int(z["nodes"]) == D.NODES
    states, log = D.run_cpu(name, free_port())
    D.check(z, name, states, log, exact=True)
