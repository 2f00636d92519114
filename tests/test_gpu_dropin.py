"""The drop-in schedule of tests/golden/dropin.npz (the reference's trainer
worker + TrainNode driving gym_amd strategies, tests/golden/gen_dropin.py)
replayed through exogym.LocalTrainer.fit on the MI355X: the HIP kernels, the
fused SPARTA draw from the CUDA generator, the model on the GPU.  The model's
own forward/backward now runs on the GPU (hipBLASLt vs the CPU), so the bar
is numerical: every parameter within 1e-4 relative + 1e-5, losses within
2e-4 relative; DeMo (sign-SGD) 99% of the elements, the rest off by at most
2 lr per step."""
import numpy as np
import pytest
import torch

import dropin_cases as D
from conftest import GOLDEN
from strategy_scenarios import free_port

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", D.NAMES)
def test_dropin_replay_on_gpu(name):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    z = np.load(f"{GOLDEN}/dropin.npz")
    states, log, final = D.run_gpu(name, free_port())
    D.check(z, name, states, log)
    for k, v in final.state_dict().items():  # the node-averaged model (trainer.py:95-119)
        want = z[f"{name}_avg_{k}"]
        err = np.abs(v.detach().cpu().numpy() - want)
        assert (err <= 1e-5 + 1e-4 * np.abs(want)).mean() >= (0.99 if name == "demo" else 1.0), (name, k)
