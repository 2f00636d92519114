"""The bench's CPU baseline (oracle/torch_diloco.py: the reference's DiLoCo
outer step restated per tensor in torch over gloo) reproduces the reference's
own run (tests/golden/diloco.npz: 3 gloo nodes, 7 steps, H=2) bit for bit, so
the number bench.py reports is the reference algorithm's cost."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN


def _worker(rank, world, port, out_dir):
    from oracle.torch_diloco import TorchDiLoCoOuter
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        z = np.load(os.path.join(GOLDEN, "diloco.npz"))
        ns, calls, H = int(z["nshapes"]), int(z["calls"]), int(z["H"])
        params = [torch.from_numpy(z[f"init_{i}"].copy()) for i in range(ns)]
        eng = TorchDiLoCoOuter(params, rank, world)
        out = {}
        for call in range(calls):  # the golden harness: per-call drift, outer step when call % H == 0 and call > 0
            g = torch.Generator().manual_seed(1000 + 100 * rank + call)
            for p in params:
                p.add_(torch.randn(p.shape, generator=g) * 1e-3)
            if call % H == 0 and call > 0:
                eng.step()
            for i, p in enumerate(params):
                out[f"after_{call}_{i}"] = p.numpy().copy()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), **out)
    finally:
        dist.destroy_process_group()


def test_torch_restatement_matches_reference_golden(tmp_path):
    z = np.load(os.path.join(GOLDEN, "diloco.npz"))
    K = int(z["K"])
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_worker, args=(K, port, str(tmp_path)), nprocs=K, join=True)
    for r in range(K):
        got = np.load(os.path.join(tmp_path, f"r{r}.npz"))
        for call in range(int(z["calls"])):
            for i in range(int(z["nshapes"])):
                assert np.array_equal(got[f"after_{call}_{i}"], z[f"after_{call}_{i}"][r]), (r, call, i)


def test_time_outer_step_runs():
    from oracle.torch_diloco import time_outer_step
    t, threads = time_outer_step([(64, 32), (100,)], nodes=2, cores=2, steps=2, warmup=1)
    assert t > 0 and threads == 1


@pytest.mark.timeout(120)
def test_cpu_baseline_under_torchrun_env(monkeypatch):
    """bench.py under torchrun (the forced-exchange rehearsal) times the CPU
    baseline from a process whose environment names torchrun's agent store
    (TORCHELASTIC_USE_AGENT_STORE): the baseline's own gloo workers must not
    use it (they waited forever on a store nobody served)."""
    from oracle.torch_diloco import time_outer_step
    monkeypatch.setenv("TORCHELASTIC_USE_AGENT_STORE", "True")
    t, threads = time_outer_step([(64, 64), (128,)], nodes=2, cores=2, steps=2, warmup=1)
    assert t > 0 and threads == 1
