"""Batched replicas == process per node.

The same strategy, data and steps run two ways:
  - process mode: one process per simulated node over gloo, the Strategy
    classes (the reference's execution model, exogym/trainer.py:222-228);
  - replica mode: ONE process hosting all K nodes on a [K, ld] ReplicaArena
    (gym_amd.replica.ReplicaRunner).
Every node must end with the same parameters (up to fp32 summation order:
in-kernel ascending sums vs gloo's ring order).  CPU runs use the oracle
stand-ins of tests/fake_ops.py; GPU runs the real kernels.
"""
import os
import random

import numpy as np
import torch
import torch.distributed as dist

from strategy_scenarios import ShapeModel, free_port

SHAPES = [(66, 32), (128,), (96, 64), (3, 7)]
STEPS = 4


FROZEN = 2  # "<name>_frozen" scenarios freeze this tensor on every node


def _model(name, dev):
    m = ShapeModel(SHAPES, seed=5).to(dev)
    if name.endswith("_frozen"):
        m.ps[FROZEN].requires_grad_(False)
    return m


def make_strategy(name):
    name = name.removesuffix("_frozen")
    from gym_amd.strategy import (DeMoStrategy, DiLoCoStrategy, FedAvgStrategy, OptimSpec, SimpleReduceStrategy,
                                  SPARTAStrategy)
    if name == "simple":
        return SimpleReduceStrategy(optim_spec=OptimSpec(torch.optim.AdamW, lr=1e-2), max_norm=1.0)
    if name == "diloco":
        return DiLoCoStrategy(optim_spec=OptimSpec(torch.optim.AdamW, lr=1e-2), H=2)
    if name == "diloco_adam":  # a non-SGD outer optimizer (diloco.py:26-28): torch's Adam on the master
        return DiLoCoStrategy(optim_spec=OptimSpec(torch.optim.AdamW, lr=1e-2),
                              outer_optim_spec=OptimSpec(torch.optim.Adam, lr=0.05), H=2)
    if name == "sparta":  # the reference's torch-drawn masks (default)
        return SPARTAStrategy(inner_optim=OptimSpec(torch.optim.AdamW, lr=1e-2), p_sparta=0.1)
    if name == "sparta_philox":
        return SPARTAStrategy(inner_optim=OptimSpec(torch.optim.AdamW, lr=1e-2), p_sparta=0.1, mask_source="philox")
    if name == "fedavg":
        return FedAvgStrategy(inner_optim=OptimSpec(torch.optim.SGD, lr=0.05), H=2, max_norm=0.5)
    if name == "fedavg_islands":  # 3 nodes in islands of 2: a pair and a node alone, reshuffled every round
        return FedAvgStrategy(inner_optim=OptimSpec(torch.optim.SGD, lr=0.05), island_size=2, H=1, max_norm=0.5)
    if name == "demo":
        return DeMoStrategy(lr=1e-2, compression_topk=8)
    raise KeyError(name)


def node_grads(node, step):
    g = torch.Generator().manual_seed(9000 + 101 * node + step)
    return [torch.randn(*s, generator=g) * 0.2 for s in SHAPES]


def _set_grads(model, node, step, dev):
    with torch.no_grad():
        for p, g in zip(model.parameters(), node_grads(node, step)):
            if p.requires_grad:
                p.grad.copy_(g.to(dev))


def _proc_worker(rank, world, port, name, device, fake, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    if fake:
        import fake_ops
        fake_ops.install()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(42)
        random.seed(1234)  # FedAvg islands: rank 0's partner draw
        dev = torch.device(device)
        model = _model(name, dev)
        s = make_strategy(name)
        s._init_node(model, rank, world)
        for t in range(STEPS):
            s.zero_grad()
            _set_grads(model, rank, t, dev)
            s.step()
        np.savez(os.path.join(out_dir, f"p{rank}.npz"),
                 **{f"p_{i}": p.detach().float().cpu().numpy() for i, p in enumerate(model.parameters())})
    finally:
        dist.destroy_process_group()


def run_process_mode(name, world, device, fake, out_dir):
    import torch.multiprocessing as mp
    mp.spawn(_proc_worker, args=(world, free_port(), name, device, fake, out_dir), nprocs=world, join=True)
    res = []
    for r in range(world):
        with np.load(os.path.join(out_dir, f"p{r}.npz")) as f:
            res.append([f[f"p_{i}"] for i in range(len(SHAPES))])
    return res


def run_replica_mode(name, K, device, fake):
    """All K nodes in this process (no process group: world 1)."""
    from gym_amd.replica import ReplicaRunner
    torch.manual_seed(42)
    random.seed(1234)  # FedAvg islands: the first process's partner draw, as rank 0's
    dev = torch.device(device)
    models = [_model(name, dev) for _ in range(K)]
    runner = ReplicaRunner(make_strategy(name), models, rank=0, num_nodes=K)
    for t in range(STEPS):
        runner.zero_grad()
        for k, m in enumerate(models):
            _set_grads(m, k, t, dev)
        runner.step()
    return [[p.detach().float().cpu().numpy() for p in m.parameters()] for m in models]


def _replica_worker(rank, world, K, port, name, device, fake, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    if fake:
        import fake_ops
        fake_ops.install()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gym_amd.replica import ReplicaRunner
        torch.manual_seed(42)
        random.seed(1234)
        dev = torch.device(device)
        models = [_model(name, dev) for _ in range(K)]
        runner = ReplicaRunner(make_strategy(name), models, rank=rank, num_nodes=world * K)
        for t in range(STEPS):
            runner.zero_grad()
            for k, m in enumerate(models):
                _set_grads(m, rank * K + k, t, dev)
            runner.step()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"),
                 **{f"p_{k}_{i}": p.detach().float().cpu().numpy() for k, m in enumerate(models)
                    for i, p in enumerate(m.parameters())})
    finally:
        dist.destroy_process_group()


def run_replica_processes(name, world, K, device, fake, out_dir):
    """world processes over gloo, each hosting K nodes (node = rank * K + k)."""
    import torch.multiprocessing as mp
    mp.spawn(_replica_worker, args=(world, K, free_port(), name, device, fake, out_dir), nprocs=world, join=True)
    res = []
    for r in range(world):
        with np.load(os.path.join(out_dir, f"r{r}.npz")) as f:
            for k in range(K):
                res.append([f[f"p_{k}_{i}"] for i in range(len(SHAPES))])
    return res


def compare(proc, rep, rtol=1e-5, atol=2e-6):
    assert len(proc) == len(rep)
    for node, (a, b) in enumerate(zip(proc, rep)):
        for i, (x, y) in enumerate(zip(a, b)):
            np.testing.assert_allclose(y, x, rtol=rtol, atol=atol, err_msg=f"node {node} tensor {i}")


def replica_eval_average(K, device, fake):
    """ReplicaRunner.averaged_flat (the evaluation's node-averaged model,
    exogym/train_node.py:183-189, for the K local nodes) after one DiLoCo inner
    step (the nodes differ): returns (average, per-node arenas)."""
    from gym_amd.replica import ReplicaRunner
    torch.manual_seed(42)
    dev = torch.device(device)
    models = [ShapeModel(SHAPES, seed=5).to(dev) for _ in range(K)]
    runner = ReplicaRunner(make_strategy("diloco"), models, rank=0, num_nodes=K)
    runner.zero_grad()
    for k, m in enumerate(models):
        _set_grads(m, k, 0, dev)
    runner.step()
    avg = runner.averaged_flat()
    return avg.float().cpu().numpy(), runner.ra.flat_set.float().cpu().numpy()
