"""Batched-replica node loop on the MI355X: the K nodes of one process on a
[K, ld] replica arena (real gfx950 kernels) end where K processes sharing the
GPU over gloo end (tests/replica_scenarios.py), for every supported strategy;
and LocalTrainer.fit runs end to end in replica mode."""
import pytest
import torch

import replica_scenarios as R

pytestmark = pytest.mark.gpu

NAMES = ["simple", "diloco", "diloco_adam", "sparta", "sparta_philox", "fedavg", "fedavg_islands", "demo", "demo_frozen",
         "sparta_frozen"]


@pytest.mark.parametrize("name", NAMES)
def test_replicas_match_process_per_node_gpu(tmp_path, name):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    proc = R.run_process_mode(name, 3, "cuda:0", False, str(tmp_path))
    rep = R.run_replica_mode(name, 3, "cuda:0", False)
    if name.startswith("demo") or name == "fedavg_islands":
        # DeMo: the same kernels on the same payloads (node order), one launch for K
        # replicas or K launches of one; FedAvg islands: the ascending-member fp32
        # sum / size on both paths: identical bits
        R.compare(proc, rep, rtol=0, atol=0)
        return
    R.compare(proc, rep)


def test_diloco_outer_adam_replicas_bit_exact_gpu(tmp_path):
    """DiLoCo with a non-SGD outer optimizer (torch Adam) in replica mode: two
    nodes in one process end bit-identical to two processes over gloo (a sum of
    two is order-free; the same inner kernel, division and torch Adam)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gym_amd.replica import ReplicaRunner
    assert ReplicaRunner.supports(R.make_strategy("diloco_adam"))
    proc = R.run_process_mode("diloco_adam", 2, "cuda:0", False, str(tmp_path))
    rep = R.run_replica_mode("diloco_adam", 2, "cuda:0", False)
    R.compare(proc, rep, rtol=0, atol=0)


@pytest.mark.parametrize("forward", ["loop", "vmap"])
def test_local_trainer_fit_replica_mode(forward):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tiny_models import TinyMLP, dataset
    from gym_amd.strategy import OptimSpec, SimpleReduceStrategy
    from gym_amd.trainer import LocalTrainer
    torch.manual_seed(0)
    model = TinyMLP()
    tr = LocalTrainer(model, dataset(256), dataset(64, seed=1), start_port=22400 if forward == "loop" else 22410)
    final = tr.fit(num_epochs=1, strategy=SimpleReduceStrategy(optim_spec=OptimSpec(torch.optim.AdamW, lr=1e-2)),
                   num_nodes=4, max_steps=6, devices=[0], batch_size=16, minibatch_size=8, val_size=16,
                   val_interval=3, replicas_per_process=4, replica_forward=forward, replica_vmap_chunk=2)
    assert final is not None
    for p in final.parameters():
        assert torch.isfinite(p).all()


def test_replica_eval_average_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import numpy as np
    from oracle.reduce import mean_reduce
    avg, rows = R.replica_eval_average(3, "cuda:0", False)
    assert not np.array_equal(rows[0], rows[1])
    assert np.array_equal(avg, mean_reduce(list(rows)))  # ascending in-kernel sum, true division: bit-exact


@pytest.mark.parametrize("strategy", ["simple", "sparta", "diloco", "fedavg"])
def test_replica_forward_vmap_matches_loop_gpu(strategy):
    """replica_forward="vmap" (one torch.func.vmap over the arena rows, BatchNorm
    and causal SDPA in the model) trains K = 3 nodes with the HIP kernels to the
    per-node loop's parameters (fp32 rounding of the batched GEMMs only)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from test_replica_vmap import _train, assert_states_close
    assert_states_close(_train("loop", "cuda:0", strategy), _train("vmap", "cuda:0", strategy))


@pytest.mark.parametrize("name", ["diloco", "simple", "fedavg", "demo"])
def test_replica_set_relocation_in_the_replica_loop(name):
    """ReplicaRunner at a size where placement runs (9.4M parameters per node,
    K = 4): the DiLoCo outer step may move the parameter set, SimpleReduce's mean
    the gradient set, FedAvg's mean the parameter set, the DeMo step all three of
    its parameter, gradient and delta sets (ReplicaArena.relocate_params /
    relocate_grads); the nodes end bit-identical to placement=False, every model
    reads its row of the current sets, and the fused AdamW steps the moved rows."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from strategy_scenarios import ShapeModel
    from gym_amd.replica import ReplicaRunner
    from gym_amd.strategy import DeMoStrategy, DiLoCoStrategy, FedAvgStrategy, OptimSpec, SimpleReduceStrategy
    shapes = [(2048, 2048), (2048, 2048), (1024, 1024), (300,)]

    def strategy(placed):
        if name == "diloco":
            return DiLoCoStrategy(optim_spec=OptimSpec(torch.optim.AdamW, lr=1e-3), H=2, placement=placed)
        if name == "simple":
            return SimpleReduceStrategy(optim_spec=OptimSpec(torch.optim.AdamW, lr=1e-3), placement=placed)
        if name == "demo":
            return DeMoStrategy(lr=1e-3, placement=placed)
        return FedAvgStrategy(inner_optim=OptimSpec(torch.optim.SGD, lr=0.05), H=2, placement=placed)

    def run(placed):
        torch.manual_seed(3)
        models = [ShapeModel(shapes, seed=5).to("cuda:0") for _ in range(4)]
        runner = ReplicaRunner(strategy(placed), models, rank=0, num_nodes=4)
        g = torch.Generator(device="cuda:0").manual_seed(11)
        for _ in range(5):
            runner.zero_grad()
            for m in models:
                for p in m.parameters():
                    p.grad.copy_(torch.randn(p.shape, device="cuda:0", generator=g) * 1e-2)
            runner.step()
        ra = runner.ra
        ra.check_bound()
        for buf, ts in ((ra.flat_set, [p.data for p in ra.params]), (ra.grad_set, [p.grad for p in ra.params])):
            lo, hi = buf.data_ptr(), buf.data_ptr() + 4 * buf.numel()
            assert all(lo <= t.data_ptr() < hi for t in ts)
        rec = {"diloco": lambda: runner.outer.placement, "demo": lambda: runner.placement}.get(
            name, lambda: runner.mean.placement)()
        if name == "demo" and runner._placed is not None and runner._placed[2] is not None:
            assert runner.delta.data_ptr() == runner._placed[2].tensor().data_ptr()  # the step's delta moved too
        return [p.detach().clone() for m in models for p in m.parameters()], rec

    placed, rec = run(True)
    cand = rec.get("replica_set", rec) if rec else {}
    assert max(cand.get("candidates", 0), cand.get("candidates_per_buffer", 0)) >= 2, rec
    plain, rec_off = run(False)
    assert rec_off == {"placed": False, "why": "placement=False"}
    for a, b in zip(placed, plain):
        assert torch.equal(a, b)
