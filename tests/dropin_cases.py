"""The drop-in schedule of tests/golden/dropin.npz (tests/golden/gen_dropin.py:
the reference's own trainer worker and TrainNode driving gym_amd strategies),
replayed through THIS repository's exogym shim (exogym.trainer / TrainNode =
gym_amd's): on CPU with the oracle stand-ins (tests/fake_ops.py) and on the
MI355X with the HIP kernels.  Test infrastructure."""
import os

import numpy as np
import torch
import torch.distributed as dist

STEPS, BATCH, MINIBATCH, VAL_SIZE, VAL_INTERVAL, NODES = 8, 32, 16, 32, 4, 2
NAMES = ("simple", "diloco", "sparta", "fedavg", "demo")


def strategies():
    """name -> gym_amd strategy object, configured as a reference user would
    (identical to what gen_dropin.py handed the reference's caller)."""
    from gym_amd.strategy import (DeMoStrategy, DiLoCoStrategy, FedAvgStrategy, OptimSpec, SPARTAStrategy,
                                  SimpleReduceStrategy)
    adamw = OptimSpec(torch.optim.AdamW, lr=3e-3)
    return {
        "simple": SimpleReduceStrategy(optim_spec=adamw, max_norm=1.0, lr_scheduler="lambda_cosine",
                                       lr_scheduler_kwargs={"warmup_steps": 2, "cosine_anneal": True}),
        "diloco": DiLoCoStrategy(optim_spec=adamw, H=3),
        "sparta": SPARTAStrategy(inner_optim=adamw, p_sparta=0.1),
        "fedavg": FedAvgStrategy(inner_optim=adamw, H=2),
        "demo": DeMoStrategy(lr=3e-3),
    }


def model_and_data():
    import tiny_models
    torch.manual_seed(7)
    return tiny_models.TinyMLP(), tiny_models.dataset(n=256, seed=3)


def gpu_stream_draw(selector, params, views, skip, iteration, state, bits=None, coll=None, defer=False):
    """The SPARTA mask a GPU run draws (ATen's HIP bernoulli per tensor from
    the CUDA generator: seed 42, offset from 0, +12 per call), on CPU
    (oracle.sparta.torch_gpu_bernoulli) -- the CPU replay's stand-in for the
    fused draw."""
    from oracle.sparta import torch_gpu_bernoulli
    off = getattr(state, "emu_offset", 0)
    for i, (p, v) in enumerate(zip(params, views)):
        if i in skip:
            v.zero_()
            continue
        m = torch_gpu_bernoulli(p.numel(), selector.p, 42, off)
        v.copy_(torch.from_numpy(m.astype(np.uint8)).view(v.shape))
        off += 12
    state.emu_offset = off
    state.mode = "torch"
    return None


from gym_amd.trainer import LocalTrainer as _LocalTrainer  # noqa: E402


class CpuStandInTrainer(_LocalTrainer):
    """gym_amd's LocalTrainer with a gloo/CPU connection (the stand-in kernels run on CPU)."""

    def _build_connection(self):
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(self.port)
        dist.init_process_group("gloo", rank=self.rank, world_size=self.num_nodes)
        self.device = torch.device("cpu")


def _cpu_node(rank, config, queue):
    import fake_ops
    fake_ops.install()
    import gym_amd.strategy.sparta as sp
    sp.draw_masks = gpu_stream_draw
    torch.set_num_threads(1)
    from gym_amd import trainer
    trainer._worker(rank, config, queue)


def run_cpu(name, port):
    """gym_amd's trainer worker -> Trainer._fit_process -> TrainNode.train, two
    nodes over gloo, kernels as the oracle stand-ins.  Returns ({rank: state},
    rank 0's run log)."""
    import torch.multiprocessing as mp
    from gym_amd.trainer import TrainingConfig
    model, ds = model_and_data()
    config = TrainingConfig(model=model, train_dataset=ds, val_dataset=ds, strategy=strategies()[name], num_epochs=1,
                            num_nodes=NODES, max_steps=STEPS, device="cpu", devices=None, batch_size=BATCH,
                            minibatch_size=MINIBATCH, shuffle=True, val_size=VAL_SIZE, val_interval=VAL_INTERVAL,
                            trainer_class=CpuStandInTrainer, kwargs={"start_port": port})
    manager = mp.Manager()
    queue = manager.Queue()
    mp.spawn(_cpu_node, args=(config, queue), nprocs=NODES, start_method="spawn", join=True)
    states, log = {}, None
    for _ in range(NODES):
        r, sd, lg = queue.get()
        states[r] = sd
        log = lg if lg is not None else log
    return states, log


def run_gpu(name, port):
    """exogym.LocalTrainer(...).fit(...) on cuda, one process per node (gloo:
    both nodes share the box's GPU), as a reference user calls it."""
    from exogym import LocalTrainer
    model, ds = model_and_data()
    tr = LocalTrainer(model, ds, ds, start_port=port)
    final = tr.fit(num_epochs=1, strategy=strategies()[name], num_nodes=NODES, max_steps=STEPS, device="cuda",
                   batch_size=BATCH, minibatch_size=MINIBATCH, val_size=VAL_SIZE, val_interval=VAL_INTERVAL,
                   replicas_per_process=1, keep_node_states=True)
    return dict(enumerate(tr.node_states)), tr.run_log, final


def check(z, name, states, log, exact=False):
    """The replay against the reference-caller fixture: every node's final
    parameters, and rank 0's logged train / local / global losses."""
    demo = name == "demo"
    for r in range(NODES):
        for k, v in states[r].items():
            want = z[f"{name}_node{r}_{k}"]
            got = v.detach().cpu().float().numpy()
            if exact:
                assert np.array_equal(got, want), (name, r, k, float(np.abs(got - want).max()))
                continue
            err = np.abs(got - want)
            lim = 1e-5 + 1e-4 * np.abs(want)
            if demo:  # sign-SGD: a sign decided by ~0 may flip (p off by 2 lr there)
                assert (err <= lim).mean() >= 0.99, (name, r, k, (err <= lim).mean())
                assert err.max() <= 2 * 3e-3 * STEPS + 1e-5, (name, r, k, err.max())
            else:
                assert (err <= lim).all(), (name, r, k, float(err.max()))
    train = np.array([loss for _, loss in log["train"]])
    want = z[f"{name}_train_loss"]
    assert len(train) == len(want) == STEPS
    if exact:
        assert np.array_equal(train.astype(np.float64), want), (name, train, want)
    else:
        np.testing.assert_allclose(train, want, rtol=2e-4 if not demo else 2e-3, atol=1e-6)
    evals = {}
    for step, kind, loss in log["evals"]:
        evals.setdefault(kind, []).append(loss)
    for kind in ("local", "global"):
        want = z[f"{name}_val_{kind}"]
        got = np.array(evals.get(kind, []))
        assert len(got) == len(want), (name, kind, got, want)
        if exact:
            assert np.array_equal(got.astype(np.float64), want), (name, kind, got, want)
        else:
            np.testing.assert_allclose(got, want, rtol=2e-4 if not demo else 2e-3, atol=1e-6)
