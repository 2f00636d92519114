"""Golden fixture tests/golden/dropin.npz: the REFERENCE's own caller driving
gym_amd strategy objects (the north star's "drops into
train_node.py unchanged").

For each of the five strategies, two simulated nodes run the reference's
exogym.trainer._worker (trainer.py:56-93) -> LocalTrainer._fit_process
(trainer.py:247-296: _build_connection over gloo, strategy deep-copy,
_init_node, DistributedSampler) -> TrainNode.train (train_node.py:575-626:
evaluation every val_interval with the node-averaged deep copy
:183-189, _train_step :154-179 -- strategy.zero_grad(), gradient accumulation,
`grad /= batch_size / minibatch_size`, strategy.step() -- the reference's
CSVLogger with the strategy's lr_callbacks, dist.barrier() every step), with a
gym_amd strategy (gym_amd.strategy.*) as `strategy`.  The strategies' kernels
run through tests/fake_ops.py (the oracle on CPU: this container has no GPU).
Recorded: every node's final state dict, the reference's
_average_model_states of them (trainer.py:95-119), and rank 0's train /
validation losses and learning rates as the reference's CSVLogger wrote them.

The SPARTA mask is the one the reference draws ON THE GPU
(torch.bernoulli(torch.full(shape, p, device=cuda)) per tensor, generator seed
42 from TrainNode, offset +12 per draw): oracle.sparta.torch_gpu_bernoulli,
pinned against torch on the MI355X by tests/test_gpu_kernels.py -- so the
-m gpu replay (tests/test_gpu_dropin.py: the same schedule through the exogym
shim's Trainer/TrainNode on the HIP kernels) draws the same masks.

Run here only:  python tests/golden/gen_dropin.py
(/root/reference does not exist on the GPU box; only the .npz is read there).
"""
import csv
import json
import os
import socket
import sys
import tempfile

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(OUT))

# the reference's exogym must win over this repository's exogym/ shim
sys.path.insert(0, REF)
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.append(p)

from dropin_cases import (BATCH, MINIBATCH, NODES, STEPS, VAL_INTERVAL, VAL_SIZE,  # noqa: E402
                          gpu_stream_draw, model_and_data, strategies)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _node(rank, config, queue, name):
    """One simulated node: the reference's trainer worker with the kernels as
    CPU stand-ins (spawned: sys.path and cwd come from the parent)."""
    import fake_ops
    fake_ops.install()
    import gym_amd.strategy.sparta as sp
    sp.draw_masks = gpu_stream_draw
    from exogym import trainer as ref_trainer  # /root/reference/exogym/trainer.py
    assert ref_trainer.__file__.startswith(REF), ref_trainer.__file__
    torch.set_num_threads(1)
    ref_trainer._worker(rank, config, queue)


def run(name, strategy, port, workdir):
    import torch.multiprocessing as mp
    from exogym import trainer as ref_trainer
    model, ds = model_and_data()
    config = ref_trainer.TrainingConfig(
        model=model, train_dataset=ds, val_dataset=ds, strategy=strategy, num_epochs=1, num_nodes=NODES,
        max_steps=STEPS, device="cpu", devices=None, batch_size=BATCH, minibatch_size=MINIBATCH, shuffle=True,
        val_size=VAL_SIZE, val_interval=VAL_INTERVAL, autocast=False, checkpoint_interval=100,
        trainer_class=ref_trainer.LocalTrainer, kwargs={"start_port": port, "run_name": f"dropin_{name}"})
    manager = mp.Manager()
    queue = manager.Queue()
    cwd = os.getcwd()
    os.chdir(workdir)
    try:
        mp.spawn(_node, args=(config, queue, name), nprocs=NODES, start_method="spawn", join=True)
    finally:
        os.chdir(cwd)
    states = {}
    for _ in range(NODES):
        r, sd = queue.get()
        states[r] = sd
    avg = ref_trainer._average_model_states(states)
    out = {}
    for r in range(NODES):
        for k, v in states[r].items():
            out[f"{name}_node{r}_{k}"] = v.numpy()
    for k, v in avg.items():
        out[f"{name}_avg_{k}"] = v.numpy()
    run_dir = os.path.join(workdir, "logs", f"dropin_{name}")
    with open(os.path.join(run_dir, "train.csv")) as f:
        rows = list(csv.DictReader(f))
    out[f"{name}_train_step"] = np.array([int(r["step"]) for r in rows])
    out[f"{name}_train_loss"] = np.array([float(r["train_loss"]) for r in rows])
    out[f"{name}_train_lr"] = np.array([float(r["lr"]) if r.get("lr") else np.nan for r in rows])
    with open(os.path.join(run_dir, "validation.csv")) as f:
        vrows = list(csv.DictReader(f))
    out[f"{name}_val_step"] = np.array([int(r["step"]) for r in vrows])
    out[f"{name}_val_local"] = np.array([float(r["local_loss"]) if r.get("local_loss") else np.nan
                                         for r in vrows])
    out[f"{name}_val_global"] = np.array([float(r["global_loss"]) if r.get("global_loss") else np.nan
                                          for r in vrows])
    with open(os.path.join(run_dir, "config.json")) as f:  # the reference logger serialised our __config__
        cfg = json.load(f)
    out[f"{name}_config_strategy"] = np.array(json.dumps(cfg.get("strategy", {}), sort_keys=True))
    return out


def main():
    import exogym
    assert exogym.__file__.startswith(REF), f"imported {exogym.__file__}, not the reference"
    out = {"steps": np.array(STEPS), "batch_size": np.array(BATCH), "minibatch_size": np.array(MINIBATCH),
           "val_size": np.array(VAL_SIZE), "val_interval": np.array(VAL_INTERVAL), "nodes": np.array(NODES)}
    with tempfile.TemporaryDirectory() as wd:
        for name, strategy in strategies().items():
            out.update(run(name, strategy, free_port(), wd))
            print(name, "loss", out[f"{name}_train_loss"][-1], flush=True)
    np.savez_compressed(os.path.join(OUT, "dropin.npz"), **out)
    print("wrote", os.path.join(OUT, "dropin.npz"))


if __name__ == "__main__":
    main()
