"""Multi-process strategy scenarios (one process per simulated node, gloo).

Each scenario replays the harness tests/golden/gen_golden.py ran against the
REFERENCE strategies, but through gym_amd's Strategy classes, and writes what
each rank ends with to <out>/r<rank>.npz.  The same code runs
  - on CPU with the oracle-backed kernel stand-ins (tests/fake_ops.py): checks
    the host orchestration (arenas, collectives, sharding, gating, masks);
  - on cuda:0 with the real gfx950 kernels (several ranks share the GPU over
    gloo): strategy-level parity of the product path.
"""
import os
import random
import socket

import numpy as np
import torch
import torch.distributed as dist


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class ShapeModel(torch.nn.Module):
    """Same construction as gen_golden.ShapeModel (so the initial values match)."""

    def __init__(self, shapes, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.ps = torch.nn.ParameterList(
            [torch.nn.Parameter(torch.randn(*s, generator=g) * 0.02) for s in shapes])


def _host(t):
    return t.detach().float().cpu().numpy().copy()


# ------------------------------------------------------------------ scenarios --
def sc_simple(rank, world, dev, golden_dir, shard=None, chunks=None):
    from gym_amd.strategy import OptimSpec, SimpleReduceStrategy
    z = np.load(os.path.join(golden_dir, "mean_reduce.npz"))
    shapes = [z[f"K{world}_in_{si}"].shape[1:] for si in range(4)]
    model = ShapeModel(shapes, seed=1).to(dev)
    s = SimpleReduceStrategy(optim_spec=OptimSpec(torch.optim.SGD, lr=0.0))
    s._init_node(model, rank, world)
    if shard is not None:  # the chunked reduce-scatter / divide / all-gather path, on gloo too
        from gym_amd.engine import MeanReduce
        a = s.arena
        s.engine = MeanReduce(s.coll, 1, a.n, a.device, a.dtype, shard=shard, chunks=chunks)
    s.zero_grad()
    for si, p in enumerate(model.parameters()):
        p.grad = torch.from_numpy(z[f"K{world}_in_{si}"][rank]).to(dev)  # not the arena view: sync_grads copies
    s.step()
    return {f"grad_{si}": _host(p.grad) for si, p in enumerate(model.parameters())}


def sc_diloco(rank, world, dev, golden_dir, shard=None, chunks=None):
    from gym_amd.strategy import DiLoCoStrategy, OptimSpec
    z = np.load(os.path.join(golden_dir, "diloco.npz"))
    ns, calls, H = int(z["nshapes"]), int(z["calls"]), int(z["H"])
    shapes = [z[f"init_{i}"].shape for i in range(ns)]
    model = ShapeModel(shapes, seed=1234).to(dev)
    s = DiLoCoStrategy(optim_spec=OptimSpec(torch.optim.SGD, lr=0.0), H=H)
    s._init_node(model, rank, world)
    if shard is not None:  # exercise the sharded (reduce-scatter/all-gather) path on gloo too
        from gym_amd.engine import DiLoCoOuter
        a = s.arena
        s.engine = DiLoCoOuter(s.coll, 1, a.n, a.device, a.dtype, shard=shard, chunks=chunks)
        s.engine.init_master(a.flat)
    out = {}
    for call in range(calls):
        g = torch.Generator().manual_seed(1000 + 100 * rank + call)
        with torch.no_grad():
            for p in model.parameters():
                p.add_((torch.randn(p.shape, generator=g) * 1e-3).to(dev))
        s.zero_grad()
        s.step()
        for i, p in enumerate(model.parameters()):
            out[f"after_{call}_{i}"] = _host(p)
    return out


class _ReplaySelector:
    """Index selector that replays the masks the reference drew (rank 0's)."""

    def __init__(self, z, K, shapes, p):
        self.z, self.K, self.shapes, self.p, self.calls = z, K, shapes, p, 0
        self.state = {}

    def get_indices(self, param, iteration):
        i = self._i
        self._i += 1
        n = int(np.prod(self.shapes[i]))
        m = np.unpackbits(self.z[f"K{self.K}_mask_{iteration}_{i}"])[:n].astype(bool).reshape(self.shapes[i])
        return torch.from_numpy(m).to(param.device)


def sc_sparta(rank, world, dev, golden_dir, replay=True):
    from gym_amd.strategy import OptimSpec, SPARTAStrategy
    z = np.load(os.path.join(golden_dir, "sparta.npz"))
    ns, calls, p = int(z["nshapes"]), int(z["calls"]), float(z["p"])
    shapes = [z[f"K{world}_before_0_{i}"].shape[1:] for i in range(ns)]
    torch.manual_seed(42)
    model = ShapeModel(shapes, seed=77 + rank).to(dev)
    s = SPARTAStrategy(inner_optim=OptimSpec(torch.optim.SGD, lr=0.0), p_sparta=p, mask_source="torch")
    s._init_node(model, rank, world)
    comm = s.communication_modules[0]
    if replay:
        sel = _ReplaySelector(z, world, shapes, p)
        comm.index_selector = sel
    out = {}
    for call in range(calls):
        if replay:
            sel._i = 0
        s.zero_grad()
        s.step()
        for i, prm in enumerate(model.parameters()):
            out[f"after_{call}_{i}"] = _host(prm)
    return out


def sc_sparta_philox(rank, world, dev, golden_dir):
    """Philox mode: every rank must derive the same mask; the result is
    checked against the oracle's Philox mask + sparse average."""
    from gym_amd.strategy import OptimSpec, SPARTAStrategy
    shapes = [(66, 32), (128,), (96, 64), (3, 7)]
    torch.manual_seed(42)
    model = ShapeModel(shapes, seed=77 + rank).to(dev)
    s = SPARTAStrategy(inner_optim=OptimSpec(torch.optim.SGD, lr=0.0), p_sparta=0.05, mask_source="philox")
    s._init_node(model, rank, world)
    out = {"before": _host(s.arena.flat)}
    s.zero_grad()
    s.step()
    s.zero_grad()
    s.step()
    out["after"] = _host(s.arena.flat)
    out["seed"] = np.array(s.communication_modules[0]._seed, dtype=np.int64)
    out["n"] = np.array(s.arena.n)
    return out


SEL_SHAPES = [(66, 32), (128,), (5, 9), (96, 64), (3, 7)]
SEL_FROZEN = 2  # a requires_grad=False tensor: never averaged (sparta.py:29-30)
SEL_P = {"random": 0.05, "shuffled": 0.1, "partitioned": 0.25, "philox": 0.05}
SEL_STEPS = 5


def make_selector(kind):
    from gym_amd.strategy.sparta import (PartitionedIndexSelector, RandomIndexSelector,
                                         ShuffledSequentialIndexSelector)
    p = SEL_P[kind]
    if kind == "shuffled":
        return ShuffledSequentialIndexSelector(p)
    if kind == "partitioned":
        return PartitionedIndexSelector(p)
    return RandomIndexSelector(p, mask_source="philox" if kind == "philox" else "torch")


def sc_sparta_sel(rank, world, dev, golden_dir, kind="random", rank_seeds=False):
    """SparseCommunicator with each index selector, driven the way a reference
    user builds it (CommunicateOptimizeStrategy([SparseCommunicator(sel)])),
    plus a frozen tensor that must be left alone.  rank_seeds: every rank
    seeds its generator differently -- rank 0's masks must still win
    (sparta.py:32-37) and every rank's generator must advance by its own
    draws."""
    from gym_amd.strategy import CommunicateOptimizeStrategy, OptimSpec
    from gym_amd.strategy.sparta import SparseCommunicator
    torch.manual_seed(42 + (rank if rank_seeds else 0))  # TrainNode seeds every rank (train_node.py:50-53)
    model = ShapeModel(SEL_SHAPES, seed=300 + rank).to(dev)
    model.ps[SEL_FROZEN].requires_grad_(False)
    comm = SparseCommunicator(make_selector(kind))
    s = CommunicateOptimizeStrategy([comm], inner_optim=OptimSpec(torch.optim.SGD, lr=0.0))
    s._init_node(model, rank, world)
    out = {}
    for step in range(SEL_STEPS):
        out[f"before_{step}"] = [_host(p) for p in model.parameters()]
        s.zero_grad()
        s.step()
        out[f"after_{step}"] = [_host(p) for p in model.parameters()]
    s.finish()
    out["mask_draw"] = [np.array(str(s.__config__().get("mask_draw")))]
    if kind == "philox":
        out["seed"] = [np.array(comm._seed, dtype=np.int64)]
        out["offsets"] = [np.array(s.arena.layout.offsets, dtype=np.int64)]
    if torch.device(dev).type == "cuda":
        gen = torch.cuda.default_generators[torch.device(dev).index or 0]
        out["gen"] = [np.array([gen.initial_seed(), gen.get_offset()], dtype=np.uint64)]
    return {f"{k}_{i}": v for k, lst in out.items() for i, v in enumerate(lst)}


def sc_eval_avg(rank, world, dev, golden_dir):
    """TrainNode._averaged_model (the evaluation's node-averaged clone,
    exogym/train_node.py:183-189) over the strategy's arena: the clone holds
    the mean of every node's parameters; the node's own model is untouched."""
    import tiny_models
    from gym_amd.strategy import OptimSpec, SimpleReduceStrategy
    from gym_amd.train_node import TrainNode
    model = ShapeModel([(66, 32), (128,), (3, 7)], seed=600 + rank).to(dev)
    s = SimpleReduceStrategy(optim_spec=OptimSpec(torch.optim.SGD, lr=0.0))
    s._init_node(model, rank, world)
    ds = tiny_models.dataset(n=64)
    node = TrainNode(model, ds, None, ds, s, dev, rank, world, num_epochs=1, max_steps=1)
    g = torch.Generator().manual_seed(700 + rank)
    with torch.no_grad():  # the constructor broadcast rank 0's parameters: make the nodes differ again
        for p in model.parameters():
            p.add_((torch.randn(p.shape, generator=g) * 0.1).to(dev))
    before = [_host(p) for p in model.parameters()]
    clone = node._averaged_model()
    return {**{f"own_{i}": v for i, v in enumerate(before)},
            **{f"avg_{i}": _host(p) for i, p in enumerate(clone.parameters())},
            **{f"after_{i}": _host(p) for i, p in enumerate(model.parameters())}}


def sc_mnist_diloco(rank, world, dev, golden_dir, steps=5, H=2):
    """configs[0]: the MNIST CNN under DiLoCoStrategy (H=2), real forward/backward on each node's synthetic MNIST-shaped
    batch, default AdamW inner optimizer (outer steps at local_step 2 and 4,
    diloco.py:62).  Records each node's parameters right
    before each outer step and after it (the checker replays the outer step
    in the oracle)."""
    import tiny_models
    from gym_amd.strategy import DiLoCoStrategy
    torch.manual_seed(0)
    model = tiny_models.MnistCNN().to(dev)  # identical start on every node (TrainNode broadcasts rank 0's)
    s = DiLoCoStrategy(H=H)
    s._init_node(model, rank, world)
    assert sum(p.numel() for p in model.parameters()) == 1_868_234
    rec = {}
    eng = s.engine

    class Tap:
        def __call__(self, reps):
            rec[f"pre_{len(rec)}"] = _host(reps[0])
            return eng(reps)
    s.engine = Tap()
    ds = tiny_models.mnist_like(n=16 * steps, seed=100 + rank)
    out = {"init": _host(s.arena.flat)}
    for t in range(steps):
        s.zero_grad()
        x, y = ds.tensors
        loss = model((x[16 * t:16 * (t + 1)].to(dev), y[16 * t:16 * (t + 1)].to(dev)))
        loss.backward()
        s.step()
        out[f"after_{t}"] = _host(s.arena.flat)
    out.update(rec)
    return out


def sc_fedavg(rank, world, dev, golden_dir, island_size=None, rounds=2, max_groups=None):
    import gym_amd.strategy.federated_averaging as fa
    from gym_amd.strategy import FedAvgStrategy, OptimSpec
    if max_groups is not None:  # bound the island sub-communicator cache
        fa.MAX_ISLAND_GROUPS = max_groups
    shapes = [(66, 32), (128,), (3, 7)]
    model = ShapeModel(shapes, seed=500 + rank).to(dev)
    random.seed(1234)  # rank 0's island shuffle (the reference leaves `random` unseeded)
    s = FedAvgStrategy(inner_optim=OptimSpec(torch.optim.SGD, lr=0.0), island_size=island_size, H=1)
    s._init_node(model, rank, world)
    out = {"before": [_host(p) for p in model.parameters()]}
    s.zero_grad()
    s.step()  # local_step 0: no communication
    out["after0"] = [_host(p) for p in model.parameters()]
    ngroups = []
    for step in range(1, rounds + 1):  # average every step (new islands: new or cached sub-communicators)
        s.zero_grad()
        s.step()
        out[f"after{step}"] = [_host(p) for p in model.parameters()]
        ngroups.append(len(s.communication_modules[0]._groups))
    res = {f"{k}_{i}": v for k, lst in out.items() for i, v in enumerate(lst)}
    res["ngroups"] = np.array(ngroups)
    res["rounds"] = np.array(rounds)
    return res


def sc_demo(rank, world, dev, golden_dir):
    from gym_amd.strategy.communicate import all_gather
    from gym_amd.strategy.demo_impl.demo import DeMo
    z = np.load(os.path.join(golden_dir, "demo_steps.npz"))
    ns, steps = int(z["nshapes"]), int(z["steps"])
    shapes = [z[f"p_before_0_{i}"].shape for i in range(ns)]
    model = ShapeModel(shapes, seed=4321).to(dev)
    opt = DeMo(model.parameters(), compression_decay=float(z["decay"]), compression_topk=int(z["topk"]),
               compression_chunk=int(z["chunk"]), weight_decay=float(z["wd"]), custom_all_gather=all_gather,
               lr=float(z["lr"]))
    out = {}
    for step in range(steps):
        # start every step from the reference's state (errors do not compound)
        with torch.no_grad():
            for i, p in enumerate(model.parameters()):
                p.copy_(torch.from_numpy(z[f"p_before_{step}_{i}"]).to(dev))
                opt.demo_state[p]["delta"].copy_(torch.from_numpy(z[f"delta_before_{step}_{i}"][rank]).to(dev))
                p.grad = torch.from_numpy(z[f"grad_{step}_{i}"][rank]).to(dev)
        opt.step()
        for i, p in enumerate(model.parameters()):
            out[f"p_{step}_{i}"] = _host(p)
            out[f"delta_{step}_{i}"] = _host(opt.demo_state[p]["delta"])
            out[f"sign_{step}_{i}"] = _host(p.grad)
        out[f"tx_{step}"] = np.array(opt.data_transmit)
        out[f"rx_{step}"] = np.array(opt.data_receive)
    return out


def _adamw_grads(rank, step, shapes):
    g = torch.Generator().manual_seed(500 + 97 * rank + step)
    return [torch.randn(*sh, generator=g) * 0.3 for sh in shapes]


ADAMW_SHAPES = [(66, 32), (128,), (3, 7)]


def sc_simple_adamw(rank, world, dev, golden_dir, steps=3):
    """SimpleReduce with the default-class inner optimizer (AdamW, fused on the
    arena) and gradient clipping: strategy.py:128-142 end to end."""
    from gym_amd.strategy import OptimSpec, SimpleReduceStrategy
    model = ShapeModel(ADAMW_SHAPES, seed=11).to(dev)
    s = SimpleReduceStrategy(optim_spec=OptimSpec(torch.optim.AdamW, lr=3e-3, weight_decay=0.05), max_norm=0.5)
    s._init_node(model, rank, world)
    out = {"fused": np.array(type(s.optim).__name__ == "ArenaAdam")}
    for step in range(steps):
        s.zero_grad()
        for p, g in zip(model.parameters(), _adamw_grads(rank, step, ADAMW_SHAPES)):
            p.grad.copy_(g.to(dev))
        s.step()
    for i, p in enumerate(model.parameters()):
        out[f"p_{i}"] = _host(p)
    return out


def engine_node(j, n, salt=0):
    """Node j's synthetic arena for the batched-replica engine scenario."""
    g = np.random.default_rng(100 + 1000 * salt + j)
    return (g.standard_normal(n) * 0.02).astype(np.float32)


def sc_engine(rank, world, dev, golden_dir, K_local=3, chunks=4, force=False):
    """Batched replicas on every rank (K_local nodes per process) through the
    sharded, chunk-pipelined exchange: DiLoCo outer steps and the mean reduce.
    force=True issues the collectives even at world size 1 (Collective
    force_exchange: the RCCL pipeline on a one-GPU box), and adds SPARTA
    (select -> all-reduce -> scatter) and DeMo (encode -> all-gather -> decode)
    through their multi-rank paths."""
    from gym_amd.comm import Collective
    from gym_amd.engine import DiLoCoOuter, MeanReduce
    coll = Collective(force_exchange=force)
    n = world * 64 * 10
    nodes = range(rank * K_local, (rank + 1) * K_local)
    reps = torch.from_numpy(np.stack([engine_node(j, n) for j in nodes])).to(dev)
    out = {}
    eng = DiLoCoOuter(coll, K_local, n, dev, torch.float32, shard=True, chunks=chunks)
    eng.init_master(torch.from_numpy(engine_node(0, n)).to(dev))
    eng(reps)
    out["d1"] = _host(reps)
    reps += torch.from_numpy(np.stack([engine_node(j, n, salt=1) for j in nodes]) * np.float32(0.05)).to(dev)
    eng(reps)
    out["d2"] = _host(reps)
    for tag, shard in (("m_shard", True), ("m_plain", False)):
        r2 = torch.from_numpy(np.stack([engine_node(j, n, salt=2) for j in nodes])).to(dev)
        MeanReduce(coll, K_local, n, dev, torch.float32, shard=shard, chunks=3)(r2)
        out[tag] = _host(r2)
    if force:
        from gym_amd.engine import DeMoCodec, Sparta
        from gym_amd.arena import ArenaLayout
        r3 = torch.from_numpy(np.stack([engine_node(j, n, salt=3) for j in nodes])).to(dev)
        sp = Sparta(coll, K_local, n, dev, torch.float32, 0.05)
        sp(r3, seed=77, iteration=5)
        sp.check()
        out["sparta"] = _host(r3)
        L = ArenaLayout([(128, 128), (768,)])
        P = torch.zeros(K_local, L.n, device=dev)
        D = torch.zeros(K_local, L.n, device=dev)
        G = torch.from_numpy(np.stack([engine_node(j, L.n, salt=4) for j in nodes])).to(dev)
        for k in range(K_local):  # zero padding, as the arena keeps it
            for o, m, o2 in zip(L.offsets, L.numels, L.offsets[1:] + [L.n]):
                G[k, o + m:o2] = 0
        out["demo_g"] = _host(G)
        codec = DeMoCodec(coll, K_local, L, dev)
        codec(P, G, D, 0.01)
        out["demo_p"] = _host(P)
        out["demo_sign"] = _host(G)
        out.update(_demo_pipe_pair(coll, K_local, nodes, dev, pieces=2))
    return out


def _demo_pipe_pair(coll, K_local, nodes, dev, pieces):
    """The same DeMo step through DeMoCodec and PipelinedDeMoCodec (async
    all-gathers of tensor groups overlapping the codec kernels)."""
    from gym_amd.arena import ArenaLayout
    from gym_amd.engine import DeMoCodec, PipelinedDeMoCodec
    L = ArenaLayout([(128, 128), (768,), (64, 192), (3, 64)])
    G0 = torch.from_numpy(np.stack([engine_node(j, L.n, salt=6) for j in nodes])).to(dev)
    D0 = torch.from_numpy(np.stack([engine_node(j, L.n, salt=7) for j in nodes]) * np.float32(0.01)).to(dev)
    P0 = torch.from_numpy(np.stack([engine_node(0, L.n, salt=8)] * len(nodes))).to(dev)
    for T in (G0, D0, P0):
        for k in range(K_local):  # zero padding, as the arena keeps it
            for o, m, o2 in zip(L.offsets, L.numels, L.offsets[1:] + [L.n]):
                T[k, o + m:o2] = 0
    out = {}
    for tag, make in (("plain", lambda: DeMoCodec(coll, K_local, L, dev)),
                      ("pipe", lambda: PipelinedDeMoCodec(coll, K_local, L, dev, pieces=pieces))):
        P, G, D = P0.clone(), G0.clone(), D0.clone()
        codec = make()
        for _ in range(2):
            codec(P, G, D, 0.01, 0.999, 0.1)
        out.update({f"pipe_{tag}_p": _host(P), f"pipe_{tag}_g": _host(G), f"pipe_{tag}_d": _host(D)})
    if tag == "pipe":
        out["pipe_pieces"] = np.array(len(codec.codecs))
    return out


def sc_demo_pipe(rank, world, dev, golden_dir, pieces=3):
    from gym_amd.comm import Collective
    return _demo_pipe_pair(Collective(), 2, range(rank * 2, rank * 2 + 2), dev, pieces)


SCENARIOS = {"simple_adamw": sc_simple_adamw, "engine": sc_engine, "simple": sc_simple, "diloco": sc_diloco, "sparta": sc_sparta, "sparta_philox": sc_sparta_philox,
             "sparta_sel": sc_sparta_sel, "eval_avg": sc_eval_avg,
             "mnist_diloco": sc_mnist_diloco,
             "fedavg": sc_fedavg, "demo": sc_demo, "demo_pipe": sc_demo_pipe}


def _worker(rank, world, port, name, device, fake, out_dir, golden_dir, kwargs, backend="gloo"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    if fake:
        import fake_ops
        fake_ops.install()
    if backend == "nccl":  # RCCL: one rank per GPU
        torch.cuda.set_device(torch.device(device))
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device(device))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device(device)
        res = SCENARIOS[name](rank, world, dev, golden_dir, **kwargs)
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), **{k: np.asarray(v) for k, v in res.items()})
    finally:
        dist.destroy_process_group()


def run(name, world, device, fake, out_dir, golden_dir, backend="gloo", **kwargs):
    import torch.multiprocessing as mp
    port = free_port()
    mp.spawn(_worker, args=(world, port, name, device, fake, out_dir, golden_dir, kwargs, backend), nprocs=world,
             join=True)
    res = []
    for r in range(world):
        with np.load(os.path.join(out_dir, f"r{r}.npz")) as f:
            res.append({k: f[k] for k in f.files})
    return res
