"""Generate the golden fixtures in tests/golden/ by running the REFERENCE
(satoutahhaithem/gym, mounted read-only at /root/reference) in this container.

Run:  PYTHONPATH=/root/reference python tests/golden/gen_golden.py
(only here: /root/reference does not exist on the GPU box; the .npz outputs are
committed and are all the tests ever read).

Each fixture exercises the reference's own code on CPU/gloo with small seeded
inputs:
  mean_reduce.npz   G1  communicate.all_reduce + div_  (strategy.py:130-133), K in {2,3,8}
  diloco.npz        G2  DiLoCoStrategy outer steps (diloco.py:51-76), K=3, H=2, 3 outer steps
  sparta.npz        G3  SPARTAStrategy communicate (sparta.py:24-44), K=2 and K=3, masks logged
  sparta_sel.npz    G3b ShuffledSequential / Partitioned selector masks (sparta.py:88-193)
  demo_codec.npz    G4  _dct/_idct bases, _get_smaller_split, TransformDCT encode/decode,
                        CompressDCT compress/decompress/batch_decompress (demo_impl/demo.py)
  demo_steps.npz    G4  3 full DeMo.step()s with K=2 over gloo (demo.py:142-209)
  demo_steps_bf16.npz G4b the same on bf16 parameters (bf16 bases, demo.py:235-236)
  lr_schedule.npz   G5  lambda_cosine LR sequence (strategy.py:65-95)
"""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

OUT = os.path.dirname(os.path.abspath(__file__))
assert "/root/reference" in sys.path[0] or any("/root/reference" in p for p in sys.path), \
    "run with PYTHONPATH=/root/reference"


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)


class ShapeModel(torch.nn.Module):
    """A module whose parameters have exactly the given shapes, in order."""

    def __init__(self, shapes, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.ps = torch.nn.ParameterList(
            [torch.nn.Parameter(torch.randn(*s, generator=g) * 0.02) for s in shapes])


class _Sink:
    """Per-rank result sink: each rank writes one .npz (no pickling, no pipe
    back-pressure while the parent waits in join)."""

    def __init__(self, d):
        self.d = d

    def put(self, item):
        rank, rec = item
        flat = {}
        for k, v in rec.items():
            if isinstance(v, list):
                for i, a in enumerate(v):
                    if a is not None:
                        flat[f"{k}__{i}"] = np.asarray(a)
            else:
                flat[k] = np.asarray(v)
        np.savez(os.path.join(self.d, f"r{rank}.npz"), **flat)


def _unflatten(z):
    rec = {}
    for k in z.files:
        if "__" in k:
            base, i = k.rsplit("__", 1)
            lst = rec.setdefault(base, {})
            lst[int(i)] = z[k]
        else:
            rec[k] = z[k]
    out = {}
    for k, v in rec.items():
        if isinstance(v, dict):
            out[k] = [v.get(i) for i in range(max(v) + 1)]
        else:
            out[k] = v
    return out


def run_spawn(fn, world, *args):
    import tempfile
    port = free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(fn, args=(world, port, _Sink(d)) + args, nprocs=world, join=True)
        out = {}
        for r in range(world):
            with np.load(os.path.join(d, f"r{r}.npz")) as z:
                out[r] = _unflatten(z)
    return out


# ---------------------------------------------------------------- G1 --------
G1_SHAPES = [(4, 3), (66, 128), (768,), (64, 1, 3, 3)]


def g1_worker(rank, world, port, q):
    from exogym.strategy.communicate import all_reduce
    init(rank, world, port)
    outs = {}
    for si, s in enumerate(G1_SHAPES):
        g = torch.Generator().manual_seed(100 * world + 10 * si + rank)
        t = torch.randn(*s, generator=g)
        outs[f"in_{si}"] = t.numpy().copy()
        all_reduce(t)
        t.div_(world)
        outs[f"out_{si}"] = t.numpy().copy()
    q.put((rank, outs))
    dist.destroy_process_group()


def gen_g1():
    res = {}
    for K in (2, 3, 8):
        out = run_spawn(g1_worker, K)
        for si in range(len(G1_SHAPES)):
            res[f"K{K}_in_{si}"] = np.stack([out[r][f"in_{si}"] for r in range(K)])
            res[f"K{K}_out_{si}"] = out[0][f"out_{si}"]
            for r in range(1, K):
                assert np.array_equal(out[r][f"out_{si}"], out[0][f"out_{si}"])
    np.savez_compressed(os.path.join(OUT, "mean_reduce.npz"), **res)


# ---------------------------------------------------------------- G2 --------
G2_SHAPES = [(4, 3), (66, 32), (768,), (64, 1, 3, 3)]
G2_H = 2
G2_CALLS = 7  # outer steps at local_step 2, 4, 6


def g2_worker(rank, world, port, q):
    from exogym.strategy import DiLoCoStrategy, OptimSpec
    init(rank, world, port)
    model = ShapeModel(G2_SHAPES, seed=1234)
    strat = DiLoCoStrategy(optim_spec=OptimSpec(torch.optim.SGD, lr=0.0), H=G2_H)
    strat._init_node(model, rank, world)
    # Q1: on CPU `.to("cpu")` aliases the node params with the master copy;
    # record GPU semantics (a copy), as every GPU run of the reference has.
    def sync_clone(self=strat):
        for name, param in self.model.named_parameters():
            param.data = self.master_model.state_dict()[name].data.clone()
    strat._synchronize_master_model = sync_clone
    rec = {"init": [p.detach().numpy().copy() for p in model.parameters()]}
    for call in range(G2_CALLS):
        g = torch.Generator().manual_seed(1000 + 100 * rank + call)
        with torch.no_grad():
            for p in model.parameters():
                p.add_(torch.randn(p.shape, generator=g) * 1e-3)
        before = [p.detach().numpy().copy() for p in model.parameters()]
        strat.step()
        after = [p.detach().numpy().copy() for p in model.parameters()]
        rec[f"before_{call}"] = before
        rec[f"after_{call}"] = after
        if rank == 0:
            rec[f"master_{call}"] = [p.detach().numpy().copy() for p in strat.master_model.parameters()]
            st = strat.outer_optimizer.state
            rec[f"mom_{call}"] = [st[p]["momentum_buffer"].numpy().copy() if p in st else None
                                  for p in strat.master_model.parameters()]
    q.put((rank, rec))
    dist.destroy_process_group()


def gen_g2():
    K = 3
    out = run_spawn(g2_worker, K)
    res = {"K": K, "H": G2_H, "calls": G2_CALLS, "nshapes": len(G2_SHAPES)}
    for i in range(len(G2_SHAPES)):
        res[f"init_{i}"] = out[0]["init"][i]
        for call in range(G2_CALLS):
            res[f"before_{call}_{i}"] = np.stack([out[r][f"before_{call}"][i] for r in range(K)])
            res[f"after_{call}_{i}"] = np.stack([out[r][f"after_{call}"][i] for r in range(K)])
            res[f"master_{call}_{i}"] = out[0][f"master_{call}"][i]
            moms = out[0].get(f"mom_{call}") or []
            m = moms[i] if i < len(moms) else None
            if m is not None:
                res[f"mom_{call}_{i}"] = m
    np.savez_compressed(os.path.join(OUT, "diloco.npz"), **res)


# ---------------------------------------------------------------- G3 --------
G3_SHAPES = [(66, 32), (128,), (96, 64), (3, 7)]
G3_P = 0.05
G3_CALLS = 3


def g3_worker(rank, world, port, q):
    from exogym.strategy import SPARTAStrategy, OptimSpec
    import exogym.strategy.sparta as sp
    init(rank, world, port)
    torch.manual_seed(42)  # TrainNode seeds every rank with 42 (train_node.py:50-53)
    model = ShapeModel(G3_SHAPES, seed=77 + rank)  # nodes differ
    strat = SPARTAStrategy(inner_optim=OptimSpec(torch.optim.SGD, lr=0.0), p_sparta=G3_P)
    strat._init_node(model, rank, world)
    masks = []
    orig = sp.RandomIndexSelector.get_indices

    def logged(self, param, iteration):
        m = orig(self, param, iteration)
        masks.append(m.clone())
        return m

    sp.RandomIndexSelector.get_indices = logged
    for p in model.parameters():
        p.grad = torch.zeros_like(p)
    rec = {}
    for call in range(G3_CALLS):
        masks.clear()
        rec[f"before_{call}"] = [p.detach().numpy().copy() for p in model.parameters()]
        strat.step()
        rec[f"after_{call}"] = [p.detach().numpy().copy() for p in model.parameters()]
        # the mask actually used is rank 0's (broadcast, sparta.py:37); log what rank 0 drew
        rec[f"mask_{call}"] = [m.numpy().copy() for m in masks]
    q.put((rank, rec))
    dist.destroy_process_group()


def gen_g3():
    res = {"p": G3_P, "calls": G3_CALLS, "nshapes": len(G3_SHAPES)}
    for K in (2, 3):
        out = run_spawn(g3_worker, K)
        for call in range(G3_CALLS):
            for i in range(len(G3_SHAPES)):
                res[f"K{K}_before_{call}_{i}"] = np.stack([out[r][f"before_{call}"][i] for r in range(K)])
                res[f"K{K}_after_{call}_{i}"] = np.stack([out[r][f"after_{call}"][i] for r in range(K)])
                res[f"K{K}_mask_{call}_{i}"] = np.packbits(out[0][f"mask_{call}"][i].reshape(-1))
    np.savez_compressed(os.path.join(OUT, "sparta.npz"), **res)


def gen_g3b():
    from exogym.strategy.sparta import ShuffledSequentialIndexSelector, PartitionedIndexSelector
    shapes = [(66, 128), (50,), (3, 7)]
    res = {}
    for name, cls, p in (("shuf", ShuffledSequentialIndexSelector, 0.1),
                         ("part", PartitionedIndexSelector, 0.25)):
        torch.manual_seed(42)
        sel = cls(p)
        params = [torch.nn.Parameter(torch.zeros(s)) for s in shapes]
        for it in range(5):
            for i, prm in enumerate(params):
                res[f"{name}_{it}_{i}"] = np.packbits(sel.get_indices(prm, it).reshape(-1).numpy())
    np.savez_compressed(os.path.join(OUT, "sparta_sel.npz"), **res)


# ---------------------------------------------------------------- G4 --------
SPLIT_SIZES = [1, 2, 3, 7, 10, 29, 33, 64, 66, 128, 768, 1024, 2304, 3072, 4096, 50257, 50304, 9216, 1000]
DEMO_SHAPES = [(128, 128), (66, 128), (768,), (8, 4, 3, 3), (10,), (58, 29)]


def gen_g4_codec():
    from exogym.strategy.demo_impl.demo import (_dct, _idct, _get_smaller_split, TransformDCT,
                                                CompressDCT)
    res = {}
    for n in (1, 3, 10, 29, 33, 64):
        eye = torch.eye(n)
        res[f"F_{n}"] = _dct(eye, norm="ortho").numpy()
        res[f"B_{n}"] = _idct(eye, norm="ortho").numpy()
    res["split_sizes"] = np.array(SPLIT_SIZES)
    for chunk in (64, 32):
        res[f"split_{chunk}"] = np.array([_get_smaller_split(s, chunk) for s in SPLIT_SIZES])
    g = torch.Generator().manual_seed(5)
    params = [torch.nn.Parameter(torch.randn(*s, generator=g)) for s in DEMO_SHAPES]
    tr = TransformDCT([{"params": params}], 64)
    cp = CompressDCT()
    for i, p in enumerate(params):
        x = torch.randn(p.shape, generator=g)
        enc = tr.encode(x, p)
        idx, val, xshape, totalk = cp.compress(enc, 32)
        dec = tr.decode(cp.decompress(p, idx, val, xshape, totalk), p)
        full = tr.decode(enc, p)
        res[f"x_{i}"] = x.numpy()
        res[f"enc_{i}"] = enc.numpy()
        res[f"idx_{i}"] = idx.numpy()
        res[f"val_{i}"] = val.numpy()
        res[f"dec_{i}"] = dec.numpy()
        res[f"roundtrip_{i}"] = full.numpy()
        # batch_decompress with duplicates: node 1 repeats half of node 0's indices
        idx2 = idx.clone()
        idx2[..., : idx.shape[-1] // 2] = idx[..., : idx.shape[-1] // 2]
        idx2[..., idx.shape[-1] // 2:] = torch.flip(idx, dims=[-1])[..., idx.shape[-1] // 2:]
        val2 = torch.randn(val.shape, generator=g)
        bd = cp.batch_decompress(p, [idx, idx2], [val, val2], xshape, totalk)
        res[f"bidx2_{i}"] = idx2.numpy()
        res[f"bval2_{i}"] = val2.numpy()
        res[f"bdec_{i}"] = bd.numpy()
    # an all-zero chunk: every |coefficient| ties; only the value multiset is defined
    z = torch.zeros(128, 128)
    enc = tr.encode(z, torch.nn.Parameter(torch.zeros(128, 128)))
    idx, val, _, _ = cp.compress(enc, 32)
    res["zero_idx"] = idx.numpy()
    res["zero_val"] = val.numpy()
    np.savez_compressed(os.path.join(OUT, "demo_codec.npz"), **res)


DEMO_STEP_SHAPES = [(128, 64), (66, 128), (768,), (8, 4, 3, 3), (10,)]
DEMO_STEPS = 3


def g4_step_worker(rank, world, port, q):
    from exogym.strategy.demo_impl.demo import DeMo
    from exogym.strategy.communicate import all_gather
    init(rank, world, port)
    model = ShapeModel(DEMO_STEP_SHAPES, seed=4321)  # identical start on every node
    opt = DeMo(model.parameters(), compression_decay=0.999, compression_topk=32, compression_chunk=64,
               weight_decay=0.1, custom_all_gather=all_gather, lr=0.01)
    rec = {}
    for step in range(DEMO_STEPS):
        g = torch.Generator().manual_seed(2000 + 10 * rank + step)
        for p in model.parameters():
            p.grad = torch.randn(p.shape, generator=g)
        rec[f"grad_{step}"] = [p.grad.numpy().copy() for p in model.parameters()]
        rec[f"p_before_{step}"] = [p.detach().numpy().copy() for p in model.parameters()]
        rec[f"delta_before_{step}"] = [opt.demo_state[p]["delta"].numpy().copy() for p in model.parameters()]
        opt.step()
        rec[f"p_after_{step}"] = [p.detach().numpy().copy() for p in model.parameters()]
        rec[f"delta_after_{step}"] = [opt.demo_state[p]["delta"].numpy().copy() for p in model.parameters()]
        rec[f"sign_{step}"] = [p.grad.numpy().copy() for p in model.parameters()]
        rec[f"tx_{step}"] = opt.data_transmit
        rec[f"rx_{step}"] = opt.data_receive
    q.put((rank, rec))
    dist.destroy_process_group()


def _gen_demo_steps(worker, shapes, fname, K=2, **extra):
    out = run_spawn(worker, K)
    res = {"K": K, "steps": DEMO_STEPS, "nshapes": len(shapes), "lr": 0.01, "wd": 0.1,
           "decay": 0.999, "topk": 32, "chunk": 64, **extra}
    for step in range(DEMO_STEPS):
        res[f"tx_{step}"] = out[0][f"tx_{step}"]
        res[f"rx_{step}"] = out[0][f"rx_{step}"]
        for i in range(len(shapes)):
            for key in ("grad", "delta_before", "delta_after"):
                res[f"{key}_{step}_{i}"] = np.stack([out[r][f"{key}_{step}"][i] for r in range(K)])
            for key in ("p_before", "p_after", "sign"):
                res[f"{key}_{step}_{i}"] = out[0][f"{key}_{step}"][i]
                assert np.array_equal(out[1][f"{key}_{step}"][i], out[0][f"{key}_{step}"][i])
    np.savez_compressed(os.path.join(OUT, fname), **res)


def gen_g4_steps():
    _gen_demo_steps(g4_step_worker, DEMO_STEP_SHAPES, "demo_steps.npz")


# bf16 parameters: the reference casts its DCT bases to p.dtype (demo.py:235-236), so
# every einsum, the top-k and the scatter-mean run in bf16 on the CPU.  Values are
# stored as their exact fp32 widening (npz has no bf16).
DEMO_BF16_SHAPES = [(128, 128), (128, 64), (768,), (64,)]


def g4_bf16_worker(rank, world, port, q):
    from exogym.strategy.demo_impl.demo import DeMo
    from exogym.strategy.communicate import all_gather
    init(rank, world, port)
    model = ShapeModel(DEMO_BF16_SHAPES, seed=8765).to(torch.bfloat16)
    opt = DeMo(model.parameters(), compression_decay=0.999, compression_topk=32, compression_chunk=64,
               weight_decay=0.1, custom_all_gather=all_gather, lr=0.01)
    rec = {}
    f = lambda t: t.detach().float().numpy().copy()  # noqa: E731
    for step in range(DEMO_STEPS):
        g = torch.Generator().manual_seed(3000 + 10 * rank + step)
        for p in model.parameters():
            p.grad = torch.randn(p.shape, generator=g).to(torch.bfloat16)
        rec[f"grad_{step}"] = [f(p.grad) for p in model.parameters()]
        rec[f"p_before_{step}"] = [f(p) for p in model.parameters()]
        rec[f"delta_before_{step}"] = [f(opt.demo_state[p]["delta"]) for p in model.parameters()]
        opt.step()
        rec[f"p_after_{step}"] = [f(p) for p in model.parameters()]
        rec[f"delta_after_{step}"] = [f(opt.demo_state[p]["delta"]) for p in model.parameters()]
        rec[f"sign_{step}"] = [f(p.grad) for p in model.parameters()]
        rec[f"tx_{step}"] = opt.data_transmit
        rec[f"rx_{step}"] = opt.data_receive
    q.put((rank, rec))
    dist.destroy_process_group()


def gen_g4_bf16():
    _gen_demo_steps(g4_bf16_worker, DEMO_BF16_SHAPES, "demo_steps_bf16.npz", dtype="bfloat16")


# ---------------------------------------------------------------- G5 --------
def g5_worker(rank, world, port, q):
    from exogym.strategy.strategy import SimpleReduceStrategy
    from exogym.strategy import OptimSpec
    init(rank, world, port)
    rec = {}
    for name, kw, max_steps in (
        ("cos", {"warmup_steps": 5, "cosine_anneal": True}, 30),
        ("cos_cap", {"warmup_steps": 3, "cosine_anneal": True, "max_steps": 12}, 40),
        ("warm", {"warmup_steps": 4}, 10),
    ):
        model = ShapeModel([(3,)], seed=1)
        s = SimpleReduceStrategy(optim_spec=OptimSpec(torch.optim.SGD, lr=0.5),
                                 lr_scheduler="lambda_cosine", lr_scheduler_kwargs=kw)
        s._init_node(model, rank, world)
        s.max_steps = max_steps
        lrs = [s.optim.param_groups[0]["lr"]]
        for _ in range(max_steps + 5):
            for p in model.parameters():
                p.grad = torch.zeros_like(p)
            s.step()
            lrs.append(s.optim.param_groups[0]["lr"])
        rec[name] = np.array(lrs)
    q.put((rank, rec))
    dist.destroy_process_group()


def gen_g5():
    out = run_spawn(g5_worker, 1)
    np.savez_compressed(os.path.join(OUT, "lr_schedule.npz"), **out[0])


if __name__ == "__main__":
    torch.set_num_threads(1)
    which = sys.argv[1:] or ["g1", "g2", "g3", "g3b", "g4c", "g4s", "g4b", "g5"]
    for w in which:
        {"g1": gen_g1, "g2": gen_g2, "g3": gen_g3, "g3b": gen_g3b, "g4c": gen_g4_codec,
         "g4s": gen_g4_steps, "g4b": gen_g4_bf16, "g5": gen_g5}[w]()
        print("wrote", w, flush=True)
