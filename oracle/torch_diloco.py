"""Pure-torch, per-parameter restatement of the reference's DiLoCo outer step
over gloo on the host CPU (TEST INFRASTRUCTURE and the bench's CPU baseline;
never part of the product path).

It follows exogym/strategy/diloco.py step by step, one tensor at a time, as
the reference runs it on a CPU/gloo node (SURVEY §6 timed the reference itself
this way in the build container):
  _average_models           diloco.py:34-37   all_reduce(SUM) + `/= num_nodes` per tensor
  rank 0: outer zero_grad   diloco.py:66-67
          _set_master_grad  diloco.py:43-45   master.grad = master - node param
          outer SGD step    diloco.py:70      torch.optim.SGD(lr 0.7, momentum 0.9, nesterov)
          _synchronize      diloco.py:47-49   node param <- master (a COPY: the GPU
                                              semantics, SURVEY Q1 -- on CPU the
                                              reference aliases the two)
  _broadcast_model_params   diloco.py:39-41   broadcast from rank 0 per tensor
Pinned bit-exact to tests/golden/diloco.npz (the reference run over gloo) by
tests/test_torch_baseline.py.  bench.py times it on the full GPT-2 124M
parameter list with K processes x T threads as the CPU baseline.
"""
import os
import time

import torch
import torch.distributed as dist


class TorchDiLoCoOuter:
    def __init__(self, params, rank, world, lr=0.7, momentum=0.9, nesterov=True):
        self.params = list(params)
        self.rank, self.world = rank, world
        if rank == 0:  # diloco.py:78-89: the master copy and the outer optimizer live on rank 0
            self.master = [torch.nn.Parameter(p.detach().clone()) for p in self.params]
            self.outer = torch.optim.SGD(self.master, lr=lr, momentum=momentum, nesterov=nesterov)

    @torch.no_grad()
    def step(self):
        for p in self.params:
            dist.all_reduce(p.data, op=dist.ReduceOp.SUM)
            p.data /= self.world
        if self.rank == 0:
            self.outer.zero_grad()
            for m, p in zip(self.master, self.params):
                m.grad = m.data - p.data
            self.outer.step()
            for m, p in zip(self.master, self.params):
                p.data.copy_(m.data)
        for p in self.params:
            dist.broadcast(p.data, src=0)


def _synth(shapes, rank, seed=1234):
    """Node parameters: shared N(0, 0.02) start + per-node N(0, 1e-3) drift
    (SURVEY §8(d) synthetic inputs)."""
    g = torch.Generator().manual_seed(seed)
    base = [torch.randn(*s, generator=g) * 0.02 for s in shapes]
    g.manual_seed(1000 + rank)
    return [b + torch.randn(b.shape, generator=g) * 1e-3 for b in base]


def _time_worker(rank, world, port, shapes, threads, steps, warmup, out_path):
    # gloo prints its connection banner on stdout: keep the parent's stdout (the
    # bench's one JSON line) clean
    devnull = os.open(os.devnull, os.O_WRONLY)
    os.dup2(devnull, 1)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # started from a torchrun-launched bench: the agent's store is not ours (with this
    # set, rank 0 would not serve the rendezvous and every worker would wait forever)
    for k in ("TORCHELASTIC_USE_AGENT_STORE", "TORCHELASTIC_RUN_ID", "GROUP_RANK", "LOCAL_WORLD_SIZE"):
        os.environ.pop(k, None)
    torch.set_num_threads(threads)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        params = _synth(shapes, rank)
        eng = TorchDiLoCoOuter(params, rank, world)
        for _ in range(warmup):
            eng.step()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.step()
        dist.barrier()
        dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        if rank == 0:
            with open(out_path, "w") as f:
                f.write(repr(float(dt) / steps))
    finally:
        dist.destroy_process_group()


def time_outer_step(shapes, nodes, cores, steps=3, warmup=1):
    """Seconds per outer step of `nodes` gloo processes x cores//nodes threads
    each, every process holding the full parameter list `shapes`."""
    import socket
    import tempfile

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    threads = max(1, cores // nodes)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "t")
        mp.spawn(_time_worker, args=(nodes, port, shapes, threads, steps, warmup, out), nprocs=nodes, join=True)
        return float(open(out).read()), threads
