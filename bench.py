"""Strategy-communication-step benchmark (BASELINE.json metric: strategy-step
param GB/s (%HBM/xGMI peak) + ms/outer step, GPT-2 124M, 1-8 GPUs).

Headline workload (configs[2]): the DiLoCo outer step of GPT-2 124M over 8
simulated nodes IN TOTAL, 8/N per GPU (N=1: a batched-replica arena [8, n] on
one GPU, averaged in-kernel; N=8: one node per GPU, RCCL reduce-scatter /
all-gather over xGMI; between, an in-kernel pre-sum over the local 8/N then
RCCL).  Total work is fixed as N grows (scaling "strong"), so the driver's
1->8 curve runs ONE configuration and at N=8 the headline's "xgmi" block is
the north star's xGMI fraction.  One timed "step" = one outer step:
sum/average of every node's parameters, pseudo-gradient, outer Nesterov SGD,
write-back into every node.  Inputs are synthetic, resident in HBM before
timing starts.

value = node-parameter bytes averaged per second over the whole job
        = K_total * 4 * N_params / t_step  ("param GB/s"); ms_per_step = t_step.
roofline = the fused ga_diloco_outer kernel: algorithmic HBM bytes per launch
        ((2*K_local + 4) * 4 * n: read every replica, master, momentum; write
        them back) / its HIP-event-timed duration, against 8 TB/s.  "traffic"
        = HBM bytes per launch from two rocprofv3 PMC passes (FETCH_SIZE x2 on
        gfx950, WRITE_SIZE) of this same configuration, run by this script as
        child processes before it touches the GPU itself; "copy_GBps" = a
        float4 streaming copy (ga_stream_copy) between two ordinary
        allocations timed in this process, what the box streams unplaced.
cpu_baseline = the reference's DiLoCo outer step restated per tensor in torch
        (oracle/torch_diloco.py, bit-exact with the reference's golden run),
        over gloo with 8 node processes x (cores/8) threads on this host, on
        the full GPT-2 124M parameter list (configs[2]: 8 nodes), run on
        rank 0 before the GPU is initialised; at N > 1 the same 8-node job.

Extra lines in "extras" (same timing rules, not the headline): SPARTA (32
nodes in total, 32/G per GPU, p=0.005, Philox mask: configs[3]), SimpleReduce
(char-level nanoGPT, 8 nodes in total, 8/G per GPU: configs[1]), DeMo (GPT-2
350M, one node per GPU, chunk 64 / top-k 32: configs[4]), the inner AdamW +
clip step on one GPT-2 124M arena (fused vs torch foreach), and at G > 1 the
weak-scaled DiLoCo step, 8 nodes per GPU (8G in total:
diloco_8_nodes_per_gpu).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-extras]
       torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)
`python bench.py --gpus N` with N > 1 and no torchrun environment launches
itself: this process runs the host legs (the CPU baseline) without touching
the GPU, starts `python -m torch.distributed.run --nproc-per-node N bench.py`
as a child process (one rank per GPU), and prints rank 0's JSON line with
the CPU baseline merged in (self_launch below).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from gym_amd import ops  # noqa: E402
from gym_amd.arena import ArenaLayout, ReplicaSet  # noqa: E402
from gym_amd.comm import Collective  # noqa: E402
from gym_amd.engine import DeMoCodec, DiLoCoOuter, MeanReduce, Sparta, place_demo_step  # noqa: E402
from gym_amd.shapes import MODELS, numel  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E, MI355X_MICROARCH.md
MFMA_F32_TFLOPS = 157.3    # dense fp32 MFMA (= f32 vector) peak
XGMI_LINK_GBS = 153.0      # per xGMI link (SURVEY §8(d) roofline model)


def setup_dist(gpus):
    if gpus > 1 or "RANK" in os.environ:
        local = int(os.environ.get("LOCAL_RANK", 0))
        from gym_amd.placement import note_devices
        if os.environ.get("GA_BENCH_BACKEND") == "gloo":
            # rehearsal of the multi-rank path on a 1-GPU box: ranks share the GPUs over gloo
            torch.cuda.set_device(local % torch.cuda.device_count())
            dist.init_process_group("gloo")
            note_devices()
            return Collective()
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        note_devices()
        if os.environ.get("GA_BENCH_FORCE_EXCHANGE") == "1":
            # rehearsal of the multi-GPU code paths on one GPU: a world-1 RCCL group whose
            # collectives are issued anyway (tests/test_gpu_rccl.py); not a measurement
            return Collective(force_exchange=True)
    else:
        torch.cuda.set_device(0)
    return Collective()


def synth_replicas(layout, K, rank, dev, dtype=torch.float32):
    """Node k: shared start N(0, 0.02) (seed 1234) + drift N(0, 1e-3) (seed 1000+k),
    the layout's padding kept at zero (SURVEY §8(d) synthetic inputs)."""
    rs = ReplicaSet(layout, K, dev, dtype)
    g = torch.Generator(device=dev)
    base = torch.empty(layout.n, device=dev)
    g.manual_seed(1234)
    base.normal_(0.0, 0.02, generator=g)
    pad = torch.ones(layout.n, device=dev, dtype=torch.bool)
    for o, n in zip(layout.offsets, layout.numels):
        pad[o:o + n] = False
    base[pad] = 0
    for k in range(K):
        g.manual_seed(1000 + rank * K + k)
        rs.data[k].normal_(0.0, 1e-3, generator=g)
        rs.data[k].add_(base)
        rs.data[k][pad] = 0
    return rs


def timed_loop(fn, steps, warmup, coll):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if coll.world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if coll.world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if coll.world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt / steps


class KernelTimer:
    """HIP events around one kernel launch, on the stream it is launched on."""

    def __init__(self):
        self.pairs = []
        self.on = False

    def wrap(self, fn):
        def timed(*a, **kw):
            if not self.on:
                return fn(*a, **kw)
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            r = fn(*a, **kw)
            e1.record(s)
            self.pairs.append((e0, e1))
            return r
        return timed

    def mean_ms(self):
        torch.cuda.synchronize()
        return float(np.mean([a.elapsed_time(b) for a, b in self.pairs])) if self.pairs else None


SUSTAINED_LAUNCHES = 1000  # the headline kernel also timed over ~2 s of back-to-back launches


def queued_ms(fn, reps, dev, fill_bytes=1 << 30, fills=4):
    """GPU time per call of fn with its launches queued back to back: streaming
    copies (ga_stream_copy, ~1.5 ms) occupy the GPU while the host enqueues the
    reps calls, so the two events bracket GPU work only, not the host's launch
    gaps.  For kernels of tens of microseconds, where HIP events around one
    launch measure the host's launch latency as much as the kernel."""
    a = torch.empty(fill_bytes // 4, device=dev)
    b = torch.empty_like(a)
    a.fill_(0.0)
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(fills):
        ops.stream_copy(a, b)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    del a, b
    return e0.elapsed_time(e1) / reps


def host_cores():
    """CPU share of this process: the job's thread budget (OMP_NUM_THREADS is
    set to the box's share on the GPU pool), capped by the visible CPUs."""
    n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(env))) if env and env.isdigit() else n


def cpu_baseline_diloco(model, K, steps=3, warmup=1):
    """The reference's outer step (oracle/torch_diloco.py, per-tensor torch over
    gloo: K node processes x cores//K threads) on the full parameter list."""
    from oracle.torch_diloco import time_outer_step
    shapes = MODELS[model]()
    cores = host_cores()
    t, threads = time_outer_step(shapes, nodes=K, cores=cores, steps=steps, warmup=warmup)
    n = numel(shapes)
    return {"value": round(K * 4 * n / t / 1e9, 4), "unit": "GB/s", "cores": K * threads, "kind": "port",
            "ms_per_step": round(t * 1e3, 1), "nproc": os.cpu_count(), "threads_per_process": threads,
            "sample": f"DiLoCo outer step (all-reduce+divide, rank-0 SGD-Nesterov on the master, broadcast) of "
                      f"{model} ({n} params, {len(shapes)} tensors) over {K} gloo processes x {threads} threads "
                      f"(oracle/torch_diloco.py, the reference's per-tensor torch ops, bit-exact with "
                      f"tests/golden/diloco.npz), full size, {steps} timed steps after {warmup} warmup; "
                      f"value = {K} x 4 x {n} B / step time"}


def pmc_traffic_live(args, alg_bytes_expected=None, timeout=150):
    """HBM bytes per ga_diloco_outer launch from two rocprofv3 PMC passes of
    this configuration (FETCH_SIZE and WRITE_SIZE need passes of their own),
    run as child processes.  MI355X_MICROARCH.md: counters in KiB; on gfx950
    FETCH_SIZE reports half the bytes of wide coalesced reads (doubled here).
    Returns (bytes, note)."""
    import shutil
    import subprocess
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_traffic import counter_values
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    vals = {}
    env = {**os.environ, "TMPDIR": "/tmp"}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="ga_pmc_", dir="/tmp")
        cmd = [prof, "--pmc", counter, "-d", d, "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.join(ROOT, "bench.py"), "--pmc-child", "--model", args.model,
               "--replicas", str(args.replicas)]
        try:
            r = subprocess.run(cmd, cwd="/tmp", env=env, timeout=timeout, stdout=subprocess.DEVNULL,
                               stderr=subprocess.PIPE)
        except subprocess.TimeoutExpired:
            return None, f"rocprofv3 --pmc {counter} timed out"
        v = counter_values(d, counter, "diloco_outer")
        shutil.rmtree(d, ignore_errors=True)
        if r.returncode != 0 or not v:
            return None, f"rocprofv3 --pmc {counter} failed (rc {r.returncode}): {r.stderr.decode()[-200:]}"
        vals[counter] = float(np.median(v))
    traffic = (2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0
    return traffic, (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this configuration (median over the "
                     f"launches; FETCH_SIZE x2 for gfx950 wide reads, KiB -> B): read "
                     f"{2.0 * vals['FETCH_SIZE'] * 1024.0:.4g} B + write {vals['WRITE_SIZE'] * 1024.0:.4g} B")


def under_profiler():
    """True inside a rocprofv3 run (its tool library is preloaded and has
    initialised the GPU): a nested rocprofv3 would have to exec from there."""
    pre = os.environ.get("LD_PRELOAD", "") + os.environ.get("HSA_TOOLS_LIB", "")
    return "rocprof" in pre or any(k.startswith("ROCPROF") for k in os.environ)


def stream_copy_rate(dev, nbytes=2 << 30, reps=10):
    """GB/s (read + write bytes) of a float4 streaming copy in this process."""
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    src.fill_(1.0)
    ops.stream_copy(src, dst)
    times = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.stream_copy(src, dst)
        e1.record()
        e1.synchronize()
        times.append(e0.elapsed_time(e1))
    del src, dst
    return 2 * nbytes / (float(np.median(times)) * 1e-3) / 1e9


def stream_copy_sustained(dev, launches, nbytes=2 << 30):
    """GB/s of the same float4 copy over `launches` back-to-back launches (~2 s)."""
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    src.fill_(1.0)
    ms = queued_ms(lambda: ops.stream_copy(src, dst), launches, dev)
    del src, dst
    return 2 * nbytes / (ms * 1e-3) / 1e9


def xgmi_block(kind, nbytes, coll_ms, world, step_ms=None, what=None, latency_bound=False):
    """The SURVEY §8(d) xGMI rooflines of one exchange at `world` GPUs.
    all_reduce of S bytes (or reduce-scatter + all-gather, the same bytes):
    bus bytes 2(G-1)/G * S; all_gather of a P-byte per-rank payload: (G-1) * P.
    Fractions against one 153 GB/s link (the per-link ring model, SURVEY §8(d)'s
    primary roofline), against the (G-1)-link multi-ring bound and against 7
    links; coll_ms = the collective timed alone, step_ms = the whole step."""
    G = world
    bus = (2.0 * (G - 1) / G * nbytes) if kind == "all_reduce" else float((G - 1) * nbytes)
    out = {"collective": kind, "bytes": int(nbytes), "bus_bytes": int(bus), "world": G,
           "collective_alone_ms": round(coll_ms, 4) if coll_ms is not None else None}
    if what:
        out["what"] = what
    if G < 2 or coll_ms is None:
        out["note"] = "world 1 (rehearsal): no bytes cross xGMI, no roofline" if G < 2 else "not timed"
        return out
    bw = bus / (coll_ms * 1e-3) / 1e9
    t_min = bus / (XGMI_LINK_GBS * 1e9) * 1e3
    # the per-link ring model is the primary roofline; the multi-ring
    # bound is (G - 1) links of a fully connected node (7 at G = 8)
    out.update({"bus_GBps": round(bw, 1), "t_min_per_link_ring_ms": round(t_min, 4),
                "frac_per_link_ring": round(bw / XGMI_LINK_GBS, 4),
                "frac_multi_ring": round(bw / ((G - 1) * XGMI_LINK_GBS), 4),
                "frac_7link": round(bw / (7 * XGMI_LINK_GBS), 4)})
    if step_ms is not None:
        sbw = bus / (step_ms * 1e-3) / 1e9
        out.update({"bus_GBps_whole_step": round(sbw, 1), "frac_per_link_ring_whole_step": round(sbw / XGMI_LINK_GBS, 4)})
    if latency_bound:
        out["bound"] = "latency (a few MB: RCCL's small-message latency, not link bandwidth, sets the time; " \
                       "reported in microseconds)"
        out["collective_alone_us"] = round(coll_ms * 1e3, 1)
    return out


def bench_diloco(args, coll, dev):
    shapes = MODELS[args.model]()
    layout = ArenaLayout(shapes)
    n = layout.padded_to(coll.world)
    layout.n = n
    K = args.replicas
    rs = synth_replicas(layout, K, coll.rank, dev)
    eng = DiLoCoOuter(coll, K, n, dev, torch.float32)
    eng.init_master(rs.data[0])
    timer = KernelTimer()
    eng._outer = timer.wrap(eng._outer)
    # as the product's replica loop does (ReplicaRunner), the step may move the replica set
    # into the memory it runs fastest on, once, at its first call (DiLoCoOuter._place)
    eng.relocate_replicas = rs.relocate
    eng(rs.data)  # first outer step (placement; momentum buffer created); timed steps use the warm buffer
    reps = rs.data
    timer.on = True
    t = timed_loop(lambda: eng(reps), args.steps, args.warmup, coll)
    kern_single = timer.mean_ms()
    timer.on = False
    kern_ms, kern_how = kern_single, "HIP events around each launch"
    if coll.world == 1 and not args.pmc_child:
        # one launch per step: time it queued back to back (what rocprofv3's kernel
        # durations measure; single-launch events add the host's launch gap)
        kern_ms = queued_ms(lambda: eng(reps), max(args.steps, 10), dev)
        kern_how = "HIP events around back-to-back launches queued behind streaming copies (queued_ms)"
        # the same, sustained for ~2 s: a few steps after idle run faster than a
        # sustained stream of them (profiles/r03af_diloco_sustained_clocks.txt)
        # (not under rocprofv3: its kernel statistics stay those of the line's kernel_ms)
        sus_ms = None if under_profiler() else queued_ms(lambda: eng(reps), SUSTAINED_LAUNCHES, dev)
    else:
        sus_ms = None
    K_total = K * coll.world
    n_params = numel(shapes)
    value = K_total * 4 * n_params / t / 1e9
    per = int(np.mean(eng.launch_elems))  # elements per ga_diloco_outer launch (one per pipeline chunk)
    if coll.world == 1:  # read every replica, master, mom; write master, mom, every replica
        alg_bytes = (2 * K + 4) * per * 4
    elif eng.shard:  # RCCL: read the reduce-scattered sum slice, master, mom; write master, mom, param slice
        alg_bytes = 6 * per * 4
    else:  # gloo rehearsal: read the all-reduced sum, master, mom; write master, mom, every replica
        alg_bytes = (5 + K) * per * 4
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic, tnote = getattr(args, "pmc", None) or (None, "not measured (N > 1 or --no-pmc)")
    if coll.world > 1:
        traffic, tnote = None, "not measured at N > 1"
    copy = None if args.pmc_child else stream_copy_rate(dev)
    copy_sus = stream_copy_sustained(dev, 2 * SUSTAINED_LAUNCHES) if sus_ms else None
    args.copy_GBps = copy
    out = {
        "ms_per_step": t * 1e3, "value": value, "K_total": K_total, "n_params": n_params,
        "kernel_ms": kern_ms, "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_over_alg": round(traffic / alg_bytes, 6) if traffic else None, "traffic_source": tnote,
            "kernel": "ga_diloco_outer", "bytes_per_launch": alg_bytes, "kernel_ms": round(kern_ms, 4),
            "kernel_timing": kern_how,
            "kernel_ms_single_launch_events": round(kern_single, 4) if kern_single is not None else None,
            "sustained": {"launches": SUSTAINED_LAUNCHES, "kernel_ms": round(sus_ms, 4),
                          "frac": round(alg_bytes / (sus_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                          "copy_GBps": round(copy_sus, 1)} if sus_ms else None,
            # a float4 copy between two ordinary allocations in this process: what the box
            # streams without placement (the placed kernel can exceed it, so no ratio is given)
            "copy_GBps": round(copy, 1) if copy else None,
            # master/momentum placement chosen by DiLoCoOuter._place (probe times per candidate)
            "placement": eng.placement},
    }
    if coll.exchange:
        # the exchange alone: reduce-scatter + all-gather of the whole arena (the bytes of one
        # all-reduce), unchunked, no kernels; then the step's own bus rate beside it
        S = 4 * n
        full = reps[0, :n]
        shard = torch.empty(n // coll.world, device=dev)
        if eng.shard:
            def exch():
                coll.reduce_scatter(shard, full)
                coll.all_gather_into(full, shard)
        else:
            def exch():
                coll.all_reduce_(full)
        t_x = timed_loop(exch, args.steps, args.warmup, coll)
        out["xgmi"] = xgmi_block("all_reduce", S, t_x * 1e3, coll.world, step_ms=t * 1e3,
                                 what="reduce_scatter + all_gather (RCCL) of the arena alone = the bytes of "
                                      "one all-reduce; the step overlaps it with the sum/update kernels"
                                 if eng.shard else "all-reduce of the arena alone")
    return out


def bench_sparta(args, coll, dev, K_total=32, p=0.005, model="gpt2-124m", layout_kind="elem", mask_source="philox"):
    """configs[3]: K=32 simulated nodes on one GPU, or the same 32 nodes sharded
    32/G per GPU over G GPUs (strong: the node count is the config's).
    layout_kind "elem": the replica set element-major [n, K] (one element's K
    replicas adjacent: at K=32 fp32 one 128-B line per selected element);
    "rows": [K, n], the replica training loop's layout (every selected
    (element, replica) a separate random 4-B word).
    mask_source "philox": the in-kernel stream (the fast mode); "torch": the
    reference's per-tensor torch.bernoulli draws (the drop-in default,
    bit-identical selections) into a uint8 mask arena inside the timed step,
    packed and broadcast from rank 0 at N > 1."""
    K = max(1, K_total // coll.world)
    shapes = MODELS[model]()
    layout = ArenaLayout(shapes)
    rs = synth_replicas(layout, K, coll.rank, dev)
    reps = rs.data
    conv_ms = None
    if layout_kind == "elem":
        # what moving the training loop's [K, n] set into the step's layout costs (untimed in the step)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        reps = rs.data.t().contiguous()  # [n, K]
        e1.record()
        e1.synchronize()
        conv_ms = e0.elapsed_time(e1)
        del rs
        torch.cuda.empty_cache()
    eng = Sparta(coll, K, layout.n, dev, torch.float32, p, layout=layout_kind)
    timer = KernelTimer()
    avg_local = ops.sparta_average_local
    ops.sparta_average_local = timer.wrap(avg_local)
    it = [0]
    if mask_source == "torch":
        from gym_amd.strategy.sparta import MaskDraw, RandomIndexSelector, draw_masks
        sel, draw = RandomIndexSelector(p), MaskDraw()
        mask = torch.zeros(layout.n, dtype=torch.uint8, device=dev)
        mviews = layout.views(mask)
        mbits = torch.zeros(ops.sparta_mask_words(layout.n), dtype=torch.int64, device=dev)
        torch.manual_seed(42)

    def step():
        if mask_source == "torch":
            packed = draw_masks(sel, mviews, mviews, set(), it[0], draw, bits=mbits, coll=coll, defer=True)
            eng(reps, mask=mask if packed is None else packed, mask_cap=eng.cap, mask_shared=packed is not None)
        else:
            eng(reps, seed=42, iteration=it[0])
        it[0] += 1

    timer.on = True
    try:
        t = timed_loop(step, args.steps, args.warmup, coll)
    finally:
        ops.sparta_average_local = avg_local
    kern = timer.mean_ms()
    # events around single launches measure host launch latency at this size; the
    # queued form brackets GPU work only (agrees with rocprofv3's kernel durations)
    queued = queued_ms(step, args.steps, dev) if coll.world == 1 else None
    eng.check()
    # the number selected (untimed; the fused single-GPU pass produces no list)
    ops.sparta_select(reps, layout.n, eng.cap, eng.idx, eng.vals, eng.count, eng.work, seed=42, iteration=0, p=p,
                      layout=layout_kind)
    M = int(eng.count[0].item())
    alg = 2 * 4 * K * M + (8 * M if coll.world > 1 else 0)  # K-replica gather + write-back (+ idx/vals list)
    # what HBM must move at its access granularity: rows -> each selected (element,
    # replica) is a random 4-B word = one 64-B read sector + one 32-B write sector;
    # elem -> one element's K values are ceil(4K/64) whole 64-B sectors each way
    sect = (64 + 32) * K * M if layout_kind == "rows" else 2 * 64 * -(-4 * K // 64) * M
    sect += 8 * M if coll.world > 1 else 0  # the packed idx/vals list
    out = {"ms_per_step": round(t * 1e3, 4),
           "layout": "[n, K] element-major" if layout_kind == "elem" else "[K, n] rows",
           "K_local": K, "K_total": K * coll.world, "p": p, "selected": M, "alg_bytes": alg,
           "alg_GBps": round(alg / t / 1e9, 1), "sector_bytes": sect, "sector_GBps": round(sect / t / 1e9, 1),
           "sector_over_alg": round(sect / max(alg, 1), 3),
           "path": "fused select+gather+average+write-back" if coll.world == 1 else
                   f"select+gather, {'RCCL' if coll.rccl else coll.backend} all-reduce of packed values, scatter",
           "mask_source": mask_source}
    if mask_source == "torch":
        out["mask_draw"] = draw.mode  # "fused" (ga_sparta_torch_bernoulli) or "torch" (the per-tensor fallback)
        out["mask"] = ("the reference's per-tensor torch.bernoulli draws, bit-identical, " +
                       ("drawn inside the average kernel (GA_MASK_TORCH), in the step" if coll.world == 1 and
                        not coll.exchange else "as one ga_sparta_torch_bernoulli launch writing the packed mask, "
                        "in the step") +
                       ("" if coll.world == 1 else "; every rank draws rank 0's masks from its broadcast generator "
                        f"state: 16 B on the wire instead of the reference's {layout.n} B of masks"))
    if coll.exchange:  # the packed-value all-reduce alone (~pN fp32, latency-bound)
        cap = eng.cap
        t_ar = timed_loop(lambda: coll.all_reduce_(eng.vals[:cap]), args.steps, args.warmup, coll)
        out["xgmi"] = xgmi_block("all_reduce", 4 * cap, t_ar * 1e3, coll.world, step_ms=t * 1e3,
                                 what="all-reduce of the packed selected values (capacity pN + 16 sigma + 1024)",
                                 latency_bound=True)
    if queued is not None:
        out["kernel_ms"] = round(queued, 4)
        out["kernel_alg_GBps"] = round(alg / (queued * 1e-3) / 1e9, 1)
        out["kernel_frac_hbm"] = round(alg / (queued * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        out["kernel_ms_single_launch_events"] = round(kern, 4) if kern is not None else None
    elif kern is not None:
        out["kernel_ms"] = round(kern, 4)
    if conv_ms is not None:
        out["rows_to_elem_transpose_ms"] = round(conv_ms, 3)
    if mask_source == "torch" and coll.world == 1 and "kernel_ms" in out:
        # the reference draw's VALU roofline: the same n / 4 Philox4x32-10 calls in the
        # draw's launch shape with nothing compared or stored (ga_probe_philox), and the
        # draw alone (ga_sparta_torch_bernoulli into the packed words), in this process
        sink = torch.zeros(1, dtype=torch.int32, device=dev)
        ceil_ms = queued_ms(lambda: ops.probe_philox(layout.n, sink), args.steps, dev)
        table, nblocks = ops.sparta_bernoulli_table(layout.offsets, layout.numels, dev)
        bits = torch.zeros(ops.sparta_mask_words(layout.n), dtype=torch.int64, device=dev)
        draw_ms = queued_ms(lambda: ops.sparta_torch_bernoulli(table, nblocks, p, 1234, 0, 12, bits), args.steps, dev)
        out["valu_roofline"] = {
            "bound": "valu", "philox_calls": -(-layout.n // 4), "philox_ceiling_ms": round(ceil_ms, 4),
            "draw_alone_ms": round(draw_ms, 4), "draw_frac_of_ceiling": round(ceil_ms / draw_ms, 3),
            "step_frac_of_ceiling": round(ceil_ms / out["kernel_ms"], 3),
            "what": "ga_probe_philox: the n/4 Philox4x32-10 calls of the reference's torch.bernoulli stream in the "
                    "draw's launch shape (one lane per 64-element word, four chains), words XOR-folded, nothing "
                    "stored -- the arithmetic the reference's stream demands; frac = ceiling / measured"}
    if layout_kind == "rows" and coll.world == 1 and "kernel_ms" in out:
        # what this layout can reach: the same (position, replica) words read and written
        # back by a bare probe kernel (no mask, no sums) on the positions this step
        # selected (the Philox draw's: the same number of uniformly random positions as a
        # reference-draw step), in this process: the random-word floor.  At the sector
        # granularity (one 64-B read + one 32-B write sector per word) the copy rate would
        # allow sector_bytes / copy rate -- random 4-B words do not stream at it.
        pos = eng.idx[:M]
        floor_rmw = queued_ms(lambda: ops.probe_random_words(reps, pos, M, write=True), args.steps, dev)
        floor_rd = queued_ms(lambda: ops.probe_random_words(reps, pos, M, write=False), args.steps, dev)
        copy = getattr(args, "copy_GBps", None)
        out["random_word_floor"] = {
            "probe_rmw_ms": round(floor_rmw, 4), "probe_read_ms": round(floor_rd, 4),
            "kernel_over_probe_rmw": round(out["kernel_ms"] / floor_rmw, 3),
            "probe_rmw_sector_GBps": round(sect / (floor_rmw * 1e-3) / 1e9, 1),
            "sector_floor_ms_at_copy_rate": round(sect / (copy * 1e9) * 1e3, 4) if copy else None,
            "what": "ga_probe_random_words on this step's selected positions of the same [K, n] set: every "
                    "(position, replica) fp32 word read and written back (rmw) or read (read), no mask; the rows "
                    "kernel's floor at this access pattern"}
    return out


def bench_sparta_replica_step(args, coll, dev, K=32, p=0.005, model="gpt2-124m"):
    """configs[3] as the replica training loop runs it (gym_amd.replica, one GPU):
    the inner AdamW over the 32 nodes' [K, ld] rows (ga_adam_step) followed by
    SPARTA's sparse average with the reference's torch.bernoulli draw in-kernel
    (ga_sparta_average_local, rows layout; communicate_optimize_strategy.py:67-85).
    added_ms = what the SPARTA average adds to the AdamW pass.  (A fused
    element-major AdamW + average pass measured no faster: the element-major
    traversal of 32 rows costs ~0.9 ms over the replica-major AdamW,
    profiles/r04f_ubench_adam_sparta.txt.)"""
    if coll.world > 1:
        return {"skipped": "single-GPU replica loop (no exchange)"}
    shapes = MODELS[model]()
    layout = ArenaLayout(shapes)
    ld = layout.n
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    P = torch.randn(K, ld, device=dev, generator=g).mul_(0.02)
    G = torch.randn(K, ld, device=dev, generator=g).mul_(1e-3)
    M, V = torch.zeros_like(P), torch.zeros_like(P)
    table, _ = ops.sparta_bernoulli_table(layout.offsets, layout.numels, dev)
    draw = ops.TorchDraw(table, p, 42, 0, 12)
    hp = dict(lerp_w=0.1, beta2=0.999, one_m_beta2=1 - 0.999, eps=1e-8, wd_factor=1 - 1e-3 * 0.01, l2_wd=0.0,
              step_size=-1e-3 / 0.1, bc2_sqrt=(1 - 0.999) ** 0.5)
    reps = max(5, args.steps // 2)
    adam_one = queued_ms(lambda: ops.adam_step(P, G, M, V, **hp), reps, dev)  # one launch, ordinary moments
    # the product's step (fused_optim.ArenaAdam at K > 1): each replica's moment rows placed
    # on their own against that replica's parameter / gradient rows, one launch per replica
    from gym_amd.fused_optim import place_moment_rows
    Mr, Vr, bufs, prec = place_moment_rows(P, G, list(M.unbind(0)), list(V.unbind(0)))
    if any(b is not None for b in bufs):
        del M, V
        torch.cuda.empty_cache()

    def adam_rows():
        for k in range(K):
            ops.adam_step(P[k], G[k], Mr[k], Vr[k], **hp)
    adam = queued_ms(adam_rows, reps, dev)
    step = queued_ms(lambda: (adam_rows(),
                              ops.sparta_average_local(P, ld, float(K), mask=draw, layout="rows")), reps, dev)
    alg = 28 * K * ld  # read p, g, m, v; write p, m, v
    del P, G, Mr, Vr, bufs
    return {"model": model, "K": K, "p": p, "mask": "the reference's torch.bernoulli draw, in-kernel",
            "adamw_alone_ms": round(adam, 4), "adamw_then_sparta_ms": round(step, 4),
            "added_ms": round(step - adam, 4),
            "adamw_what": "ArenaAdam's K > 1 step: moment rows placed per replica (place_moment_rows), one "
                          "ga_adam_step launch per replica",
            "adamw_one_launch_unplaced_ms": round(adam_one, 4),
            "adamw_one_launch_unplaced_frac_hbm": round(alg / (adam_one * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "placement": {k: v for k, v in prec.items() if k != "probe_ms"},
            "adamw_alg_GBps": round(alg / (adam * 1e-3) / 1e9, 1),
            "adamw_frac_hbm": round(alg / (adam * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def bench_simple(args, coll, dev, K_total=8, model="gpt2-char"):
    """configs[1]: 8 char-level nodes, on one GPU or one per GPU (8/G per GPU)."""
    K = max(1, K_total // coll.world)
    shapes = MODELS[model]()
    layout = ArenaLayout(shapes)
    layout.n = layout.padded_to(coll.world)
    rs = synth_replicas(layout, K, coll.rank, dev)
    eng = MeanReduce(coll, K, layout.n, dev, torch.float32)
    # as the replica loop does: the mean may move the set it averages into the memory it
    # runs fastest on, once, at its first call (MeanReduce._place; sets of >= 32 MB per row)
    eng.relocate_replicas = rs.relocate
    t = timed_loop(lambda: eng(rs.data), args.steps, args.warmup, coll)
    out = {"ms_per_step": round(t * 1e3, 4), "param_GBps": round(K * coll.world * 4 * numel(shapes) / t / 1e9, 1),
           "K_local": K, "K_total": K * coll.world, "model": model}
    if coll.exchange:  # the exchange alone: one all-reduce of the arena (RS + AG when sharded)
        full = rs.data[0, :layout.n]
        if eng.shard:
            shard = torch.empty(layout.n // coll.world, device=dev)

            def exch():
                coll.reduce_scatter(shard, full)
                coll.all_gather_into(full, shard)
        else:
            def exch():
                coll.all_reduce_(full)
        t_x = timed_loop(exch, args.steps, args.warmup, coll)
        S = 4 * layout.n
        out["xgmi"] = xgmi_block("all_reduce", S, t_x * 1e3, coll.world, step_ms=t * 1e3,
                                 what=("reduce_scatter + all_gather" if eng.shard else "one all-reduce") +
                                      f" of the {S / 1e6:.1f} MB gradient arena alone",
                                 latency_bound=S < (32 << 20))
    if coll.world == 1:  # one ga_replica_mean launch: read K replicas, write K
        q = queued_ms(lambda: eng(rs.data), args.steps, dev)
        alg = 2 * K * 4 * layout.n
        out.update({"kernel_ms": round(q, 4), "kernel_alg_GBps": round(alg / (q * 1e-3) / 1e9, 1),
                    "kernel_frac_hbm": round(alg / (q * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
        pl = eng.placement
        if pl and pl.get("probe_ms"):
            out["placement"] = {"candidates": pl["candidates"], "chosen": pl["chosen"],
                                "probe_ms_own_vs_best": [pl["probe_ms"][0], min(pl["probe_ms"])]}
    return out


def bench_demo(args, coll, dev, model="gpt2-350m"):
    shapes = MODELS[model]()
    layout = ArenaLayout(shapes)
    P = synth_replicas(layout, 1, 0, dev).data  # identical params on every node
    G = synth_replicas(layout, 1, coll.rank + 7, dev).data
    D = torch.zeros_like(P)
    codec = DeMoCodec(coll, 1, layout, dev)
    plan = codec.plan
    # the decode of 8 gathered payloads (what every GPU runs at 8 nodes): 8 nodes' own
    # payloads, each encoded from its own gradient (seeds 7..14) on the shared start,
    # so every chunk sees up to 8 * 32 distinct coefficients with 1-8 hitters each
    gathered8 = torch.empty(8, codec.payload.shape[1], dtype=torch.int32, device=dev)
    Gk, Dk = torch.empty_like(G), torch.empty_like(D)
    gk = torch.Generator(device=dev)
    for k in range(8):
        gk.manual_seed(7 + k)
        Gk.normal_(0.0, 1e-3, generator=gk)
        Dk.zero_()
        ops.demo_encode(plan, P, Gk, Dk, gathered8[k:k + 1], 1e-3, 0.999, 1.0)
    del Gk, Dk
    # the product's placement (the DeMo optimizer after its first step, probing with the
    # payload it gathered: 8 sources at 8 nodes): G, P, D moved into the allocations the
    # step runs fastest on
    from gym_amd.placement import policy
    ok, why = policy(True)  # as the DeMo optimizer decides (no placement when ranks share a GPU)
    placed, placement = None, {"placed": False, "why": why}
    if ok:
        scratch = torch.empty_like(codec.payload)
        placed, moved, placement = place_demo_step(
            lambda p, g, d: ops.demo_encode(plan, p, g, d, scratch, 1e-3, 0.999, 1.0),
            lambda p, g: ops.demo_decode(plan, gathered8, p, g, 0.0), P, G, D)
        del scratch
    if placed is not None:
        P, G, D = moved
        placement["probed_with"] = "the 8-source payload"
    te, td = KernelTimer(), KernelTimer()
    codec.encode = te.wrap(codec.encode)
    codec.decode = td.wrap(codec.decode)
    te.on = td.on = True
    t = timed_loop(lambda: codec(P, G, D, 1e-3, 0.999, 0.0), args.steps, args.warmup, coll)
    flops_one = 0
    for s in shapes:
        from gym_amd.demo_codec import codec_view
        R, C, n1, n2 = codec_view(s, 64)
        flops_one += 2 * (R // n1) * (C // n2) * 2 * 64 ** 3  # two zero-padded 64^3 products per transform
    enc_ev, dec_ev = te.mean_ms(), td.mean_ms()
    te.on = td.on = False
    overlap = None
    if plan.M >= 32000:  # distinct (chunk, coefficient) hits over the 8 payloads, first 1000 chunks of wte
        e = torch.arange(32000, device=dev) // 32  # wte: 64x64 chunks, k = 32, chunk-local indices
        key = e[None, :] * 4096 + gathered8[:, :32000].long()
        overlap = round(float(torch.unique(key).numel()) / key.numel(), 4)
    t8 = KernelTimer()
    dec8 = t8.wrap(lambda: ops.demo_decode(plan, gathered8, P, G, 1e-3))
    t8.on = True
    timed_loop(dec8, args.steps, args.warmup, coll)
    dec8_ev = t8.mean_ms()
    t8.on = False
    tn = KernelTimer()  # the same decode without the grad write (p only)
    decn = tn.wrap(lambda: ops.demo_decode(plan, codec.payload[0:1], P, None, 1e-3))
    tn.on = True
    timed_loop(decn, args.steps, args.warmup, coll)
    # the kernels' GPU time, as the headline's kernel_ms (and rocprofv3) measure it: launches
    # queued back to back behind streaming copies; single-launch events add the host's launch
    # gap and are kept beside them
    reps_q = max(args.steps, 10)
    enc_ms = queued_ms(lambda: codec.encode(P, G, D, 1e-3, 0.999, 0.0), reps_q, dev)
    dec_ms = queued_ms(lambda: codec.decode(P, G, 1e-3), reps_q, dev)
    dec8_ms = queued_ms(lambda: ops.demo_decode(plan, gathered8, P, G, 1e-3), reps_q, dev)
    pipe_ms = None
    if coll.exchange and coll.rccl:  # the exchange as the strategies run it: async all-gathers of tensor groups
        from gym_amd.engine import DEMO_PIECES, PipelinedDeMoCodec
        pipe = PipelinedDeMoCodec(coll, 1, layout, dev, pieces=DEMO_PIECES)
        pipe_ms = timed_loop(lambda: pipe(P, G, D, 1e-3, 0.999, 0.0), args.steps, args.warmup, coll) * 1e3
        del pipe
    xgmi = None
    if coll.exchange:  # the payload all-gather alone, (G-1) * P bytes into every GPU
        ag_ms = timed_loop(codec.exchange, args.steps, args.warmup, coll) * 1e3
        Pb = codec.payload.numel() * 4
        step_ms = pipe_ms if pipe_ms is not None else t * 1e3
        xgmi = xgmi_block("all_gather", Pb, ag_ms, coll.world, step_ms=step_ms,
                          what=f"all-gather of the packed DeMo payload (int32 idx + fp32 val, {Pb / 1e6:.1f} MB "
                               f"per rank) alone")
        # how much of it the step hides behind the codec kernels: the step's time beyond
        # encode + decode, against the all-gather alone
        exposed = max(0.0, step_ms - (enc_ev + dec_ev))
        xgmi["codec_kernels_ms"] = round(enc_ev + dec_ev, 4)
        xgmi["exposed_ms"] = round(exposed, 4)
        xgmi["hidden_frac"] = round(max(0.0, min(1.0, 1.0 - exposed / ag_ms)), 4) if ag_ms > 0 else None
        xgmi["step"] = "pipelined over tensor groups (async RCCL)" if pipe_ms is not None else "one exchange"
    n = numel(shapes)
    copy = getattr(args, "copy_GBps", None)
    # the encode's access-pattern floor on this box: the chunk kernels' 64x64 traffic with no
    # transform (ga_probe_chunk_stream) over a [rows, 1024] matrix of ~n elements, scaled to n
    cols = 1024
    rows = (n // cols) // 64 * 64
    scale = n / (rows * cols)
    flo_enc = min(queued_ms(lambda: ops.probe_chunk_stream(D.view(-1), G.view(-1), rows, cols, m), args.steps, dev)
                  for m in (0, 2)) * scale  # plain and non-temporal: the faster is the floor

    # algorithmic HBM bytes: encode reads delta, g and writes delta (wd = 0) + the
    # payload; decode reads p, writes p and grad + S payloads (8 B per entry)
    enc_bytes = 12 * n + 8 * plan.M
    dec_bytes = 12 * n + 8 * plan.M
    return {"ms_per_step": round(t * 1e3, 4), "model": model, "nodes": coll.world,
            "ms_per_step_pipelined": round(pipe_ms, 4) if pipe_ms is not None else None,
            "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4), "decode_8src_ms": round(dec8_ms, 4),
            "decode_nograd_ms": round(tn.mean_ms(), 4),
            "kernel_timing": "encode_ms / decode_ms / decode_8src_ms: HIP events around back-to-back launches queued "
                             "behind streaming copies (queued_ms, GPU time as rocprofv3 measures it); *_single_launch_"
                             "events: events around each launch of the timed step loop",
            "encode_ms_single_launch_events": round(enc_ev, 4), "decode_ms_single_launch_events": round(dec_ev, 4),
            "decode_8src_ms_single_launch_events": round(dec8_ev, 4),
            "decode_8src_input": "8 distinct nodes' payloads (own gradients, seeds 7..14)",
            "decode_8src_distinct_entry_frac": overlap,
            "encode_HBM_GBps": round(enc_bytes / (enc_ms * 1e-3) / 1e9, 1),
            "decode_HBM_GBps": round(dec_bytes / (dec_ms * 1e-3) / 1e9, 1),
            "decode_8src_HBM_GBps": round((dec_bytes + 7 * 8 * plan.M) / (dec8_ms * 1e-3) / 1e9, 1),
            # against 8 TB/s and against this process's streaming copy (the DiLoCo line's copy_GBps)
            "encode_frac_hbm": round(enc_bytes / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "decode_8src_frac_hbm": round((dec_bytes + 7 * 8 * plan.M) / (dec8_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "encode_frac_of_copy": round(enc_bytes / (enc_ms * 1e-3) / 1e9 / copy, 4) if copy else None,
            "decode_8src_frac_of_copy": (round((dec_bytes + 7 * 8 * plan.M) / (dec8_ms * 1e-3) / 1e9 / copy, 4)
                                         if copy else None),
            # the MFMA work the kernels issue: the DCT products folded by F[63-i][k] = (-1)^k F[i][k]
            # (half the dense formulation's 2 * 64^3 per product) and the residual as sparse synthesis,
            # so SURVEY 8(d)'s dense flop count is not a bound for them; the MFMA pipe is busy 41% of
            # the encode's SIMD cycles (profiles/r02l_pmc_demo_encode.txt)
            "dense_formulation_GFLOP_per_encode": round(2 * flops_one / 1e9, 1),
            "encode_access_pattern_floor": {
                "ms": round(flo_enc, 4), "frac": round(flo_enc / enc_ms, 3),
                "what": "ga_probe_chunk_stream: one wavefront per 64x64 chunk in the encode kernel's grid and "
                        "coalesced layout, its 12 B per element (read delta, g; write delta) with no transform, "
                        "over a [rows, 1024] fp32 matrix scaled to the model's element count, plain and "
                        "non-temporal streams (the faster counts); frac = floor / encode time.  (The decode's "
                        "pattern probed this way ran slower than the 1-source decode itself, so it is no floor "
                        "and is not reported.)"},
            "payload_entries": plan.M, "ref_bytes_tx": plan.reference_bytes(), "xgmi": xgmi,
            "placement": placement}


def bench_demo_bf16(args, coll, dev, model="gpt2-350m"):
    """DeMo on bf16 parameters (one node, GPT-2 350M): the default transform
    (fp32 bases and arithmetic on the bf16 values: the wave kernels) and
    bf16_transform="reference" (GA_BF16_REF: the reference's bf16 bases and
    per-stage bf16 rounding, bit-identical to torch's op sequence on the GPU:
    the block kernels).  Kernel GPU time queued back to back, as the fp32 DeMo
    line; 1-source and 8-source decodes.  No BASELINE config is bf16: this
    prices the drop-in's bf16 path."""
    if coll.world > 1:
        return {"skipped": "single-GPU kernel timing"}
    from gym_amd.demo_codec import DemoPlan
    shapes = MODELS[model]()
    layout = ArenaLayout(shapes)
    bf = torch.bfloat16
    P = synth_replicas(layout, 1, 0, dev).data.to(bf)
    G = synth_replicas(layout, 1, 7, dev).data.to(bf)
    D = torch.zeros_like(P)
    out = {"model": model, "dtype": "bf16"}
    reps_q = max(args.steps, 10)
    for name in ("fp32", "reference"):
        plan = DemoPlan(layout, chunk=64, topk=32, bf16_transform=name).to(dev)
        pay = torch.zeros(8, 2 * plan.M, dtype=torch.int32, device=dev)
        gk = torch.Generator(device=dev)
        Gk = torch.empty_like(G)
        for k in range(8):  # 8 nodes' own payloads, as the fp32 line's 8-source decode
            gk.manual_seed(7 + k)
            Gk.copy_(torch.randn(G.shape, device=dev, generator=gk).mul_(1e-3))
            D.zero_()
            ops.demo_encode(plan, P, Gk, D, pay[k:k + 1], 1e-3, 0.999, 1.0)
        del Gk
        D.zero_()
        enc = queued_ms(lambda: ops.demo_encode(plan, P, G, D, pay[0:1], 1e-3, 0.999, 1.0), reps_q, dev)
        dec1 = queued_ms(lambda: ops.demo_decode(plan, pay[0:1], P, G, 1e-3), reps_q, dev)
        dec8 = queued_ms(lambda: ops.demo_decode(plan, pay, P, G, 1e-3), reps_q, dev)
        n = numel(shapes)
        byt = 6 * n + 8 * plan.M  # bf16: read delta, g; write delta (2 B each) + the payload
        out[f"transform_{name}"] = {
            "kernels": "wave (ga_demo_encode_sym / decode_sym)" if plan.wave_encode else "block (ga_demo_encode / decode)",
            "encode_ms": round(enc, 4), "decode_ms": round(dec1, 4), "decode_8src_ms": round(dec8, 4),
            "encode_frac_hbm": round(byt / (enc * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        del pay
    return out


def bench_diloco_torch_gpu(args, coll, dev, fused_ms, model="gpt2-124m", K=8):
    """The reference's DiLoCo outer step (diloco.py:34-76) as per-tensor torch
    ops on this GPU, the un-fused baseline on the same hardware: for each of
    the model's tensors the K nodes' values are summed and divided (the
    all_reduce(SUM) + `/= num_nodes` of :34-37, here over K local replicas),
    master.grad = master - avg (:43-45), torch.optim.SGD(lr 0.7, momentum
    0.9, nesterov; foreach) steps the master (:70), and every node copies the
    master (:47-49 + :39-41)."""
    shapes = MODELS[model]()
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    base = [torch.randn(*sh, device=dev, generator=g) * 0.02 for sh in shapes]
    reps = [[b + torch.randn(b.shape, device=dev, generator=g) * 1e-3 for b in base] for _ in range(K)]
    master = [torch.nn.Parameter(b.clone()) for b in base]
    opt = torch.optim.SGD(master, lr=0.7, momentum=0.9, nesterov=True)

    @torch.no_grad()
    def step():
        for i, m in enumerate(master):
            acc = reps[0][i].clone()
            for k in range(1, K):
                acc.add_(reps[k][i])
            acc /= K
            m.grad = m.data - acc
        opt.step()
        for i, m in enumerate(master):
            for k in range(K):
                reps[k][i].copy_(m.data)

    t = timed_loop(step, max(3, args.steps // 4), 2, coll)
    del reps, master, base
    return {"ms_per_step": round(t * 1e3, 4), "model": model, "nodes": K, "tensors": len(shapes),
            "fused_ms_per_step": round(fused_ms, 4), "fused_speedup": round(t * 1e3 / fused_ms, 2),
            "what": "reference op sequence per tensor in torch on this GPU (sum over K replicas, divide, "
                    "master grad, torch SGD-Nesterov foreach, copy to every node)"}


def bench_inner_adamw(args, coll, dev, model="gpt2-124m", max_norm=1.0):
    """Inner optimizer step on one node's arena: fused
    clip + AdamW (ga_grad_clip_coef + ga_adam_step) vs torch.optim.AdamW
    (foreach, the reference's default) + clip_grad_norm_ on the same GPU."""
    from gym_amd.arena import ParamArena
    from gym_amd.fused_optim import ArenaAdam
    shapes = MODELS[model]()
    params = [torch.nn.Parameter(torch.randn(*sh, device=dev) * 0.02) for sh in shapes]
    arena = ParamArena(params)
    arena.grad_flat.normal_(0.0, 1e-3)
    opt = ArenaAdam(params, arena, lr=1e-3)
    timer = KernelTimer()
    ops_adam = ops.adam_step
    ops.adam_step = timer.wrap(ops.adam_step)
    timer.on = True
    t = timed_loop(lambda: opt.step(max_norm=max_norm), args.steps, args.warmup, coll)
    kern = timer.mean_ms()
    ops.adam_step = ops_adam
    tparams = [torch.nn.Parameter(torch.randn(*sh, device=dev) * 0.02) for sh in shapes]
    for p in tparams:
        p.grad = torch.randn_like(p) * 1e-3
    topt = torch.optim.AdamW(tparams, lr=1e-3, foreach=True)

    def ref_step():
        torch.nn.utils.clip_grad_norm_(tparams, max_norm)
        topt.step()

    tt = timed_loop(ref_step, args.steps, args.warmup, coll)
    n = arena.n
    alg = 28 * n  # read p, g, m, v; write p, m, v
    return {"model": model, "n": n, "ms_per_step": round(t * 1e3, 4), "kernel_ms": round(kern, 4),
            "kernel_GBps": round(alg / (kern * 1e-3) / 1e9, 1),
            "kernel_frac_hbm": round(alg / (kern * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "torch_adamw_foreach_ms": round(tt * 1e3, 4), "speedup_vs_torch": round(tt / t, 2),
            "placement": {k: v for k, v in (opt.placement or {}).items() if k != "probe_ms"} or None,
            "placement_probe_ms_best_vs_ordinary": ([round(min(opt.placement["probe_ms"]), 4),
                                                     opt.placement["probe_ms"][0]]
                                                    if opt.placement and "probe_ms" in opt.placement else None)}


def replicas_per_gpu(nodes, world, override=None):
    """Simulated nodes each GPU hosts: `override` (--replicas) if given, else
    the configuration's node count spread over the GPUs (8 nodes: 8 / 4 / 2 / 1
    per GPU at N = 1 / 2 / 4 / 8), at least one.  The total is then
    replicas x world (= nodes when world divides it)."""
    if override:
        return int(override)
    if nodes % world:
        raise SystemExit(f"--nodes {nodes} is not a multiple of {world} GPUs (give --replicas per GPU instead)")
    return max(1, nodes // world)


def launch_world(args):
    """World size this process will run at: torchrun's WORLD_SIZE, else --gpus."""
    return int(os.environ["WORLD_SIZE"]) if "WORLD_SIZE" in os.environ else args.gpus


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def child_command(argv, gpus, port):
    """The torch.distributed.run command of a self-launched N-rank bench: one
    rank per GPU on this node, 127.0.0.1 rendezvous, the parent's arguments
    passed on (the host legs already ran in the parent: --no-cpu-baseline)."""
    rest = [a for a in argv if a != "--no-cpu-baseline"]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.join(ROOT, "bench.py"), *rest, "--no-cpu-baseline"]


def merge_child_line(stdout_text, cpu, legs, cmd):
    """Rank 0's one JSON line from the child's stdout, with the parent's CPU
    baseline and host legs merged in; None when the child printed none."""
    line = None
    for raw in stdout_text.splitlines():
        raw = raw.strip()
        if raw.startswith("{") and '"metric"' in raw:
            try:
                line = json.loads(raw)
            except ValueError:
                continue
    if line is None:
        return None
    line["cpu_baseline"] = cpu
    hl = dict(line.get("host_legs_s") or {})
    hl.update({f"parent_{k}": v for k, v in legs.items()})
    line["host_legs_s"] = hl
    line["launch"] = ("self-launched: this process ran the host legs without touching the GPU, then "
                      f"`{' '.join(os.path.basename(c) if c == sys.executable else c for c in cmd[1:7])} ...` "
                      "as a child process; rank 0's line")
    return line


def self_launch(args, argv):
    """`bench.py --gpus N` (N > 1) outside torchrun: host legs here, N ranks in a
    fresh torch.distributed.run child (this process never initialises the GPU,
    so nothing execs from a GPU-initialised process).  Returns the exit code."""
    import subprocess
    legs = {}
    t0 = time.perf_counter()
    cpu = None
    if not args.no_cpu_baseline and args.only is None:
        cpu = cpu_baseline_diloco(args.model, args.nodes)
    legs["cpu_baseline_s"] = round(time.perf_counter() - t0, 1)
    cmd = child_command(argv, args.gpus, free_port())
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this pool
    print(f"[bench] self-launch: {' '.join(cmd)}", file=sys.stderr, flush=True)
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True)
    line = merge_child_line(r.stdout, cpu, legs, cmd)
    if line is None:
        sys.stderr.write(r.stdout[-4000:])
        print(f"[bench] the {args.gpus}-rank child printed no JSON line (rc {r.returncode})", file=sys.stderr)
        return r.returncode or 1
    print(json.dumps(line), flush=True)
    return r.returncode


def main():
    t_start = time.perf_counter()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="gpt2-124m")
    ap.add_argument("--nodes", type=int, default=8,
                    help="simulated nodes in total (configs[2]: 8), spread nodes/N per GPU")
    ap.add_argument("--replicas", type=int, default=None,
                    help="simulated nodes per GPU (overrides --nodes / N; e.g. 8 for the weak-scaled form)")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--only", default=None,
                    help="diloco|sparta|simple|demo|adamw or an extras name, e.g. sparta_k32_rows_torch_mask "
                         "(profiling runs)")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if os.environ.get("GA_BENCH_WATCHDOG"):  # debugging aid: Python stacks on stderr every N s
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["GA_BENCH_WATCHDOG"]), repeat=True, file=sys.stderr)
    if args.gpus > 1 and "RANK" not in os.environ and not args.pmc_child:
        sys.exit(self_launch(args, sys.argv[1:]))
    single = args.gpus == 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1
    args.replicas = replicas_per_gpu(args.nodes, launch_world(args), args.replicas)
    rank0 = int(os.environ.get("RANK", "0")) == 0
    if args.pmc_child:  # a rocprofv3 PMC pass: the headline kernel only, a few launches
        coll = setup_dist(1)
        dev = torch.device("cuda", 0)
        bench_diloco(argparse.Namespace(**{**vars(args), "steps": 3, "warmup": 1}), coll, dev)
        return
    # host-side legs first, while this process has not touched the GPU (the
    # children are started by fork+exec; none of them runs in a GPU-initialised process)
    cpu = None
    legs = {}
    t0 = time.perf_counter()
    if rank0 and not args.no_cpu_baseline and args.only is None:
        # at N > 1 under torchrun the other ranks wait in the rendezvous meanwhile; the
        # baseline is the reference's configs[2] job (8 gloo node processes) on this host
        cpu = cpu_baseline_diloco(args.model, args.nodes)
    legs["cpu_baseline_s"] = round(time.perf_counter() - t0, 1)
    args.pmc = (None, "not measured (N > 1 or --no-pmc)")
    t0 = time.perf_counter()
    if single and not args.no_pmc and args.only is None and not under_profiler():
        args.pmc = pmc_traffic_live(args)
    legs["pmc_passes_s"] = round(time.perf_counter() - t0, 1)

    coll = setup_dist(args.gpus)
    dev = torch.device("cuda", torch.cuda.current_device())
    torch.backends.cuda.matmul.allow_tf32 = False

    extra_runs = [("sparta_k32", bench_sparta),
                  ("sparta_k32_rows", lambda a, c, d: bench_sparta(a, c, d, layout_kind="rows")),
                  ("sparta_k32_rows_torch_mask",  # the replica training loop's own step: rows + the reference draw
                   lambda a, c, d: bench_sparta(a, c, d, layout_kind="rows", mask_source="torch")),
                  ("sparta_k32_torch_mask", lambda a, c, d: bench_sparta(a, c, d, mask_source="torch")),
                  ("sparta_k32_replica_step", bench_sparta_replica_step),
                  ("simple_reduce_char_k8", bench_simple),
                  # the same mean over GPT-2 124M gradients (SimpleReduce / FedAvg in the replica loop)
                  ("simple_reduce_124m_k8", lambda a, c, d: bench_simple(a, c, d, model="gpt2-124m")),
                  ("demo_350m", bench_demo), ("demo_350m_bf16", bench_demo_bf16),
                  ("inner_adamw_clip_124m", bench_inner_adamw)]
    if args.only and args.only != "diloco":
        fn = {"sparta": bench_sparta, "simple": bench_simple, "demo": bench_demo,
              "adamw": bench_inner_adamw, **dict(extra_runs)}[args.only]
        r = fn(args, coll, dev)
        if coll.rank == 0:
            print(json.dumps({"only": args.only, **r}), flush=True)
        return

    head = bench_diloco(args, coll, dev)
    extras = {}
    if not args.no_extras and args.only != "diloco":
        runs = list(extra_runs)
        if coll.world == 1:
            runs.insert(0, ("diloco_torch_per_tensor_gpu",
                            lambda a, c, d: bench_diloco_torch_gpu(a, c, d, head["ms_per_step"])))
        if coll.world > 1:  # the weak-scaled form: 8 nodes on every GPU (8N in total)
            def diloco_weak(a, c, d):
                r = bench_diloco(argparse.Namespace(**{**vars(a), "replicas": 8}), c, d)
                for key in ("ms_per_step", "value", "kernel_ms"):
                    r[key] = round(r[key], 4)
                r["scaling"] = "weak"
                return r
            runs.insert(0, ("diloco_8_nodes_per_gpu", diloco_weak))
        for name, fn in runs:
            if coll.rank == 0:  # progress on stderr (the JSON line stays the only stdout line)
                print(f"[bench] {name}", file=sys.stderr, flush=True)
            torch.cuda.empty_cache()
            t_leg = time.perf_counter()
            try:
                extras[name] = fn(args, coll, dev)
            except Exception as e:  # keep the headline line even if an extra fails
                extras[name] = {"error": repr(e)[:300]}
            extras[name]["leg_s"] = round(time.perf_counter() - t_leg, 1)
    if coll.rank != 0:
        if coll.world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    K_total = head["K_total"]
    line = {
        "metric": "strategy-step param GB/s (%HBM/xGMI peak) + ms/outer step, GPT-2 124M, 1-8 GPUs",
        "value": round(head["value"], 2),
        "unit": "GB/s",
        "n_gpus": coll.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(head["ms_per_step"], 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (GPT-2 124M parameter shapes, N(0,0.02) start + per-node N(0,1e-3) drift)",
        "config": {"workload": f"DiLoCo outer step (configs[2]), {args.model}, {K_total} simulated nodes in total, "
                               f"{args.replicas} per GPU ({'a batched-replica arena, ' if args.replicas > 1 else ''}"
                               f"fused average+pseudo-grad+Nesterov SGD(lr=0.7, mu=0.9)"
                               f"{(', RCCL reduce-scatter/all-gather' if coll.rccl else f', {coll.backend} all-reduce') + ' across GPUs' if coll.world > 1 else ''})",
                   "model": args.model, "nodes_per_gpu": args.replicas, "nodes_total": K_total,
                   "n_params": head["n_params"], "parallelism": f"dp{K_total} (simulated nodes)"},
        "roofline": head["roofline"],
        "cpu_baseline": cpu,
    }
    if "xgmi" in head:
        line["xgmi"] = head["xgmi"]
    if coll.exchange and coll.world == 1:
        line["rehearsal"] = "world-1 RCCL group with forced exchange: the multi-GPU code paths, not a measurement"
    if extras:
        line["extras"] = extras
    line["bench_wall_s"] = round(time.perf_counter() - t_start, 1)  # this process, CPU baseline + PMC passes included
    line["host_legs_s"] = legs
    print(json.dumps(line), flush=True)
    if coll.world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
