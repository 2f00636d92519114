"""Physical placement of the state buffers the strategy step owns (DiLoCo
master/momentum, AdamW moments): candidates probed with the step's own access
pattern, the fastest kept.

On MI355X the fused DiLoCo step runs 1.57-1.65 ms or 1.88 ms for the same
virtual layout (GPT-2 124M x 8 replicas), depending on where its streams sit
PHYSICALLY: device memory comes in regions of several GB whose addresses map to
the HBM channels/banks in different ways, and master/momentum in a region that
maps like the replica set's make the same-offset accesses of the 20 streams
collide (tools/ubench_diloco_layout.cpp map mode, profiles/r04i_placement_map.txt:
the (replica region, master region) grid is slow exactly where the two regions
share a class; tools/ubench_diloco_vmm.cpp, r04j: 1 GiB physical chunks created
one by one fall in either class).  Which class a buffer gets is the driver's
choice and differs between processes, so it cannot be fixed by a virtual layout.

The product's candidates are DeviceBuffer: fresh ordinary device allocations
(each a new block of the caching allocator, i.e. its own hipMalloc), created
one at a time and all held until the choice, so they land in different
physical regions; engines time the kernel's own access pattern on each (a probe
that writes every value back unchanged), keep the fastest and drop the rest.
At GPT-2 124M x 8 the DiLoCo candidates fall in the 1.88 / 1.74 / 1.69 /
1.76 ms classes and the chosen one runs the bench's step at 1.70 ms (frac
0.731, profiles/r04w_*).

Policy (round 5): placement is on by default and can be turned off per
strategy / optimizer (`placement=False`, e.g. DiLoCoStrategy(placement=False),
DeMo(..., placement=False)) or for the process (GA_PLACEMENT=0); it is skipped
by itself when several processes of the job share one GPU (more ranks than
visible devices, e.g. nodes over gloo on one card), since each would size its
candidates from the same free memory.  `policy()` decides and says why; the
engines record the decision and the probe times in their `placement` record,
which the strategies expose in __config__().

hipMemCreate candidates (tools/placed_buffer.py) reach the same classes but were
seen corrupted on this stack when interleaved with ordinary allocations
(profiles/r04u_vmm_alias.txt); they are kept for experiments under tools/ only.
This module only moves memory; every kernel stays behind the C ABI.
"""
import os
import socket
import time

import torch
import torch.distributed as dist


_VISIBLE_ENVS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")
_SHARING = None  # (process group, shared?) recorded by note_devices() for that group


def device_identity():
    """This process's GPU as the machine knows it: host, UUID and PCI location
    (the same physical card gives the same string in every process, whatever
    its visible-devices numbering)."""
    host = socket.gethostname()
    if not torch.cuda.is_available():
        return f"{host}|cpu"
    p = torch.cuda.get_device_properties(torch.cuda.current_device())
    pci = tuple(getattr(p, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    return f"{host}|{getattr(p, 'uuid', None)}|{pci}"


def note_devices(group=None):
    """Collective, once per process group right after init_process_group (the
    trainer's and the bench's setup do it): every rank's device_identity() is
    gathered and this rank records whether another rank of the group drives the
    same physical GPU.  Returns that answer (None without a process group)."""
    global _SHARING
    if not (dist.is_available() and dist.is_initialized()):
        return None
    group = group or dist.group.WORLD
    ids = [None] * dist.get_world_size(group)
    mine = device_identity()
    dist.all_gather_object(ids, mine, group=group)
    _SHARING = (group, ids.count(mine) > 1)
    return _SHARING[1]


def device_shared():
    """True when this process shares its GPU with other ranks of the job.  After
    note_devices(): by device identity.  Otherwise a heuristic: more ranks on
    this host (LOCAL_WORLD_SIZE) than visible devices -- the reference's
    nodes-over-gloo-on-one-card layout -- except under a launcher that pins one
    GPU per rank through a visible-devices variable (one device visible), which
    it cannot tell apart without the exchange and so does not call shared."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    if _SHARING is not None and _SHARING[0] is dist.group.WORLD:
        return _SHARING[1]
    local = int(os.environ.get("LOCAL_WORLD_SIZE", dist.get_world_size()))
    count = max(1, torch.cuda.device_count())
    if count == 1 and any(os.environ.get(v) for v in _VISIBLE_ENVS):
        return False
    return local > count


def policy(requested=True):
    """(enabled, reason): whether a step may probe and move its buffers now.
    requested = the owner's `placement` option (True by default)."""
    if requested is False:
        return False, "placement=False"
    if os.environ.get("GA_PLACEMENT", "1") == "0":
        return False, "GA_PLACEMENT=0"
    if device_shared():
        return False, "GPU shared by several processes of the job"
    return True, None


class DeviceBuffer:
    """One ordinary device allocation: the candidates the product probes.
    choose() empties the caching allocator's cache first, so each candidate of
    this size is a new block (its own hipMalloc) rather than cached memory; all
    are held until the choice, so each is distinct memory; `release()` drops
    it (choose() empties the cache again afterwards)."""

    def __init__(self, nbytes, device):
        self.nbytes = -(-int(nbytes) // 16) * 16
        self.device = torch.device(device)
        self._t = torch.empty(self.nbytes, dtype=torch.uint8, device=self.device)

    def tensor(self, dtype=torch.float32):
        return self._t.view(dtype)

    def release(self):
        self._t = None


class Stopwatch:
    """Wall time of one owner's placement search (its record's "search_s")."""

    def __init__(self):
        self.t0 = time.perf_counter()

    def stamp(self, record):
        if record is not None:
            record["search_s"] = round(time.perf_counter() - self.t0, 3)
        return record


def time_probe(fn, reps=3):
    """ms per call of fn (one warm-up, then reps calls between two events)."""
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


# wall-time cap of one candidate search when the caller gives no deadline (a box whose
# large allocations are slow took 4.2 s for AdamW's 48 candidates, profiles/r06q_bench.json)
SEARCH_BUDGET_S = 1.0


def choose(nbytes, device, probe, baseline_ms, max_candidates, max_frac, kind=DeviceBuffer, patience=None,
           min_gain=0.02, deadline=None):
    """Create up to max_candidates - 1 allocations of nbytes one at a time (all
    held until the choice is made, so each is distinct memory), time
    probe(buffer) on each, and return (the fastest buffer, or None when none
    beats baseline_ms -- the caller's own allocation --, every time in creation
    order with the baseline first).  At most max_frac of the free device memory
    is taken; an allocation failure (OutOfMemoryError) ends the search with what
    was probed.  Any other error -- a rejected or faulting probe launch -- is
    raised: the search must not hide a poisoned context.

    Budget: with `patience`, the search stops after that many candidates unless
    the best so far beats baseline_ms by more than min_gain (the caller's memory
    is then already in a fast class, and more candidates would only cost time);
    with `deadline` (a time.perf_counter() value; default SEARCH_BUDGET_S from
    now) no candidate is created after it.  The best candidate found is kept
    either way."""
    if deadline is None:
        deadline = time.perf_counter() + SEARCH_BUDGET_S
    dev = torch.device(device)
    torch.cuda.empty_cache()  # fresh blocks, not cached free memory
    times = [baseline_ms]
    best, best_t, held = None, baseline_ms, []
    budget = max_frac * torch.cuda.mem_get_info(dev)[0]
    try:
        while len(times) < max_candidates and (len(held) + 1) * nbytes <= budget:
            if deadline is not None and time.perf_counter() >= deadline:
                break
            if patience is not None and len(held) >= patience and best_t >= baseline_ms * (1.0 - min_gain):
                break
            try:
                buf = kind(nbytes, dev)
            except torch.cuda.OutOfMemoryError:
                break
            held.append(buf)
            t = probe(buf)
            times.append(t)
            if t < best_t:
                best, best_t = buf, t
    finally:
        for b in held:
            if b is not best:
                b.release()
        held = None
        torch.cuda.empty_cache()
    return best, times


def place_each(tensors, run, max_candidates, max_frac, reps=3):
    """Placement for buffers a step streams together (the DeMo step's gradient,
    parameters and delta), one buffer at a time: `run(*ts)` launches the step's
    kernels on any buffers of these shapes.  The buffers are snapshotted and the
    ordinary set timed; then for each buffer in turn up to max_candidates fresh
    allocations are probed with the others where they are by then (moved or
    not), and the fastest is kept when it beats the set's best time so far.
    Every buffer is restored from the snapshot (the probe may write what it
    likes) and each moved one receives its contents.  Returns (per buffer: its
    candidate buffer or None, per buffer: the tensor to use from now on, the
    stage times: ordinary set first)."""
    for t in tensors:
        if not t.is_contiguous():
            raise ValueError("place_each: contiguous buffers")
    saved = [t.clone() for t in tensors]  # the only allocation before the buffers are touched
    cur = list(tensors)
    placed = [None] * len(tensors)

    def view(buf, i):
        return buf.tensor(tensors[i].dtype)[:tensors[i].numel()].view(tensors[i].shape)

    best_t = time_probe(lambda: run(*cur), reps)
    stages = [best_t]
    for i, t in enumerate(tensors):
        def probe(buf, i=i):
            c = view(buf, i)
            c.copy_(saved[i])
            args = list(cur)
            args[i] = c
            return time_probe(lambda: run(*args), reps)
        best, times = choose(t.numel() * t.element_size(), t.device, probe, best_t, max_candidates, max_frac)
        if best is not None:
            placed[i], cur[i] = best, view(best, i)
            best_t = min(times)
        stages.append(min(times))
        torch.cuda.empty_cache()
    for t, c, sv in zip(tensors, cur, saved):
        t.copy_(sv)
        if c is not t:
            c.copy_(sv)
    return placed, cur, stages
