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

PlacedBuffer -- one hipMemCreate allocation mapped at its own virtual range,
wrapped via __cuda_array_interface__ -- is kept for the experiments under
tools/ only: its candidates reach 1.65-1.66 ms, but on this stack such
allocations were seen corrupted when interleaved with ordinary ones
(profiles/r04u_vmm_alias.txt), and the product's bit-exact churn test failed
with them once inside the full GPU suite.  This module only moves memory;
every kernel stays behind the C ABI.
"""
import ctypes
import os

import torch


class _Location(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]


class _AllocProp(ctypes.Structure):  # hipMemAllocationProp (hip_runtime_api.h)
    _fields_ = [("type", ctypes.c_int), ("requestedHandleType", ctypes.c_int), ("location", _Location),
                ("win32HandleMetaData", ctypes.c_void_p), ("compressionType", ctypes.c_ubyte),
                ("gpuDirectRDMACapable", ctypes.c_ubyte), ("usage", ctypes.c_ushort)]


class _AccessDesc(ctypes.Structure):  # hipMemAccessDesc
    _fields_ = [("location", _Location), ("flags", ctypes.c_int)]


_PINNED, _LOC_DEVICE, _PROT_RW, _GRAN_MIN = 1, 1, 3, 0
_HIP = None


def _hip():
    """The HIP runtime torch itself runs on (already loaded in this process)."""
    global _HIP
    if _HIP is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
        lib = ctypes.CDLL(path if os.path.exists(path) else "libamdhip64.so")
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        sig = {"hipMemGetAllocationGranularity": [ctypes.POINTER(sz), ctypes.POINTER(_AllocProp), ctypes.c_int],
               "hipMemCreate": [ctypes.POINTER(vp), sz, ctypes.POINTER(_AllocProp), ctypes.c_ulonglong],
               "hipMemAddressReserve": [ctypes.POINTER(vp), sz, sz, vp, ctypes.c_ulonglong],
               "hipMemMap": [vp, sz, sz, vp, ctypes.c_ulonglong],
               "hipMemSetAccess": [vp, sz, ctypes.POINTER(_AccessDesc), sz],
               "hipMemUnmap": [vp, sz], "hipMemRelease": [vp], "hipMemAddressFree": [vp, sz]}
        for name, args in sig.items():
            fn = getattr(lib, name)
            fn.argtypes, fn.restype = args, ctypes.c_int
        _HIP = lib
    return _HIP


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed (hipError {rc})")


def _prop(device_index):
    p = _AllocProp()
    p.type, p.requestedHandleType = _PINNED, 0
    p.location = _Location(_LOC_DEVICE, device_index)
    return p


def granularity(device):
    g = ctypes.c_size_t(0)
    p = _prop(torch.device(device).index or 0)
    _check(_hip().hipMemGetAllocationGranularity(ctypes.byref(g), ctypes.byref(p), _GRAN_MIN),
           "hipMemGetAllocationGranularity")
    return max(int(g.value), 1)


class _CAI:
    def __init__(self, ptr, numel, typestr):
        self.__cuda_array_interface__ = {"shape": (int(numel),), "typestr": typestr, "data": (int(ptr), False),
                                         "strides": None, "version": 2}


class PlacedBuffer:
    """One physical allocation of `nbytes` (rounded up to whole 2 MiB pages)
    mapped read-write at a virtual range of its own, on `device`.  Experiments
    only (tools/): not used by the product, see the module docstring."""

    ALIGN = 2 << 20  # virtual alignment of the mapping

    def __init__(self, nbytes, device):
        dev = torch.device(device)
        self.device = dev
        # whole 2 MiB pages (the minimum granularity the driver reports is 4 KiB);
        # see profiles/r04u_vmm_alias.txt for what is and is not safe with these
        # allocations on this stack
        gran = max(granularity(dev), self.ALIGN)
        self.nbytes = -(-int(nbytes) // gran) * gran
        hip = _hip()
        self.handle, self.va = ctypes.c_void_p(), ctypes.c_void_p()
        prop = _prop(dev.index or 0)
        _check(hip.hipMemCreate(ctypes.byref(self.handle), self.nbytes, ctypes.byref(prop), 0), "hipMemCreate")
        try:
            _check(hip.hipMemAddressReserve(ctypes.byref(self.va), self.nbytes, self.ALIGN, None, 0),
                   "hipMemAddressReserve")
            _check(hip.hipMemMap(self.va, self.nbytes, 0, self.handle, 0), "hipMemMap")
            acc = _AccessDesc(_Location(_LOC_DEVICE, dev.index or 0), _PROT_RW)
            _check(hip.hipMemSetAccess(self.va, self.nbytes, ctypes.byref(acc), 1), "hipMemSetAccess")
        except Exception:
            self.release()
            raise

    def tensor(self, dtype=torch.float32):
        """A 1-D tensor over the whole mapping (borrowed: this object owns the memory)."""
        esz = torch.empty((), dtype=dtype).element_size()
        typestr = {torch.float32: "<f4", torch.bfloat16: "<V2", torch.uint8: "|u1"}[dtype]
        t = torch.as_tensor(_CAI(self.va.value, self.nbytes // esz, typestr), device=self.device)
        return t if t.dtype == dtype else t.view(dtype)

    def release(self):
        hip = _hip()
        if self.va.value:
            hip.hipMemUnmap(self.va, self.nbytes)
            hip.hipMemAddressFree(self.va, self.nbytes)
            self.va = ctypes.c_void_p()
        if self.handle.value:
            hip.hipMemRelease(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            torch.cuda.synchronize(self.device)  # no kernel may still use the mapping
            self.release()
        except Exception:
            pass


class DeviceBuffer:
    """One ordinary device allocation (the caching allocator's, i.e. hipMalloc
    for a fresh block of this size) with PlacedBuffer's interface: the
    candidates the product probes.  Held until the choice, so each candidate is
    distinct memory; `release()` drops it (the caller empties the cache once)."""

    def __init__(self, nbytes, device):
        self.nbytes = -(-int(nbytes) // 16) * 16
        self.device = torch.device(device)
        self._t = torch.empty(self.nbytes, dtype=torch.uint8, device=self.device)

    def tensor(self, dtype=torch.float32):
        return self._t.view(dtype)

    def release(self):
        self._t = None


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


def choose(nbytes, device, probe, baseline_ms, max_candidates, max_frac, kind=DeviceBuffer):
    """Create up to max_candidates - 1 allocations of nbytes one at a time (all
    held until the choice is made, so each is distinct memory; `kind` =
    DeviceBuffer, ordinary allocations -- what the product uses -- or
    PlacedBuffer), time probe(buffer) on each, and return (the fastest buffer, or
    None when none beats baseline_ms -- the caller's own allocation --, every
    time in creation order with the baseline first).  At most max_frac of the
    free device memory is taken; running out ends the search with what was
    probed."""
    times = [baseline_ms]
    best, best_t, held = None, baseline_ms, []
    budget = max_frac * torch.cuda.mem_get_info(torch.device(device))[0]
    try:
        while len(times) < max_candidates and (len(held) + 1) * nbytes <= budget:
            buf = kind(nbytes, device)
            held.append(buf)
            t = probe(buf)
            times.append(t)
            if t < best_t:
                best, best_t = buf, t
    except (RuntimeError, torch.cuda.OutOfMemoryError):
        pass
    for b in held:
        if b is not best:
            b.release()
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
