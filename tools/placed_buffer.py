"""PlacedBuffer: one hipMemCreate allocation mapped at a virtual range of its
own, wrapped as a torch tensor via __cuda_array_interface__.  Experiments only
(tools/dbg_placed_alias*.py, tools/exp_*placement.py): NOT part of gym_amd.

Moved out of gym_amd/placement.py in round 5.  On this stack such allocations
were seen corrupted when interleaved with ordinary torch allocations
(profiles/r04u_vmm_alias.txt), so the product's placement candidates are
ordinary device allocations (gym_amd.placement.DeviceBuffer).
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
