"""ctypes binding of libgym_amd.so (the C ABI declared in include/gym_amd.h).

The library is built in-tree (`make`, or `python __graft_entry__.py`), so it
travels with the repository to the GPU box.  There is no fallback: if the
library is missing every operation raises.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# GYM_AMD_LIB: an alternative in-tree build of the same library (kernel variants
# compared by tools/; the ABI must match this file)
LIB_PATH = os.environ.get("GYM_AMD_LIB") or os.path.join(_HERE, "_lib", "libgym_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "gym_amd.h")

GA_F32 = 0
GA_BF16 = 1
GA_BF16_REF = 2  # DeMo entry points: bf16 arenas, the reference's bf16 arithmetic
GA_LAYOUT_ROWS = 0
GA_LAYOUT_ELEM_MAJOR = 1
GA_MASK_BYTES = 0
GA_MASK_BITS = 1
GA_MASK_TORCH = 2

c_i32, c_i64, c_u32, c_u64, c_f32, c_f64 = (ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32,
                                            ctypes.c_uint64, ctypes.c_float, ctypes.c_double)
c_p = ctypes.c_void_p


class TorchDraw(ctypes.Structure):
    """Mirror of `ga_sparta_torch_draw` (include/gym_amd.h)."""
    _fields_ = [("table", c_p), ("ntens", c_i32), ("p", c_f32), ("seed", c_u64), ("offset0", c_u64),
                ("offset_step", c_u64), ("seedoff", c_p)]


class DemoTensor(ctypes.Structure):
    """Mirror of `ga_demo_tensor` (include/gym_amd.h)."""
    _fields_ = [
        ("offset", c_i64), ("payload_off", c_i64),
        ("rows", c_i32), ("cols", c_i32),
        ("n1", c_i32), ("n2", c_i32),
        ("gy", c_i32), ("gx", c_i32),
        ("k", c_i32),
        ("basis1", c_i32), ("basis2", c_i32),
        ("chunk_start", c_i32),
    ]


class DemoRowGroup(ctypes.Structure):
    """Mirror of `ga_demo_rowgroup` (include/gym_amd.h)."""
    _fields_ = [("offset", c_i64), ("payload_off", c_i64), ("rows", c_i32), ("k", c_i32)]


# name -> (restype, argtypes); kept in the order of include/gym_amd.h
SIGNATURES = {
    "ga_abi_version": (c_i32, []),
    "ga_last_error": (ctypes.c_char_p, []),
    "ga_stream_copy": (c_i32, [c_p, c_p, c_i64, c_p]),
    "ga_probe_random_words": (c_i32, [c_p, c_i64, c_i64, c_p, c_i64, c_i32, c_p]),
    "ga_probe_philox": (c_i32, [c_i64, c_p, c_p]),
    "ga_probe_chunk_stream": (c_i32, [c_p, c_p, c_i64, c_i64, c_i32, c_p]),
    "ga_probe_diloco_placement": (c_i32, [c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p]),
    "ga_probe_mean_placement": (c_i32, [c_p, c_i64, c_i64, c_i64, c_p]),
    "ga_probe_adam_placement": (c_i32, [c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p]),
    "ga_replica_mean": (c_i32, [c_i32, c_p, c_i64, c_i64, c_p, c_i64, c_f32, c_p, c_i64, c_i64, c_p]),
    "ga_diloco_outer": (c_i32, [c_i32, c_p, c_i64, c_i64, c_i64, c_f32, c_p, c_p, c_i32, c_i32, c_f32, c_f32,
                                c_f32, c_f32, c_i32, c_p, c_i64, c_i64, c_p]),
    "ga_sparta_workspace_bytes": (c_i64, [c_i64]),
    "ga_sparta_gap_table": (None, [c_f64, c_p]),
    "ga_sparta_pack_mask": (c_i32, [c_p, c_i64, c_p, c_p]),
    "ga_sparta_torch_bernoulli_span": (c_i64, []),
    "ga_sparta_torch_draw_bytes": (c_i32, []),
    "ga_sparta_torch_bernoulli": (c_i32, [c_p, c_i32, c_i64, c_f32, c_u64, c_u64, c_u64, c_p, c_p, c_i32, c_p]),
    "ga_sparta_select": (c_i32, [c_i32, c_p, c_i64, c_i64, c_i32, c_i64, c_p, c_i32, c_u64, c_u64, c_f64, c_p, c_i64,
                                 c_i64, c_p, c_p, c_p, c_p, c_p]),
    "ga_sparta_scatter": (c_i32, [c_i32, c_p, c_p, c_p, c_i64, c_f32, c_p, c_i64, c_i64, c_i32, c_p]),
    "ga_sparta_average_local": (c_i32, [c_i32, c_p, c_i64, c_i64, c_i32, c_i64, c_p, c_i32, c_u64, c_u64, c_f64, c_p,
                                        c_i64, c_f32, c_p, c_p, c_i64, c_p, c_p, c_p]),
    "ga_demo_tensor_bytes": (c_i32, []),
    "ga_demo_encode": (c_i32, [c_i32, c_p, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_f32, c_f32,
                               c_f32, c_p, c_i64, c_i64, c_p]),
    "ga_demo_encode_sym": (c_i32, [c_i32, c_p, c_i32, c_i32, c_p, c_i32, c_p, c_p, c_p, c_p, c_i64, c_i64,
                                   c_f32, c_f32, c_f32, c_p, c_i64, c_i64, c_p]),
    "ga_demo_decode": (c_i32, [c_i32, c_p, c_i32, c_i32, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_i64,
                               c_i64, c_f32, c_p]),
    "ga_demo_decode_sym": (c_i32, [c_i32, c_p, c_i32, c_i32, c_p, c_i32, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p,
                                   c_i64, c_i64, c_f32, c_p]),
    "ga_sumsq_partials_count": (c_i32, []),
    "ga_grad_clip_coef": (c_i32, [c_i32, c_p, c_i64, c_i64, c_i64, c_f32, c_p, c_p, c_p]),
    "ga_adam_step": (c_i32, [c_i32, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_f32, c_f32, c_f32, c_f32, c_f32,
                             c_f32, c_f32, c_f32, c_p, c_p]),
}

_lib = None
_lock = threading.Lock()


class HipLibraryError(RuntimeError):
    pass


def lib():
    """Load (once) and return the library; raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise HipLibraryError(
                    f"{LIB_PATH} is not built: run `make` (or `python __graft_entry__.py`) in the repo root; "
                    "gym_amd has no CPU fallback")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            if L.ga_demo_tensor_bytes() != ctypes.sizeof(DemoTensor):
                raise HipLibraryError("ga_demo_tensor layout mismatch between libgym_amd.so and gym_amd/_lib.py")
            _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().ga_last_error().decode(errors="replace")
        raise HipLibraryError(f"{what} failed (code {rc}): {msg}")


def header_symbols(path=HEADER_PATH):
    """Function names declared with GA_API in the public header."""
    import re
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return re.findall(r"GA_API\s+[\w\s\*]+?\b(ga_\w+)\s*\(", txt)
