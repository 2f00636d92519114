"""Tensor-level wrappers of the gfx950 kernels (libgym_amd.so).

Every function takes torch tensors that live on the GPU, checks shapes and
dtypes on the host (so a kernel never runs on operands it was not sized for),
and enqueues the kernel on torch's current stream.  There is no CPU path:
a CPU tensor raises.

Replica sets are 2-D tensors [K, ld]; a 1-D tensor is one replica.  The
SPARTA wrappers also take element-major replica sets (layout="elem"): a 2-D
tensor [n, K] whose row i holds element i of every replica.
"""
import ctypes
import os

import torch

from . import _lib
from ._lib import DemoTensor, check, lib

_DT = {torch.float32: _lib.GA_F32, torch.bfloat16: _lib.GA_BF16}


def _dtype_code(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"gym_amd: unsupported dtype {t.dtype} (float32 / bfloat16)") from None


def _gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("gym_amd kernels run on the MI355X only: got a CPU tensor (there is no CPU fallback)")


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _as2d(t):
    return t if t.dim() == 2 else t.view(1, -1)


def _rows_ld(t2):
    assert t2.dim() == 2
    if t2.shape[0] > 1 and t2.stride(1) != 1:
        raise ValueError("replica set must be row-major contiguous")
    return t2.shape[0], (t2.stride(0) if t2.shape[0] > 1 else t2.shape[1])


def replica_mean(src, dst, n=None, divisor=None, rows=None):
    """dst[j, :n] = (sum_k src[k, :n]) / divisor for every row j of dst
    (divisor defaults to the number of summed replicas; rows = optional int32
    device tensor of replica indices to sum instead of all)."""
    src2, dst2 = _as2d(src), _as2d(dst)
    _gpu(src2, dst2, rows)
    if src2.dtype != dst2.dtype:
        raise TypeError("replica_mean: src/dst dtype mismatch")
    K, lds = _rows_ld(src2)
    Ko, ldd = _rows_ld(dst2)
    n = min(src2.shape[1], dst2.shape[1]) if n is None else int(n)
    if n > src2.shape[1] or n > dst2.shape[1]:
        raise ValueError("replica_mean: n exceeds the row length")
    if rows is not None:
        if rows.dtype != torch.int32:
            raise TypeError("rows must be int32")
        K = rows.numel()
    d = float(K if divisor is None else divisor)
    check(lib().ga_replica_mean(_dtype_code(src2), _p(src2), K, lds, _p(rows), n, d, _p(dst2), Ko, ldd,
                                _stream()), "ga_replica_mean")


def diloco_outer(src, master, mom, dst, n, divisor, lr, momentum, dampening, weight_decay, nesterov,
                 first_step):
    """Fused DiLoCo outer step over [0, n) of master/mom (see include/gym_amd.h)."""
    src2 = _as2d(src)
    dst2 = _as2d(dst) if dst is not None else None
    _gpu(src2, master, mom, dst2)
    K, lds = _rows_ld(src2)
    Ko, ldd = _rows_ld(dst2) if dst2 is not None else (0, 0)
    if master.numel() < n or (mom is not None and mom.numel() < n) or src2.shape[1] < n:
        raise ValueError("diloco_outer: buffers shorter than n")
    if dst2 is not None and dst2.shape[1] < n:
        raise ValueError("diloco_outer: dst shorter than n")
    master_f32 = 1 if master.dtype == torch.float32 else 0
    if master.dtype not in (torch.float32, src2.dtype):
        raise TypeError("diloco_outer: master must be float32 or the arena dtype")
    if mom is not None and mom.dtype != master.dtype:
        raise TypeError("diloco_outer: momentum dtype must match master")
    check(lib().ga_diloco_outer(_dtype_code(src2), _p(src2), K, lds, int(n), float(divisor), _p(master), _p(mom),
                                master_f32, int(bool(first_step)), float(lr), float(momentum), float(dampening),
                                float(weight_decay), int(bool(nesterov)), _p(dst2), Ko, ldd, _stream()),
          "ga_diloco_outer")


def sparta_gap_table(p):
    """The 64-entry gap table of the Philox mask stream (include/gym_amd.h)."""
    import ctypes
    buf = (ctypes.c_uint64 * 64)()
    lib().ga_sparta_gap_table(float(p), buf)
    return [int(v) for v in buf]


def _rate(p, mask):
    if mask is not None:
        return 0.0
    p = float(p)
    if not 0.0 <= p <= 1.0:
        raise ValueError(f"SPARTA selection rate p={p} outside [0, 1]")
    return p


def sparta_mask_words(n):
    """int64 words of a packed SPARTA mask of n elements (ga_sparta_pack_mask)."""
    return (int(n) + 63) // 64


def sparta_pack_mask(mask, n, bits):
    """bits (int64 [>= ceil(n/64)]) <- the uint8/bool mask arena packed one bit
    per element (bit j of word w = element 64 w + j)."""
    _gpu(mask, bits)
    if mask.dtype not in (torch.uint8, torch.bool) or mask.numel() < n or not mask.is_contiguous():
        raise ValueError("sparta_pack_mask: mask must be a contiguous uint8/bool tensor with >= n elements")
    if bits.dtype != torch.int64 or bits.numel() < sparta_mask_words(n) or not bits.is_contiguous():
        raise ValueError("sparta_pack_mask: bits must be a contiguous int64 tensor of >= ceil(n/64) words")
    check(lib().ga_sparta_pack_mask(_p(mask), int(n), _p(bits), _stream()), "ga_sparta_pack_mask")


def sparta_bernoulli_table(offsets, numels, device):
    """(int64 [T, 3] device table, workgroups) for ga_sparta_torch_bernoulli:
    per drawn tensor its arena offset (a multiple of 64: the packed form's
    words never straddle tensors), numel and first workgroup."""
    rows, b = [], 0
    per = int(lib().ga_sparta_torch_bernoulli_span())
    for o, n in zip(offsets, numels):
        if o % 64:
            raise ValueError("sparta_bernoulli_table: arena offsets must be multiples of 64")
        rows.append((int(o), int(n), b))
        b += (int(n) + per - 1) // per
    t = torch.tensor(rows, dtype=torch.int64, device=device).view(-1, 3)
    return t, b


def sparta_torch_bernoulli(table, nblocks, p, seed, offset0, offset_step, mask, seedoff=None):
    """Element e of drawn tensor i <- torch.bernoulli(torch.full(shape_i, p))
    element e as ATen's HIP kernel draws it with generator (seed, offset0 + i *
    offset_step); every drawn tensor in one launch.  mask: the uint8 arena
    (byte at arena offset + e) or int64 packed words (bit arena offset + e).
    seedoff: optional int64 [2] device tensor {seed, offset0} read by the
    kernel instead of the two arguments (rank 0's generator state, broadcast)."""
    _gpu(table, mask, seedoff)
    if seedoff is not None and (seedoff.dtype != torch.int64 or seedoff.numel() < 2):
        raise ValueError("sparta_torch_bernoulli: seedoff must be an int64 [2] tensor")
    if mask.dtype not in (torch.uint8, torch.int64) or not mask.is_contiguous():
        raise ValueError("sparta_torch_bernoulli: mask must be a contiguous uint8 arena or int64 packed words")
    fmt = _lib.GA_MASK_BITS if mask.dtype == torch.int64 else _lib.GA_MASK_BYTES
    if table.dtype != torch.int64 or table.dim() != 2 or table.shape[1] != 3 or not table.is_contiguous():
        raise ValueError("sparta_torch_bernoulli: table must be a contiguous int64 [T, 3] tensor")
    check(lib().ga_sparta_torch_bernoulli(_p(table), int(table.shape[0]), int(nblocks), float(p),
                                          int(seed) & (2**64 - 1), int(offset0), int(offset_step), _p(seedoff),
                                          _p(mask), fmt,
                                          _stream()), "ga_sparta_torch_bernoulli")


class TorchDraw:
    """The reference's mask draw described for the SPARTA kernels to compute
    in-kernel (GA_MASK_TORCH): the table of sparta_bernoulli_table, p, the
    generator state of the first drawn tensor (or a device {seed, offset}
    tensor), the offset step per tensor."""

    def __init__(self, table, p, seed, offset0, offset_step, seedoff=None):
        self.table, self.p, self.seed, self.offset0 = table, float(p), int(seed), int(offset0)
        self.offset_step, self.seedoff = int(offset_step), seedoff

    def struct(self):
        return _lib.TorchDraw(table=_p(self.table), ntens=int(self.table.shape[0]), p=self.p,
                              seed=self.seed & (2**64 - 1), offset0=self.offset0, offset_step=self.offset_step,
                              seedoff=_p(self.seedoff))


def _mask_arg(mask, n, who):
    """(mask, format code) of a SPARTA mask: uint8/bool per element, int64
    packed words (sparta_pack_mask), or a TorchDraw (drawn in-kernel).  For a
    TorchDraw the returned object is the ctypes struct (kept alive by the
    caller for the call)."""
    if mask is None:
        return None, _lib.GA_MASK_BYTES
    if isinstance(mask, TorchDraw):
        _gpu(mask.table, mask.seedoff)
        return mask.struct(), _lib.GA_MASK_TORCH
    if mask.dtype in (torch.uint8, torch.bool):
        if mask.numel() < n:
            raise ValueError(f"{who}: mask must have >= n elements")
        return mask, _lib.GA_MASK_BYTES
    if mask.dtype == torch.int64:
        if mask.numel() < sparta_mask_words(n):
            raise ValueError(f"{who}: packed mask must have >= ceil(n/64) words")
        return mask, _lib.GA_MASK_BITS
    raise ValueError(f"{who}: mask must be uint8/bool (per element) or int64 (packed words)")


def _mptr(mask):
    if isinstance(mask, ctypes.Structure):
        return ctypes.addressof(mask)
    return _p(mask)


def sparta_workspace(n, device):
    nbytes = int(lib().ga_sparta_workspace_bytes(int(n)))
    return torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)  # tile counts + offsets, written per launch


def _sparta_set(t, layout):
    """(K, ld, layout code) of a SPARTA replica set."""
    t2 = _as2d(t)
    if layout == "rows":
        K, ld = _rows_ld(t2)
        return t2, K, ld, _lib.GA_LAYOUT_ROWS
    if layout == "elem":
        if t.dim() != 2 or t.stride(1) != 1:
            raise ValueError("element-major replica set must be a [n, K] tensor with unit replica stride")
        return t, t.shape[1], t.stride(0), _lib.GA_LAYOUT_ELEM_MAJOR
    raise ValueError(f"layout must be 'rows' or 'elem', got {layout!r}")


def _rows_of(t2, code):
    """Elements per replica available in a set."""
    return t2.shape[0] if code == _lib.GA_LAYOUT_ELEM_MAJOR else t2.shape[1]


def _skip_table(skip):
    """skip: None or an int64 device tensor [R, 2] of sorted disjoint [lo, hi)
    element ranges the Philox draw never selects."""
    if skip is None or skip.numel() == 0:
        return None, 0
    if skip.dtype != torch.int64 or skip.dim() != 2 or skip.shape[1] != 2 or not skip.is_contiguous():
        raise ValueError("sparta skip table must be a contiguous int64 [R, 2] tensor")
    return skip, skip.shape[0]


def sparta_select(src, n, cap, idx, vals, count, work, mask=None, seed=0, iteration=0, p=0.0, skip=None,
                  layout="rows"):
    """Compact the selected elements of [0, n) (mask != 0, or the Philox draw
    outside the `skip` ranges) into idx (int32) and vals (= sum over the
    replicas of src); count[0] = number selected, count[1] = overflow flag."""
    _gpu(src, idx, vals, count, work, None if isinstance(mask, TorchDraw) else mask, skip)
    src2, K, ld, code = _sparta_set(src, layout)
    if _rows_of(src2, code) < n:
        raise ValueError("sparta_select: replica set shorter than n")
    skip, nskip = _skip_table(skip)
    if idx.dtype != torch.int32 or count.dtype != torch.int64 or count.numel() < 2:
        raise TypeError("sparta_select: idx int32, count int64[2]")
    if vals.dtype != src2.dtype or idx.numel() < cap or vals.numel() < cap:
        raise ValueError("sparta_select: idx/vals smaller than cap")
    if work.numel() < lib().ga_sparta_workspace_bytes(int(n)):
        raise ValueError("sparta_select: workspace too small")
    mask, mfmt = _mask_arg(mask, n, "sparta_select")
    thr = _rate(p, mask)
    check(lib().ga_sparta_select(_dtype_code(src2), _p(src2), K, ld, code, int(n), _mptr(mask), mfmt,
                                 int(seed) & (2**64 - 1),
                                 int(iteration) & (2**64 - 1), thr, _p(skip), nskip, int(cap), _p(idx), _p(vals),
                                 _p(count),
                                 _p(work), _stream()), "ga_sparta_select")


def sparta_average_local(reps, n, divisor, mask=None, seed=0, iteration=0, p=0.0, idx=None, vals=None, cap=0,
                         count=None, work=None, skip=None, layout="rows"):
    """Single-process SPARTA step over a replica set ([K, ld] rows, or [n, K]
    element-major): selected elements of every replica <- (sum over replicas)
    / divisor, one pass (optional packed idx/vals/count outputs as sparta_select)."""
    _gpu(reps, None if isinstance(mask, TorchDraw) else mask, idx, vals, count, work, skip)
    r2, K, ld, code = _sparta_set(reps, layout)
    if _rows_of(r2, code) < n:
        raise ValueError("sparta_average_local: replica set shorter than n")
    skip, nskip = _skip_table(skip)
    mask, mfmt = _mask_arg(mask, n, "sparta_average_local")
    if idx is not None:
        if idx.dtype != torch.int32 or vals.dtype != r2.dtype or count.dtype != torch.int64:
            raise TypeError("sparta_average_local: idx int32, vals arena dtype, count int64")
        if idx.numel() < cap or vals.numel() < cap or work.numel() < lib().ga_sparta_workspace_bytes(int(n)):
            raise ValueError("sparta_average_local: output buffers too small")
    thr = _rate(p, mask)
    check(lib().ga_sparta_average_local(_dtype_code(r2), _p(r2), K, ld, code, int(n), _mptr(mask), mfmt,
                                        int(seed) & (2**64 - 1),
                                        int(iteration) & (2**64 - 1), thr, _p(skip), nskip, float(divisor),
                                        _p(idx), _p(vals),
                                        int(cap), _p(count), _p(work), _stream()), "ga_sparta_average_local")


def sparta_scatter(vals, idx, count, cap, divisor, dst, layout="rows"):
    _gpu(vals, idx, count, dst)
    dst2, K, ld, code = _sparta_set(dst, layout)
    if vals.dtype != dst2.dtype:
        raise TypeError("sparta_scatter: dtype mismatch")
    check(lib().ga_sparta_scatter(_dtype_code(dst2), _p(vals), _p(idx), _p(count), int(cap), float(divisor),
                                  _p(dst2), K, ld, code, _stream()), "ga_sparta_scatter")


def _demo_dtype(plan, t):
    """The arena dtype code, or GA_BF16_REF for a bf16 arena under a plan with
    the reference's bf16 arithmetic (DemoPlan(bf16_transform="reference"))."""
    if getattr(plan, "bf16_reference", False):
        if t.dtype != torch.bfloat16:
            raise ValueError("DeMo bf16_transform='reference' applies to bf16 arenas only")
        return _lib.GA_BF16_REF
    return _dtype_code(t)


def demo_encode(plan, param, grad, delta, payload, lr, decay, wd_factor):
    """plan: gym_amd.demo_codec.DemoPlan.  param/grad/delta: [K, ld] replica sets
    (or 1-D); payload: int32 [K, 2*M]."""
    p2, g2, d2, pl2 = _as2d(param), _as2d(grad), _as2d(delta), _as2d(payload)
    _gpu(p2, g2, d2, pl2)
    K, ld = _rows_ld(p2)
    if g2.shape != p2.shape or d2.shape != p2.shape or g2.stride() != p2.stride() or d2.stride() != p2.stride():
        raise ValueError("demo_encode: param/grad/delta must be replica sets of one shape")
    if p2.shape[1] < plan.n_arena:
        raise ValueError("demo_encode: arena shorter than the plan")
    if pl2.dtype != torch.int32 or pl2.shape[0] != K or pl2.shape[1] < 2 * plan.M:
        raise ValueError("demo_encode: payload must be int32 [K, >= 2*M]")
    plan.to(p2.device)
    # 64x64 / 1x64 chunks with k <= 64: the wave-per-chunk kernel (GA_DEMO_ENCODE=block forces the other)
    if plan.wave_encode and os.environ.get("GA_DEMO_ENCODE") != "block":
        check(lib().ga_demo_encode_sym(_dtype_code(p2), _p(plan.desc64), plan.n64tensors, plan.n64chunks,
                                       _p(plan.groups), plan.ngroups, _p(plan.F64), _p(p2), _p(g2), _p(d2), K, ld,
                                       float(lr), float(decay), float(wd_factor), _p(pl2), pl2.stride(0), plan.M,
                                       _stream()), "ga_demo_encode_sym")
        return
    check(lib().ga_demo_encode(_demo_dtype(plan, p2), _p(plan.desc), plan.ntensors, plan.nchunks, _p(plan.F), _p(plan.B),
                               _p(p2), _p(g2), _p(d2), K, ld, float(lr), float(decay), float(wd_factor), _p(pl2),
                               pl2.stride(0), plan.M, _stream()), "ga_demo_encode")


DECODE_SYM_MAX_SOURCES = 15


def demo_decode(plan, gathered, param, grad, lr):
    """gathered: int32 [S, >= 2*M] payloads of every node in node order;
    param/grad: [K, ld] replica sets (grad may be None)."""
    p2 = _as2d(param)
    g2 = _as2d(grad) if grad is not None else None
    ga = _as2d(gathered)
    _gpu(p2, g2, ga)
    K, ld = _rows_ld(p2)
    if g2 is not None and (g2.shape != p2.shape or g2.stride() != p2.stride()):
        raise ValueError("demo_decode: grad must match param")
    if ga.dtype != torch.int32 or ga.shape[1] < 2 * plan.M:
        raise ValueError("demo_decode: gathered payload must be int32 [S, >= 2*M]")
    if p2.shape[1] < plan.n_arena:
        raise ValueError("demo_decode: arena shorter than the plan")
    plan.to(p2.device)
    S = ga.shape[0]
    # the wave-per-chunk decode for the same plans as the wave encode and S <= 15
    # sources (4-bit hit counts); GA_DEMO_DECODE=block forces the block kernel
    if plan.wave_encode and S <= DECODE_SYM_MAX_SOURCES and os.environ.get("GA_DEMO_DECODE") != "block":
        check(lib().ga_demo_decode_sym(_dtype_code(p2), _p(plan.desc64), plan.n64tensors, plan.n64chunks,
                                       _p(plan.groups), plan.ngroups, _p(plan.F64), _p(ga), ga.stride(0), plan.M, S,
                                       _p(p2), _p(g2), K, ld, float(lr), _stream()), "ga_demo_decode_sym")
        return
    check(lib().ga_demo_decode(_demo_dtype(plan, p2), _p(plan.desc), plan.ntensors, plan.nchunks, _p(plan.B), _p(ga),
                               ga.stride(0), plan.M, S, _p(p2), _p(g2), K, ld, float(lr), _stream()),
          "ga_demo_decode")


def stream_copy(src, dst):
    """dst <- src as a float4 streaming copy (calibration helper)."""
    _gpu(src, dst)
    nb = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() < nb or not src.is_contiguous() or not dst.is_contiguous():
        raise ValueError("stream_copy: contiguous buffers, dst at least as large as src")
    check(lib().ga_stream_copy(_p(src), _p(dst), nb, _stream()), "ga_stream_copy")


def probe_random_words(reps, pos, M, write=True):
    """The random-word floor of a [K, ld] rows set (calibration helper): the
    fp32 words reps[k, pos[j]] for j < M, read (and written back as x*0.5+1).
    write: 0 read, 1 the word read and written back, 2 / 3 the whole aligned
    64-B sector / 128-B line around it read and written back."""
    _gpu(reps, pos)
    r2 = _as2d(reps)
    if r2.dtype != torch.float32 or pos.dtype != torch.int32 or r2.stride(1) != 1:
        raise ValueError("probe_random_words: fp32 [K, ld] rows, int32 positions")
    check(lib().ga_probe_random_words(_p(r2), r2.stride(0), r2.shape[0], _p(pos), int(M), int(write),
                                      _stream()), "ga_probe_random_words")


def probe_philox(n, sink):
    """The Philox4x32-10 issue ceiling of an n-element reference draw
    (calibration helper): n / 4 calls in the packed draw's launch shape, no
    compare, no store.  sink: a uint32/int32 device tensor of >= 1 element."""
    _gpu(sink)
    check(lib().ga_probe_philox(int(n), _p(sink), _stream()), "ga_probe_philox")


def probe_chunk_stream(a, b, rows, cols, mode):
    """The DeMo codec's 64x64-chunk memory floor (calibration helper): a, b fp32
    buffers of >= rows * cols elements viewed as [rows, cols]; mode 0 = the
    encode's traffic, 1 = the decode's, | 2 = non-temporal (include/gym_amd.h)."""
    _gpu(a, b)
    if a.dtype != torch.float32 or b.dtype != torch.float32 or min(a.numel(), b.numel()) < rows * cols:
        raise ValueError("probe_chunk_stream: fp32 buffers of rows * cols elements")
    check(lib().ga_probe_chunk_stream(_p(a), _p(b), int(rows), int(cols), int(mode), _stream()),
          "ga_probe_chunk_stream")


def probe_diloco_placement(reps, n, master, mom):
    """ga_diloco_outer's access pattern over fp32 replicas [K, ld] (K <= 16) and a
    master / momentum pair, every value written back unchanged (placement probe)."""
    r2 = _as2d(reps)
    _gpu(r2, master, mom)
    K, ld = _rows_ld(r2)
    for t in (r2, master, mom):
        if t.dtype != torch.float32:
            raise ValueError("probe_diloco_placement: fp32 buffers")
    if master.numel() < n or mom.numel() < n:
        raise ValueError("probe_diloco_placement: master/mom shorter than n")
    check(lib().ga_probe_diloco_placement(_p(r2), K, ld, int(n), _p(master), _p(mom), _stream()),
          "ga_probe_diloco_placement")


def probe_mean_placement(reps, n):
    """The in-place ga_replica_mean's access pattern over fp32 replicas [K, ld]
    (K <= 16), every value written back unchanged (placement probe)."""
    r2 = _as2d(reps)
    _gpu(r2)
    K, ld = _rows_ld(r2)
    if r2.dtype != torch.float32:
        raise ValueError("probe_mean_placement: fp32 buffers")
    check(lib().ga_probe_mean_placement(_p(r2), K, ld, int(n), _stream()), "ga_probe_mean_placement")


def probe_adam_placement(param, grad, exp_avg, exp_avg_sq):
    """ga_adam_step's access pattern over fp32 [K, ld] sets of one layout, every
    value written back unchanged (placement probe)."""
    ts = [_as2d(t) for t in (param, grad, exp_avg, exp_avg_sq)]
    _gpu(*ts)
    K, ld = _rows_ld(ts[0])
    for t in ts:
        if t.dtype != torch.float32 or t.shape != ts[0].shape or t.stride() != ts[0].stride() or t.stride(-1) != 1:
            raise ValueError("probe_adam_placement: fp32 replica sets of one layout")
    check(lib().ga_probe_adam_placement(_p(ts[0]), _p(ts[1]), _p(ts[2]), _p(ts[3]), K, ld, ts[0].shape[1],
                                        _stream()), "ga_probe_adam_placement")


def sumsq_partials(device, K=1):
    return torch.empty(int(K) * int(lib().ga_sumsq_partials_count()), dtype=torch.float32, device=device)


def grad_clip_coef(grad, n, max_norm, partials, out):
    """Per replica k of grad ([K, ld] set or 1-D): out[2k] <- min(1, max_norm /
    (||grad_k[:n]||_2 + 1e-6)), out[2k+1] <- the norm (device side)."""
    g2 = _as2d(grad)
    _gpu(g2, partials, out)
    K, ld = _rows_ld(g2)
    if partials.numel() < K * lib().ga_sumsq_partials_count() or out.numel() < 2 * K or out.dtype != torch.float32:
        raise ValueError("grad_clip_coef: partials/out too small")
    check(lib().ga_grad_clip_coef(_dtype_code(g2), _p(g2), K, ld, int(n), float(max_norm), _p(partials), _p(out),
                                  _stream()), "ga_grad_clip_coef")


def adam_step(param, grad, exp_avg, exp_avg_sq, lerp_w, beta2, one_m_beta2, eps, wd_factor, l2_wd, step_size,
              bc2_sqrt, clip_coef=None, n=None):
    """One fused Adam/AdamW step over fp32 [K, ld] replica sets (or 1-D buffers)
    of one shape; every replica's first n elements (see include/gym_amd.h)."""
    ts = [_as2d(t) for t in (param, grad, exp_avg, exp_avg_sq)]
    _gpu(*ts, clip_coef)
    K, ld = _rows_ld(ts[0])
    for t in ts:
        if t.dtype != torch.float32 or t.shape != ts[0].shape or t.stride() != ts[0].stride() or t.stride(-1) != 1:
            raise ValueError("adam_step: param/grad/exp_avg/exp_avg_sq must be fp32 replica sets of one layout")
    n = ts[0].shape[1] if n is None else int(n)
    if clip_coef is not None and clip_coef.numel() < 2 * K:
        raise ValueError("adam_step: clip_coef must hold 2 floats per replica")
    check(lib().ga_adam_step(_GA_F32, _p(ts[0]), _p(ts[1]), _p(ts[2]), _p(ts[3]), K, ld, n, float(lerp_w),
                             float(beta2), float(one_m_beta2), float(eps), float(wd_factor), float(l2_wd),
                             float(step_size), float(bc2_sqrt), _p(clip_coef), _stream()), "ga_adam_step")


_GA_F32 = _lib.GA_F32
