"""Host-side plan for the DeMo DCT codec kernels (ga_demo_encode / ga_demo_decode).

Built once per arena layout (the analogue of TransformDCT.__init__,
exogym/strategy/demo_impl/demo.py:214-236): per tensor, the 2-D view and
chunk sizes chosen by `_get_smaller_split` (demo.py:489-498), the per-chunk
entry count k = clamp(topk, 1, n1*n2) (demo.py:307-312), the payload offsets,
and the DCT-II / inverse bases as zero-padded 64x64 fp32 tables.
"""
import ctypes
import math

import numpy as np
import torch

from ._lib import DemoRowGroup, DemoTensor

TILE = 64


def _prime_factors(n):
    f, d = [], 2
    while d * d <= n:
        while n % d == 0:
            f.append(d)
            n //= d
        d += 1
    if n > 1:
        f.append(n)
    return f


def smaller_split(n, target):
    """Chunk size for a dimension of size n (demo.py:489-498): `target` if it
    divides n, else the largest divisor below target; if 1 already exceeds
    target, the smallest divisor; n when every divisor is below target."""
    divs = {1}
    for p in _prime_factors(n):
        divs |= {d * p for d in divs}
    ds = sorted(divs)
    prev = None
    for v in ds:
        if v == target:
            return v
        if v > target:
            return v if prev is None else prev
        prev = v
    return n


def codec_view(shape, chunk):
    """(rows, cols, n1, n2) of the 2-D view the codec uses for a parameter."""
    shape = tuple(int(s) for s in shape)
    if len(shape) == 1:
        return 1, shape[0], 1, smaller_split(shape[0], chunk)
    if len(shape) == 2:
        return shape[0], shape[1], smaller_split(shape[0], chunk), smaller_split(shape[1], chunk)
    if len(shape) == 4:  # conv kernels: full DCT over (h, w) per (out, in) pair (demo.py:256-260)
        b, c, h, w = shape
        if smaller_split(h, chunk) != h or smaller_split(w, chunk) != w:
            raise ValueError(f"DeMo: 4-D parameter {shape} needs its spatial dims to be whole chunks")
        return b * c * h, w, h, w
    raise ValueError(f"DeMo: parameters of rank {len(shape)} are not supported (shape {shape})")


def dct_table(n):
    """F[i, k] = c_k cos(pi (2i+1) k / 2n): the ortho DCT-II basis the reference
    builds as _dct(eye(n), 'ortho') (demo.py:364-395), spatial i, frequency k."""
    i = np.arange(n)[:, None]
    k = np.arange(n)[None, :]
    c = np.where(k == 0, math.sqrt(1.0 / n), math.sqrt(2.0 / n))
    return c * np.cos(math.pi * (2 * i + 1) * k / (2 * n))


BF16_TRANSFORMS = ("fp32", "reference")


class DemoPlan:
    """bf16_transform (bf16 arenas only): "fp32" -- fp32 DCT bases and fp32
    arithmetic on the bf16 values (the product's default, closer to the exact
    transform); "reference" -- the reference's bf16 arithmetic: bases rounded
    to bf16 (demo.py:235-236) and every transform stage rounded to bf16 in the
    reference's contraction order (ga_demo_encode / ga_demo_decode with
    GA_BF16_REF; the block kernels)."""

    def __init__(self, layout, chunk=64, topk=32, bf16_transform="fp32"):
        if bf16_transform not in BF16_TRANSFORMS:
            raise ValueError(f"bf16_transform must be one of {BF16_TRANSFORMS}, got {bf16_transform!r}")
        self.layout = layout
        self.chunk = int(chunk)
        self.topk = int(topk)
        self.bf16_reference = bf16_transform == "reference"
        sizes, descs = [], []
        basis_of = {}
        payload_off = 0
        chunk_start = 0
        self.entries_per_tensor = []
        for shape, off in zip(layout.shapes, layout.offsets):
            R, C, n1, n2 = codec_view(shape, self.chunk)
            if n1 > TILE or n2 > TILE:
                raise NotImplementedError(f"DeMo chunk {n1}x{n2} > {TILE}x{TILE} (compression_chunk <= 64)")
            for n in (n1, n2):
                if n not in basis_of:
                    basis_of[n] = len(sizes)
                    sizes.append(n)
            gy, gx = R // n1, C // n2
            k = max(1, min(self.topk, n1 * n2))
            if k > 512:
                raise NotImplementedError("DeMo: more than 512 entries per chunk (compression_topk <= 512)")
            d = DemoTensor(offset=off, payload_off=payload_off, rows=R, cols=C, n1=n1, n2=n2, gy=gy, gx=gx, k=k,
                           basis1=basis_of[n1], basis2=basis_of[n2], chunk_start=chunk_start)
            descs.append(d)
            self.entries_per_tensor.append(gy * gx * k)
            payload_off += gy * gx * k
            chunk_start += gy * gx
        if chunk_start >= 2**31:
            raise ValueError("DeMo: too many chunks for one launch")
        self.ntensors = len(descs)
        self.nchunks = chunk_start
        # every chunk 64x64 or 1x64 with k <= 64: the wave-per-chunk encode applies
        # (ga_demo_encode_sym: the 64x64 tensors re-numbered, the 1x64 chunks in row groups)
        self.wave_encode = (not self.bf16_reference
                            and all(d.n2 == TILE and d.n1 in (1, TILE) and d.k <= 64 for d in descs))
        self._wave_host = None
        if self.wave_encode:
            d64, groups, start = [], [], 0
            for d in descs:
                if d.n1 == TILE:
                    d64.append(DemoTensor(offset=d.offset, payload_off=d.payload_off, rows=d.rows, cols=d.cols,
                                          n1=d.n1, n2=d.n2, gy=d.gy, gx=d.gx, k=d.k, basis1=d.basis1,
                                          basis2=d.basis2, chunk_start=start))
                    start += d.gy * d.gx
                else:  # 1x64 chunk c of this tensor at offset + 64c (codec_view: C = 64 gx)
                    nch = d.gy * d.gx
                    for c0 in range(0, nch, TILE):
                        groups.append(DemoRowGroup(offset=d.offset + TILE * c0, payload_off=d.payload_off + c0 * d.k,
                                                   rows=min(TILE, nch - c0), k=d.k))
            a64 = (DemoTensor * max(1, len(d64)))(*d64)
            ag = (DemoRowGroup * max(1, len(groups)))(*groups)
            self.n64tensors, self.n64chunks, self.ngroups = len(d64), start, len(groups)
            self._wave_host = (torch.frombuffer(bytearray(bytes(a64)), dtype=torch.uint8),
                               torch.frombuffer(bytearray(bytes(ag)), dtype=torch.uint8))
        self.M = payload_off
        self.n_arena = layout.n
        arr = (DemoTensor * len(descs))(*descs)
        self._desc_host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        F = np.zeros((len(sizes), TILE, TILE), np.float64)
        for j, n in enumerate(sizes):
            F[j, :n, :n] = dct_table(n)
        self._F_host = torch.from_numpy(F.astype(np.float32))
        if self.bf16_reference:  # the reference's bases cast to the parameter dtype (demo.py:235-236)
            self._F_host = self._F_host.to(torch.bfloat16).to(torch.float32)
        # the inverse of an orthonormal basis is its transpose (idct(eye(n)), demo.py:398-442)
        self._B_host = self._F_host.transpose(1, 2).contiguous()
        self.basis_sizes = sizes
        self._F64_host = self._F_host[basis_of[TILE]].contiguous() if TILE in basis_of else None
        self.device = None
        self.desc = self.F = self.B = None
        self.desc64 = self.groups = self.F64 = None

    def to(self, device):
        device = torch.device(device)
        if self.device != device:
            self.desc = self._desc_host.to(device)
            self.F = self._F_host.to(device)
            self.B = self._B_host.to(device)
            if self._wave_host is not None:
                self.desc64, self.groups = (t.to(device) for t in self._wave_host)
                self.F64 = self._F64_host.to(device)
            self.device = device
        return self

    def reference_bytes(self, val_itemsize=4):
        """DeMo.data_transmit of the reference for one step (int64 idx + value)."""
        return self.M * (8 + val_itemsize)
