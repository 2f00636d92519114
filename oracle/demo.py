"""DeMo DCT codec and optimizer step (oracle; test infrastructure only).

Reference: exogym/strategy/demo_impl/demo.py
  _get_prime_divisors/_get_divisors/_get_smaller_split   :445-498
  _dct / _idct (ortho) of eye(n) -> bases F, B           :364-442, built at :227-236
  TransformDCT.encode / decode                           :255-299
  CompressDCT.compress / decompress / batch_decompress   :315-352
  DeMo.step                                              :142-209
Restated in float64.  The DCT-II basis is the closed form
F[i, k] = c_k cos(pi (2i+1) k / 2n), c_0 = sqrt(1/n), c_k = sqrt(2/n) (spatial
index i, frequency k), which the reference's FFT construction equals to within
6e-8 (pinned against the reference's F/B in tests/golden/demo_codec.npz);
B = F^T (orthonormal).
Top-k tie rule (the reference's torch.topk(sorted=False) order is unspecified):
among |coefficients| equal to the k-th largest, the lowest index wins; a
chunk's entries are listed in ascending index order.
"""
import math

import numpy as np


def _prime_divisors(n):
    out = []
    while n % 2 == 0:
        out.append(2)
        n //= 2
    while n % 3 == 0:
        out.append(3)
        n //= 3
    i = 5
    while i * i <= n:
        for k in (i, i + 2):
            while n % k == 0:
                out.append(k)
                n //= k
        i += 6
    if n > 1:
        out.append(n)
    return out


def divisors(n):
    if n < 1:
        return []
    ds = {1}
    for p in _prime_divisors(n):
        ds |= {d * p for d in ds}
    return sorted(ds)


def smaller_split(n, close_to):
    """_get_smaller_split: close_to itself if it divides n, else the largest
    divisor below close_to (the smallest divisor if even 1 exceeds it), n if all
    divisors are below close_to."""
    ds = divisors(n)
    for ix, v in enumerate(ds):
        if v == close_to:
            return v
        if v > close_to:
            return v if ix == 0 else ds[ix - 1]
    return n


def dct_basis(n):
    i = np.arange(n)[:, None]
    k = np.arange(n)[None, :]
    c = np.where(k == 0, math.sqrt(1.0 / n), math.sqrt(2.0 / n))
    return c * np.cos(math.pi * (2 * i + 1) * k / (2 * n))


def idct_basis(n):
    return dct_basis(n).T.copy()


def tensor_view(shape, chunk):
    """(rows, cols, n1, n2) of the 2-D view the codec works on (demo.py:255-276)."""
    shape = tuple(int(s) for s in shape)
    if len(shape) == 1:
        return 1, shape[0], 1, smaller_split(shape[0], chunk)
    if len(shape) == 4:
        b, c, h, w = shape
        n1, n2 = smaller_split(h, chunk), smaller_split(w, chunk)
        if n1 != h or n2 != w:
            raise ValueError(f"DeMo 4-D tensor {shape}: chunked spatial dims are unsupported by the reference")
        return b * c * h, w, h, w
    if len(shape) == 2:
        r, c = shape
        return r, c, smaller_split(r, chunk), smaller_split(c, chunk)
    raise ValueError(f"DeMo: unsupported parameter rank {len(shape)} (shape {shape})")


def encode(x, shape, chunk):
    """Y[gy, gx, n1, n2] = F1^T X_chunk F2 for every chunk (float64)."""
    R, C, n1, n2 = tensor_view(shape, chunk)
    X = np.asarray(x, dtype=np.float64).reshape(R // n1, n1, C // n2, n2)
    F1, F2 = dct_basis(n1), dct_basis(n2)
    return np.einsum("yhxw,hb,wd->yxbd", X, F1, F2)


def decode(Y, shape, chunk):
    """Inverse of encode: X_chunk = B1^T Y B2, reassembled to `shape`."""
    R, C, n1, n2 = tensor_view(shape, chunk)
    B1, B2 = idct_basis(n1), idct_basis(n2)
    X = np.einsum("yxkl,kb,ld->ybxd", np.asarray(Y, dtype=np.float64), B1, B2)
    return X.reshape(shape)


def topk_chunks(Y, k):
    """Per chunk: indices (ascending) and values of the k largest |y| over the
    flattened n1*n2 coefficients; ties at the boundary -> lowest index."""
    gy, gx, n1, n2 = Y.shape
    flat = Y.reshape(gy * gx, n1 * n2)
    k = max(1, min(k, n1 * n2))
    order = np.argsort(-np.abs(flat), axis=1, kind="stable")[:, :k]
    idx = np.sort(order, axis=1)
    val = np.take_along_axis(flat, idx, axis=1)
    return idx.reshape(gy, gx, k), val.reshape(gy, gx, k)


def kth_margin(Y, k):
    """Per chunk: |y|_(k) - |y|_(k+1) (sorted descending); 0 means a boundary tie."""
    gy, gx, n1, n2 = Y.shape
    a = -np.sort(-np.abs(Y.reshape(gy * gx, n1 * n2)), axis=1)
    k = max(1, min(k, n1 * n2))
    if k == n1 * n2:
        return np.full(gy * gx, np.inf)
    return a[:, k - 1] - a[:, k]


def scatter_mean(idx_list, val_list, n1, n2):
    """batch_decompress + decompress: concatenate the K lists on the last dim,
    then each coefficient = mean of the entries that hit it, 0 where none did."""
    idx = np.concatenate([np.asarray(i) for i in idx_list], axis=-1)
    val = np.concatenate([np.asarray(v, dtype=np.float64) for v in val_list], axis=-1)
    gy, gx, m = idx.shape
    s = np.zeros((gy * gx, n1 * n2))
    c = np.zeros((gy * gx, n1 * n2))
    rows = np.repeat(np.arange(gy * gx), m)
    np.add.at(s, (rows, idx.reshape(-1)), val.reshape(-1))
    np.add.at(c, (rows, idx.reshape(-1)), 1.0)
    out = np.where(c > 0, s / np.maximum(c, 1.0), 0.0)
    return out.reshape(gy, gx, n1, n2)


def entries(shape, chunk, topk):
    R, C, n1, n2 = tensor_view(shape, chunk)
    return (R // n1) * (C // n2) * max(1, min(topk, n1 * n2))


def demo_step(p, deltas, grads, lr, decay=0.999, topk=32, chunk=64, weight_decay=0.0, detail=False):
    """One DeMo.step for one tensor over K nodes (params identical across nodes).
    Returns (p_new, [delta_new_k], sign_grad, [(idx_k, val_k)]); with
    detail=True also (decoded_grad, [(per-chunk k-th margin, max |coefficient|)
    of node k]) -- the
    value whose sign is applied and how far each node's top-k set is from a
    tie (test infrastructure decides where a sign is unambiguous from these)."""
    shape = np.shape(p)
    p64 = np.asarray(p, dtype=np.float64)
    if weight_decay != 0.0:
        p64 = p64 * np.float64(np.float32(1.0 - lr * weight_decay))
    R, C, n1, n2 = tensor_view(shape, chunk)
    new_deltas, sent, margins = [], [], []
    for d, g in zip(deltas, grads):
        d64 = np.asarray(d, dtype=np.float64)
        if decay != 1:
            d64 = d64 * decay
        d64 = d64 + lr * np.asarray(g, dtype=np.float64)
        Y = encode(d64, shape, chunk)
        idx, val = topk_chunks(Y, topk)
        if detail:
            margins.append((kth_margin(Y, topk), np.abs(Y).max()))
        tx = decode(scatter_mean([idx], [val], n1, n2), shape, chunk)
        new_deltas.append(d64 - tx)
        sent.append((idx, val))
    S = scatter_mean([s[0] for s in sent], [s[1] for s in sent], n1, n2)
    g = decode(S, shape, chunk)
    sgn = np.sign(g)
    if detail:
        return p64 - lr * sgn, new_deltas, sgn, sent, g, margins
    return p64 - lr * sgn, new_deltas, sgn, sent


def transmit_bytes(shapes, chunk, topk, val_itemsize=4):
    """DeMo.data_transmit (demo.py:188): int64 idx + p.dtype val per entry."""
    return sum(entries(s, chunk, topk) * (8 + val_itemsize) for s in shapes)
