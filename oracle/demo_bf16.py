"""The reference DeMo step's bf16 arithmetic as torch runs it on the CPU
(oracle; test infrastructure only; pinned to tests/golden/demo_steps_bf16.npz,
the reference's own bf16 run, by tests/test_oracle_golden.py).

Reference: exogym/strategy/demo_impl/demo.py
  bases cast to the parameter dtype                 :235-236
  TransformDCT.encode / decode (einsum, 2 stages)   :255-299 (einsum_2d :238-244, einsum_2d_t :246-252)
  CompressDCT.compress / decompress / batch_decompress :315-352
  DeMo.step                                         :142-209
What bf16 changes against the fp32/fp64 restatement in oracle/demo.py:
  - the DCT bases are rounded to bf16;
  - every einsum contracts left to right (torch without opt_einsum) and each
    of its two stages rounds to bf16: encode Y = bf16(bf16(F1^T X) F2),
    decode R = bf16(bf16(B1^T S) B2) (stage 1 contracts the chunk rows);
  - delta.mul_(decay) and delta.add_(grad, alpha=lr) round separately, and
    torch's CPU add_ rounds alpha (lr) to bf16 first (on the GPU it stays
    fp32); the same for the SGD step p.add_(sign, alpha=-lr);
  - the top-k runs on the bf16 coefficients with torch.topk's CPU tie order
    (not the product's lowest-index rule).
This module runs those torch ops on CPU tensors in the reference's order;
it does not import the reference.  The product's GA_BF16_REF kernels restate
the same sequence on the MFMA (fp32 accumulation, bf16 rounding per stage).
"""
import numpy as np
import torch

from .demo import dct_basis, idct_basis, smaller_split, tensor_view


def _bases(n, dtype, device="cpu"):
    return (torch.from_numpy(dct_basis(n)).to(torch.float32).to(dtype).to(device),
            torch.from_numpy(idct_basis(n)).to(torch.float32).to(dtype).to(device))


def _chunks(x, shape, chunk):
    """[gy, n1, gx, n2] chunk view of the 2-D view (rows, cols) of a tensor."""
    rows, cols, n1, n2 = tensor_view(shape, chunk)
    return x.reshape(rows // n1, n1, cols // n2, n2), n1, n2


def encode(x, shape, chunk, dtype):
    """Y[gy, gx, b, d] = bf16(bf16(sum_j F1[j, b] X[j, l]) . F2[l, d]) -- one
    three-operand einsum, contracted left to right as torch does without
    opt_einsum (the rows first); a 1-D tensor: one stage over its chunks."""
    if len(shape) == 1:
        n = smaller_split(shape[0], chunk)
        F, _ = _bases(n, dtype, x.device)
        return torch.einsum("xl,ld->xd", x.reshape(-1, n), F).reshape(1, -1, 1, n)
    xc, n1, n2 = _chunks(x, shape, chunk)
    F1, _ = _bases(n1, dtype, x.device)
    F2, _ = _bases(n2, dtype, x.device)
    return torch.einsum("yjxl,jb,ld->yxbd", xc, F1, F2)


def decode(y, shape, chunk, dtype):
    """The inverse: X[(gy n1), (gx n2)] = bf16(bf16(B1-contraction of the
    coefficient rows) . B2), left to right; 1-D: one stage."""
    rows, cols, n1, n2 = tensor_view(shape, chunk)
    if len(shape) == 1:
        _, B = _bases(n2, dtype, y.device)
        return torch.einsum("xl,ld->xd", y.reshape(-1, n2), B).reshape(rows, cols)
    _, B1 = _bases(n1, dtype, y.device)
    _, B2 = _bases(n2, dtype, y.device)
    return torch.einsum("yxkl,kb,ld->ybxd", y, B1, B2).reshape(rows, cols)


def topk(y, k):
    flat = y.reshape(*y.shape[:2], -1)
    k = max(1, min(k, flat.shape[-1]))
    idx = torch.topk(flat.abs(), k=k, dim=-1, largest=True, sorted=False).indices
    return idx, torch.gather(flat, -1, idx)


def scatter_mean(like, idx_list, val_list):
    flat = torch.zeros_like(like).reshape(*like.shape[:2], -1)
    idx = torch.cat(idx_list, dim=-1)
    val = torch.cat(val_list, dim=-1)
    flat.scatter_reduce_(-1, idx, val, reduce="mean", include_self=False)
    return flat.reshape(like.shape)


def demo_step(p, deltas, grads, lr, decay, topk_k, chunk, wd=0.0, dtype=torch.bfloat16, device="cpu"):
    """One reference DeMo step of one tensor over K nodes (node order) in
    `dtype`, with torch's ops on `device` (the CPU: the reference's golden run;
    a GPU: the same ops as torch runs them there -- fp32 alpha, its topk tie
    order).  p: the shared parameter (numpy), deltas / grads: per node (numpy).
    Returns (p after, per-node deltas after, sign) as fp32 numpy."""
    shape = p.shape
    P = torch.from_numpy(np.asarray(p, np.float32)).to(dtype).to(device)
    if wd != 0.0:
        P.mul_(1.0 - lr * wd)
    idxs, vals, Ds, Y0 = [], [], [], None
    for d, g in zip(deltas, grads):
        D = torch.from_numpy(np.asarray(d, np.float32)).to(dtype).to(device)
        G = torch.from_numpy(np.asarray(g, np.float32)).to(dtype).to(device)
        if decay != 1:
            D.mul_(decay)
        D.add_(G, alpha=lr)
        Y = encode(D.reshape(-1) if len(shape) == 1 else D, shape, chunk, dtype)
        i, v = topk(Y, topk_k)
        S = scatter_mean(Y, [i], [v])
        D.sub_(decode(S, shape, chunk, dtype).reshape(D.shape))
        idxs.append(i)
        vals.append(v)
        Ds.append(D)
        Y0 = Y
    g_new = decode(scatter_mean(Y0, idxs, vals), shape, chunk, dtype).reshape(shape)
    sign = g_new.sign()
    P.add_(sign, alpha=-lr)
    f = lambda t: t.float().cpu().numpy()  # noqa: E731
    return f(P), [f(D) for D in Ds], f(sign)
