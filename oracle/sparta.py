"""SPARTA sparse averaging and the selector masks (oracle; test infrastructure only).

Reference: SparseCommunicator.communicate (exogym/strategy/sparta.py:24-44):
  mask = rank 0's index_selector.get_indices(param, iteration)   (:32-37, broadcast)
  v = param.data[mask]            row-major order over the tensor (:38)
  v = (sum_k v_k) / num_nodes     all_reduce SUM then true division (:39-40)
  param.masked_scatter_(mask, v)  (:42)
  tensors with `not requires_grad or grad is None` are skipped (:29-30).
Selectors restated given their torch random draws as inputs:
  RandomIndexSelector (:80-85), ShuffledSequentialIndexSelector (:88-136),
  PartitionedIndexSelector (:139-193).

gym_amd's fast mask mode has no reference counterpart: it draws the mask from
Philox4x32-10 (Salmon et al., SC'11, "Parallel random numbers: as easy as
1, 2, 3"; constants as in Random123) keyed by (seed, iteration), as the
geometric gaps between selected elements of each 64-element group (one
Bernoulli(p) draw per element in distribution; `philox_mask`).
`philox4x32_10` restates that generator; it is pinned by the Random123
known-answer vectors in tests/test_oracle_golden.py.
`torch_gpu_bernoulli` restates the reference draw as torch runs it on a GPU
(ATen's HIP bernoulli kernel over rocrand Philox4x32-10; third-party code, no
reference source), pinned on the GPU box against torch.bernoulli itself.
"""
import math

import numpy as np

from .reduce import mean_reduce

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr, key):
    """ctr: uint32 array [..., 4]; key: uint32 array [..., 2] (broadcastable)."""
    c = [np.asarray(ctr[..., i], dtype=np.uint32) for i in range(4)]
    k0 = np.asarray(key[..., 0], dtype=np.uint32)
    k1 = np.asarray(key[..., 1], dtype=np.uint32)
    with np.errstate(over="ignore"):
        return _philox_rounds(c, k0, k1)


def _philox_rounds(c, k0, k1):
    for _ in range(10):
        p0 = c[0].astype(np.uint64) * M0
        p1 = c[2].astype(np.uint64) * M1
        hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & MASK32).astype(np.uint32)
        hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & MASK32).astype(np.uint32)
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
        k0 = (k0 + W0).astype(np.uint32)
        k1 = (k1 + W1).astype(np.uint32)
    return np.stack(c, axis=-1)


GAP_TABLE = 64


def gap_table(p):
    """T[j] = round(2^32 (1 - (1 - p)^(j+1))) for j < 64 (include/gym_amd.h,
    ga_sparta_gap_table): a 32-bit word u gives the gap #{j : T[j] <= u}."""
    out = []
    for j in range(GAP_TABLE):
        if not p > 0.0:
            v = 0.0
        elif p >= 1.0:
            v = 4294967296.0
        else:
            v = math.floor(-math.expm1((j + 1) * math.log1p(-p)) * 4294967296.0 + 0.5)
        out.append(int(min(v, 4294967296.0)))
    return np.array(out, dtype=np.uint64)


def philox_mask(n, seed, iteration, p, start=0, skip=None):
    """Mask bits of arena elements [start, start+n) for (seed, iteration):
    i.i.d. Bernoulli(p) as geometric gaps -- group g = 64 elements reads the
    words of philox(key=seed, ctr={g, r, iteration}), r = 0, 1, ..., in order;
    u >= T[63] ends the group, else pos += #{j : T[j] <= u}, element 64g+pos is
    selected (pos < 64), pos += 1.  Elements inside a `skip` range [lo, hi)
    are never selected (tensors without a gradient, which
    SparseCommunicator.communicate skips, exogym/strategy/sparta.py:29-30)."""
    if n <= 0:
        return np.zeros(0, dtype=bool)
    tab = gap_table(p)
    g0, g1 = start // 64, (start + n - 1) // 64 + 1
    G = g1 - g0
    groups = np.arange(g0, g1, dtype=np.uint64)
    bits = np.zeros((G, 64), dtype=bool)
    pos = np.zeros(G, dtype=np.int64)
    live = np.ones(G, dtype=bool)
    key = np.array([seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF], dtype=np.uint32)
    r = 0
    while live.any():
        act = np.flatnonzero(live)
        ctr = np.stack([(groups[act] & MASK32).astype(np.uint32), np.full(act.size, r, np.uint32),
                        np.full(act.size, iteration & 0xFFFFFFFF, np.uint32),
                        np.full(act.size, (iteration >> 32) & 0xFFFFFFFF, np.uint32)], axis=-1)
        words = philox4x32_10(ctr, key)
        for j in range(4):
            lv = live[act]
            u = words[:, j].astype(np.uint64)
            end = lv & (u >= tab[GAP_TABLE - 1])
            live[act[end]] = False
            go = lv & ~end
            a = act[go]
            gap = np.searchsorted(tab, u[go], side="right")  # #{j : T[j] <= u}
            pos[a] += gap
            sel = pos[a] < 64
            bits[a[sel], pos[a[sel]]] = True
            pos[a] += 1
            live[a[pos[a] >= 64]] = False
        r += 1
    m = bits.reshape(-1)[start - 64 * g0: start - 64 * g0 + n].copy()
    for lo, hi in (skip if skip is not None else ()):
        a, b = max(int(lo) - start, 0), min(int(hi) - start, n)
        if a < b:
            m[a:b] = False
    return m


def sparse_average(node_params, mask, divisor=None):
    """node_params: list of K arrays of one tensor; mask: bool array of the same
    shape.  Returns the K updated arrays (sparta.py:38-42)."""
    flat_mask = np.asarray(mask, dtype=bool).reshape(-1)
    vals = [np.asarray(p, dtype=np.float32).reshape(-1)[flat_mask] for p in node_params]
    avg = mean_reduce(vals, divisor if divisor is not None else len(node_params))
    out = []
    for p in node_params:
        q = np.asarray(p, dtype=np.float32).reshape(-1).copy()
        q[flat_mask] = avg
        out.append(q.reshape(np.shape(p)))
    return out


def selected_indices(mask):
    """param.data[mask] order: ascending flat index."""
    return np.flatnonzero(np.asarray(mask).reshape(-1))


def shuffled_sequential_mask(numel, p, shuffled_indices, iteration):
    """ShuffledSequentialIndexSelector.get_indices (sparta.py:95-136) given the
    tensor's randperm drawn on first use."""
    if numel == 0:
        return np.zeros(0, dtype=bool)
    num_partitions = max(1, math.ceil(1.0 / p))
    chunk = iteration % num_partitions
    size, rem = divmod(numel, num_partitions)
    start = chunk * size + min(chunk, rem)
    end = start + size + (1 if chunk < rem else 0)
    m = np.zeros(numel, dtype=bool)
    m[np.asarray(shuffled_indices)[start:end]] = True
    return m


def partitioned_masks(numel, p, rank_orders, calls):
    """PartitionedIndexSelector.get_indices (sparta.py:146-193) for `calls`
    consecutive calls on one tensor, given the orders torch.rand(numel).argsort()
    produced at each (re)partition (rank_orders[j] for the j-th; argsort's order
    among tied draws is torch's, so it is an input here, like the randperm of
    the shuffled selector)."""
    nparts = max(1, min(math.ceil(1.0 / p), numel))
    out, cur, draw = [], None, 0
    parts = None
    for _ in range(calls):
        if parts is None or cur >= nparts:
            parts = np.asarray(rank_orders[draw]) % nparts
            draw += 1
            cur = 0
        out.append(parts == cur)
        cur += 1
    return out


def pack_mask(mask):
    """The wire form of a mask arena (gym_amd's ga_sparta_pack_mask, no
    reference counterpart): bit j of int64 word w = (mask[64 w + j] != 0),
    ceil(n/64) words, bits past n zero."""
    m = np.asarray(mask).reshape(-1) != 0
    words = -(-m.size // 64)
    pad = np.zeros(words * 64, dtype=bool)
    pad[:m.size] = m
    return np.packbits(pad.reshape(words, 64), axis=1, bitorder="little").reshape(-1).view("<i8").copy()


def unpack_mask(words, n):
    """Inverse of pack_mask: the n-element bool mask."""
    b = np.unpackbits(np.asarray(words, dtype="<i8").view(np.uint8), bitorder="little")
    return b[:n].astype(bool)


def torch_gpu_bernoulli(numel, p, seed, offset):
    """torch.bernoulli(torch.full((numel,), p, device=cuda)) as ATen's HIP
    kernel draws it (bernoulli_tensor_cuda_kernel via CUDA_tensor_apply2<.., 4>,
    hiprand/rocrand Philox4x32-10): thread t = element // 4 initialises the
    generator with (seed, subsequence t, offset) -- counter {offset/4, t}, key
    seed -- and element 4t + j is selected iff float32(w_j) * 2^-32 + 2^-32 <=
    float32(p) (float32 arithmetic), w_j the j-th word of its first Philox call.
    Third-party restatement (torch 2.10 / ROCm rocrand, no reference source):
    pinned by tests/test_gpu_kernels.py against torch.bernoulli on the GPU."""
    assert offset % 4 == 0
    T = -(-int(numel) // 4)
    t = np.arange(T, dtype=np.uint64)
    q = np.uint64(offset // 4)
    ctr = np.stack([np.full(T, q & MASK32), np.full(T, q >> np.uint64(32)), t & MASK32, t >> np.uint64(32)],
                   axis=-1).astype(np.uint32)
    key = np.array([seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF], dtype=np.uint32)
    w = philox4x32_10(ctr, key).reshape(-1)[:numel]
    inv = np.float32(2.0 ** -32)
    u = w.astype(np.float32) * inv + inv
    return u <= np.float32(p)
