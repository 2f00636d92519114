"""Parity of the gfx950 kernels (through the C ABI) against the oracle and the
reference's golden fixtures.  Bars: integer/index work bit-exact; fp32 sums
in the same order bit-exact; reordered fp32 within 1e-6 relative; bf16 1e-2.
"""
import numpy as np
import pytest
import torch

from oracle import demo as odemo
from oracle import diloco as odiloco
from oracle import reduce as oreduce
from oracle import sparta as osparta
import demo_checks

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gym_amd import _lib
    _lib.lib()


def t(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a)).to(DEV, dtype)


def host(x):
    torch.cuda.synchronize()
    return x.float().cpu().numpy()


# ---------------------------------------------------------------- mean --------
@pytest.mark.parametrize("K", [1, 2, 3, 8, 32])
@pytest.mark.parametrize("n", [4096, 1000, 12345, 1])
def test_replica_mean_bit_exact(K, n):
    from gym_amd import ops
    rng = np.random.default_rng(K * 1000 + n)
    ld = ((n + 63) // 64) * 64
    x = rng.standard_normal((K, ld)).astype(np.float32)
    src = t(x)
    dst = torch.full((1, ld), 7.0, device=DEV)
    ops.replica_mean(src, dst, n=n)
    want = oreduce.mean_reduce(list(x[:, :n]))
    got = host(dst)[0]
    assert np.array_equal(got[:n], want)
    assert (got[n:] == 7.0).all()  # nothing past n is written


def test_replica_mean_in_place_all_replicas_and_rows():
    from gym_amd import ops
    rng = np.random.default_rng(3)
    x = rng.standard_normal((5, 4160)).astype(np.float32)
    src = t(x)
    ops.replica_mean(src, src, n=4160)  # in place, every replica gets the mean
    want = oreduce.mean_reduce(list(x))
    got = host(src)
    assert all(np.array_equal(got[k], want) for k in range(5))
    # island subset (FedAvg islands), ascending member order
    src = t(x)
    rows = torch.tensor([1, 3, 4], dtype=torch.int32, device=DEV)
    out = torch.empty(2, 4160, device=DEV)
    ops.replica_mean(src, out, n=4160, rows=rows)
    want = oreduce.mean_reduce(list(x), rows=[1, 3, 4])
    assert np.array_equal(host(out)[0], want) and np.array_equal(host(out)[1], want)


def test_replica_mean_sum_and_divisor():
    from gym_amd import ops
    x = np.random.default_rng(1).standard_normal((3, 640)).astype(np.float32)
    out = torch.empty(640, device=DEV)
    ops.replica_mean(t(x), out, divisor=1.0)
    s = oreduce.mean_reduce(list(x), divisor=1)
    assert np.array_equal(host(out), s)
    ops.replica_mean(out, out, divisor=6.0)  # cross-GPU style: global divide after a sum
    assert np.array_equal(host(out), (s / np.float32(6)).astype(np.float32))


def test_replica_mean_bf16():
    from gym_amd import ops
    x = np.random.default_rng(2).standard_normal((4, 1024)).astype(np.float32)
    src = t(x, torch.bfloat16)
    out = torch.empty(1024, device=DEV, dtype=torch.bfloat16)
    ops.replica_mean(src, out)
    want = oreduce.mean_reduce(list(src.float().cpu().numpy()))
    np.testing.assert_allclose(host(out), want, rtol=1e-2, atol=1e-2)


def test_replica_mean_matches_reference_golden(golden):
    from gym_amd import ops
    z = golden("mean_reduce.npz")
    for K in (2, 3, 8):
        for si in range(4):
            xs = z[f"K{K}_in_{si}"].reshape(K, -1)
            ref = z[f"K{K}_out_{si}"].reshape(-1)
            out = torch.empty(xs.shape[1], device=DEV)
            ops.replica_mean(t(xs), out)
            got = host(out)
            if K == 2:
                assert np.array_equal(got, ref)
            else:
                np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-7)


# ---------------------------------------------------------------- DiLoCo ------
@pytest.mark.parametrize("K,first,nesterov", [(1, True, True), (3, True, True), (3, False, True),
                                             (8, False, False), (4, False, True)])
def test_diloco_outer_matches_oracle(K, first, nesterov):
    from gym_amd import ops
    rng = np.random.default_rng(K + 10 * first)
    n = 50_000
    master = (rng.standard_normal(n) * 0.02).astype(np.float32)
    reps = (master + rng.standard_normal((K, n)) * 1e-3).astype(np.float32)
    mom = None if first else (rng.standard_normal(n) * 1e-3).astype(np.float32)
    want_m, want_b, _ = odiloco.outer_step(master, mom, list(reps), lr=0.7, momentum=0.9, nesterov=nesterov)
    g_master, g_mom = t(master), t(mom if mom is not None else np.zeros(n, np.float32))
    src = t(reps)
    dst = torch.empty(K, n, device=DEV)
    ops.diloco_outer(src, g_master, g_mom, dst, n, K, 0.7, 0.9, 0.0, 0.0, nesterov, first)
    gm, gb, gd = host(g_master), host(g_mom), host(dst)
    np.testing.assert_allclose(gm, want_m, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(gb, want_b, rtol=0, atol=1e-6 * np.abs(master).max())
    assert all(np.array_equal(gd[k], gm) for k in range(K))
    # same op order as torch's SGD: all but a handful of elements bit-identical
    assert (gm == want_m).mean() > 0.999


@pytest.mark.parametrize("dampening,wd,nesterov", [(0.1, 0.0, False), (0.0, 1e-3, True), (0.2, 1e-3, False)])
def test_diloco_outer_dampening_weight_decay_vs_torch_sgd(dampening, wd, nesterov):
    """The outer step with the SGD options a user's outer OptimSpec may set
    (dampening, weight_decay; diloco.py:26-28 builds any torch.optim.SGD) against
    torch.optim.SGD itself (fp32, single-tensor) over three outer steps: master,
    momentum and every replica."""
    from gym_amd import ops
    K, n = 3, 40_000
    g = torch.Generator().manual_seed(int(100 * dampening + 1e4 * wd) + nesterov)
    master0 = torch.randn(n, generator=g) * 0.02
    ref = torch.nn.Parameter(master0.clone())
    opt = torch.optim.SGD([ref], lr=0.7, momentum=0.9, dampening=dampening, weight_decay=wd, nesterov=nesterov,
                          foreach=False)
    g_master, g_mom = master0.clone().to(DEV), torch.zeros(n, device=DEV)
    for step in range(3):
        reps = (ref.detach() + torch.randn(K, n, generator=g) * 1e-3).float()
        avg = reps.sum(0) / K
        ref.grad = ref.detach() - avg
        opt.step()
        dst = torch.empty(K, n, device=DEV)
        ops.diloco_outer(reps.to(DEV), g_master, g_mom, dst, n, K, 0.7, 0.9, dampening, wd, nesterov, step == 0)
        want_m, want_b = ref.detach().numpy(), opt.state[ref]["momentum_buffer"].numpy()
        gm, gb = host(g_master), host(g_mom)
        np.testing.assert_allclose(gm, want_m, rtol=1e-6, atol=1e-8)
        np.testing.assert_allclose(gb, want_b, rtol=1e-5, atol=1e-9)
        assert all(np.array_equal(d, gm) for d in host(dst))
        g_master.copy_(t(want_m))  # continue from torch's state (the fp32 sum order of avg may differ by an ulp)
        g_mom.copy_(t(want_b))


def test_diloco_matches_reference_golden_chain(golden):
    """Three outer steps of the reference's DiLoCoStrategy (K=3, H=2), replayed
    on the GPU with the K nodes as replicas."""
    from gym_amd import ops
    from gym_amd.arena import ArenaLayout
    z = golden("diloco.npz")
    K, H, calls, ns = int(z["K"]), int(z["H"]), int(z["calls"]), int(z["nshapes"])
    shapes = [z[f"init_{i}"].shape for i in range(ns)]
    L = ArenaLayout(shapes)
    master = torch.zeros(L.n, device=DEV)
    mom = torch.zeros(L.n, device=DEV)
    for i, v in enumerate(L.views(master)):
        v.copy_(t(z[f"init_{i}"]))
    reps = torch.zeros(K, L.n, device=DEV)
    first = True
    for call in range(calls):
        if not odiloco.is_outer_step(call, H):
            continue
        for k in range(K):
            for i, v in enumerate(L.views(reps[k])):
                v.copy_(t(z[f"before_{call}_{i}"][k]))
        ops.diloco_outer(reps, master, mom, reps, L.n, K, 0.7, 0.9, 0.0, 0.0, True, first)
        first = False
        for i in range(ns):
            ref_m = z[f"master_{call}_{i}"]
            np.testing.assert_allclose(host(L.views(master)[i]), ref_m, rtol=1e-6, atol=1e-8)
            for k in range(K):
                np.testing.assert_allclose(host(L.views(reps[k])[i]), z[f"after_{call}_{i}"][k], rtol=1e-6,
                                           atol=1e-8)
        # continue from the reference's own state (as the oracle test does)
        for i, v in enumerate(L.views(master)):
            v.copy_(t(z[f"master_{call}_{i}"]))
        for i, v in enumerate(L.views(mom)):
            v.copy_(t(z[f"mom_{call}_{i}"]))


def test_diloco_bf16_params_fp32_master():
    from gym_amd import ops
    rng = np.random.default_rng(9)
    n, K = 8192, 4
    master = (rng.standard_normal(n) * 0.02).astype(np.float32)
    reps = (master + rng.standard_normal((K, n)) * 1e-2).astype(np.float32)
    src = t(reps, torch.bfloat16)
    want_m, _, _ = odiloco.outer_step(master, None, list(src.float().cpu().numpy()))
    gm, gb = t(master), torch.zeros(n, device=DEV)
    ops.diloco_outer(src, gm, gb, src, n, K, 0.7, 0.9, 0.0, 0.0, True, True)
    np.testing.assert_allclose(host(gm), want_m, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(host(src)[0], want_m, rtol=1e-2, atol=1e-3)


# ---------------------------------------------------------------- SPARTA ------
def _sparta_buffers(n, cap):
    from gym_amd import ops
    return (torch.empty(cap, dtype=torch.int32, device=DEV), torch.zeros(2, dtype=torch.int64, device=DEV),
            ops.sparta_workspace(n, DEV))


@pytest.mark.parametrize("n,p,K", [(1_000_003, 0.005, 1), (65_536, 0.3, 3), (4095, 0.5, 2), (5, 0.9, 1)])
def test_sparta_philox_select_gather_scatter(n, p, K):
    from gym_amd import ops
    rng = np.random.default_rng(n)
    x = rng.standard_normal((K, n)).astype(np.float32)
    seed, it = 0x1234_5678_9ABC, 17
    mask = osparta.philox_mask(n, seed, it, p)
    want_idx = np.flatnonzero(mask)
    cap = len(want_idx) + 64
    idx, count, work = _sparta_buffers(n, cap)
    vals = torch.empty(cap, device=DEV)
    src = t(x)
    ops.sparta_select(src, n, cap, idx, vals, count, work, seed=seed, iteration=it, p=p)
    c = host(count).astype(np.int64)
    assert c[0] == len(want_idx) and c[1] == 0
    assert np.array_equal(idx.cpu().numpy()[: c[0]], want_idx)
    assert np.array_equal(host(vals)[: c[0]], oreduce.mean_reduce(list(x[:, want_idx]), divisor=1))
    ops.sparta_scatter(vals, idx, count, cap, float(K), src)
    want = osparta.sparse_average(list(x), mask)
    got = host(src)
    for k in range(K):
        assert np.array_equal(got[k], want[k])


@pytest.mark.parametrize("K,with_list,use_mask", [(32, False, False), (3, True, False), (2, False, True)])
def test_sparta_average_local(K, with_list, use_mask):
    """Fused single-process step: select + gather + average + write-back."""
    from gym_amd import ops
    n, p = 300_001, 0.01
    rng = np.random.default_rng(K)
    x = rng.standard_normal((K, n)).astype(np.float32)
    seed, it = 99, 4
    if use_mask:
        m = rng.random(n) < 0.02
        mask_t = torch.zeros(n + 15, dtype=torch.uint8, device=DEV)
        mask_t[:n] = torch.from_numpy(m.astype(np.uint8)).to(DEV)
    else:
        m = osparta.philox_mask(n, seed, it, p)
        mask_t = None
    src = t(x)
    kw = {}
    if with_list:
        cap = int(m.sum()) + 16
        idx, count, work = _sparta_buffers(n, cap)
        vals = torch.empty(cap, device=DEV)
        kw = dict(idx=idx, vals=vals, cap=cap, count=count, work=work)
    ops.sparta_average_local(src, n, float(K), mask=mask_t, seed=seed, iteration=it, p=p, **kw)
    want = osparta.sparse_average(list(x), m)
    got = host(src)
    for k in range(K):
        assert np.array_equal(got[k], want[k])
    if with_list:
        c = int(count[0].item())
        assert c == int(m.sum()) and np.array_equal(idx[:c].cpu().numpy(), np.flatnonzero(m))


@pytest.mark.parametrize("fused", [False, True])
def test_sparta_philox_skip_ranges(fused):
    """Tensors without a gradient are never selected (sparta.py:29-30): skip
    ranges that start/end inside a 16-element group, adjacent ranges, one
    covering whole tiles, one at the arena end."""
    from gym_amd import ops
    n, p, K = 200_003, 0.2, 2
    skip = [(0, 5), (5, 17), (33, 34), (1000, 9192), (12_301, 12_302), (50_000, 150_000), (199_990, 200_003)]
    rng = np.random.default_rng(7)
    x = rng.standard_normal((K, n)).astype(np.float32)
    seed, it = 0xABCDEF, 3
    m = osparta.philox_mask(n, seed, it, p, skip=skip)
    assert not any(m[a:b].any() for a, b in skip) and m.sum() > 0
    cap = int(m.sum()) + 16
    idx, count, work = _sparta_buffers(n, cap)
    vals = torch.empty(cap, device=DEV)
    sk = torch.tensor(skip, dtype=torch.int64, device=DEV)
    src = t(x)
    if fused:
        ops.sparta_average_local(src, n, float(K), seed=seed, iteration=it, p=p, idx=idx, vals=vals, cap=cap,
                                 count=count, work=work, skip=sk)
    else:
        ops.sparta_select(src, n, cap, idx, vals, count, work, seed=seed, iteration=it, p=p, skip=sk)
        ops.sparta_scatter(vals, idx, count, cap, float(K), src)
    c = int(count[0].item())
    assert c == int(m.sum()) and np.array_equal(idx[:c].cpu().numpy(), np.flatnonzero(m))
    want = osparta.sparse_average(list(x), m)
    got = host(src)
    for k in range(K):
        assert np.array_equal(got[k], want[k])


@pytest.mark.parametrize("K,use_mask,with_list", [(32, False, False), (32, False, True), (5, True, False),
                                                   (64, False, False), (3000, False, False)])
def test_sparta_average_local_element_major(K, use_mask, with_list):
    """[n, K] element-major replica sets (one element's K replicas adjacent):
    the same selection and ascending-replica fp32 mean as the [K, n] layout."""
    from gym_amd import ops
    n, p = (300_001, 0.01) if K < 1000 else (20_000, 0.002)
    rng = np.random.default_rng(K + 7)
    x = rng.standard_normal((K, n)).astype(np.float32)
    seed, it = 1234, 9
    if use_mask:
        m = rng.random(n) < 0.02
        mask_t = torch.zeros(n + 15, dtype=torch.uint8, device=DEV)
        mask_t[:n] = torch.from_numpy(m.astype(np.uint8)).to(DEV)
    else:
        m = osparta.philox_mask(n, seed, it, p)
        mask_t = None
    em = t(np.ascontiguousarray(x.T))  # [n, K]
    kw = {}
    if with_list:
        cap = int(m.sum()) + 16
        idx, count, work = _sparta_buffers(n, cap)
        kw = dict(idx=idx, vals=torch.empty(cap, device=DEV), cap=cap, count=count, work=work)
    ops.sparta_average_local(em, n, float(K), mask=mask_t, seed=seed, iteration=it, p=p, layout="elem", **kw)
    want = osparta.sparse_average(list(x), m)
    got = host(em).T
    for k in range(K):
        assert np.array_equal(got[k], want[k])
    if with_list:
        c = int(kw["count"][0].item())
        assert c == int(m.sum()) and np.array_equal(kw["idx"][:c].cpu().numpy(), np.flatnonzero(m))


def test_sparta_select_scatter_element_major_padded_rows():
    """Element-major set with a row stride > K ([n, 40] buffer, K = 32 used):
    select+gather, scatter; the 8 spare columns are never touched."""
    from gym_amd import ops
    n, p, K = 100_003, 0.02, 32
    rng = np.random.default_rng(3)
    x = rng.standard_normal((K, n)).astype(np.float32)
    buf = torch.full((n, 40), 5.0, device=DEV)
    buf[:, :K] = t(np.ascontiguousarray(x.T))
    em = buf[:, :K]
    seed, it = 77, 2
    skip = [(100, 5000), (60_001, 60_017)]
    m = osparta.philox_mask(n, seed, it, p, skip=skip)
    cap = int(m.sum()) + 32
    idx, count, work = _sparta_buffers(n, cap)
    vals = torch.empty(cap, device=DEV)
    sk = torch.tensor(skip, dtype=torch.int64, device=DEV)
    ops.sparta_select(em, n, cap, idx, vals, count, work, seed=seed, iteration=it, p=p, skip=sk, layout="elem")
    c = int(count[0].item())
    assert c == int(m.sum()) and np.array_equal(idx[:c].cpu().numpy(), np.flatnonzero(m))
    assert np.array_equal(host(vals)[:c], oreduce.mean_reduce(list(x[:, m]), divisor=1))
    ops.sparta_scatter(vals, idx, count, cap, float(K), em, layout="elem")
    want = osparta.sparse_average(list(x), m)
    got = host(buf)
    assert np.array_equal(got[:, :K].T, np.stack(want))
    assert (got[:, K:] == 5.0).all()


@pytest.mark.parametrize("src,p", [("philox", 1.0), ("philox", 0.9), ("philox", 0.0), ("mask", 0.95)])
def test_sparta_dense_selection_windows(src, p):
    """Selections denser than one list window per 16384-element tile (kSelCap):
    p = 1 (every element: 17 Philox calls per 64-element group), p = 0.9, a
    95%-dense uint8 mask; p = 0 selects nothing.  List and fused forms."""
    from gym_amd import ops
    n, K = 70_001, 2
    rng = np.random.default_rng(int(p * 100))
    x = rng.standard_normal((K, n)).astype(np.float32)
    seed, it = 5, 11
    mask_t = None
    if src == "mask":
        m = rng.random(n) < p
        mask_t = torch.zeros(n + 15, dtype=torch.uint8, device=DEV)
        mask_t[:n] = torch.from_numpy(m.astype(np.uint8)).to(DEV)
    else:
        m = osparta.philox_mask(n, seed, it, p)
    cap = int(m.sum()) + 16
    idx, count, work = _sparta_buffers(n, cap)
    vals = torch.empty(cap, device=DEV)
    a = t(x)
    ops.sparta_select(a, n, cap, idx, vals, count, work, mask=mask_t, seed=seed, iteration=it, p=p)
    c = int(count[0].item())
    assert c == int(m.sum()) and np.array_equal(idx[:c].cpu().numpy(), np.flatnonzero(m))
    assert np.array_equal(host(vals)[:c], oreduce.mean_reduce(list(x[:, m]), divisor=1))
    b = t(x)
    ops.sparta_average_local(b, n, float(K), mask=mask_t, seed=seed, iteration=it, p=p)
    want = osparta.sparse_average(list(x), m)
    got = host(b)
    for k in range(K):
        assert np.array_equal(got[k], want[k])


def test_sparta_overflow_flag():
    from gym_amd import ops
    n = 10_000
    x = t(np.ones((1, n), np.float32))
    idx, count, work = _sparta_buffers(n, 100)
    vals = torch.empty(100, device=DEV)
    ops.sparta_select(x, n, 100, idx, vals, count, work, seed=1, iteration=0, p=0.5)
    c = count.cpu().numpy()
    assert c[0] > 100 and c[1] == 1
    ops.sparta_scatter(vals, idx, count, 100, 1.0, x)  # writes only the first cap entries
    torch.cuda.synchronize()


@pytest.mark.parametrize("K", [2, 3])
def test_sparta_mask_mode_matches_reference_golden(golden, K):
    """The reference's own masks (rank 0's, logged) through the mask-mode
    kernels, the K nodes as replicas: identical to SPARTAStrategy's result."""
    from gym_amd import ops
    from gym_amd.arena import ArenaLayout
    z = golden("sparta.npz")
    calls, ns = int(z["calls"]), int(z["nshapes"])
    shapes = [z[f"K{K}_before_0_{i}"].shape[1:] for i in range(ns)]
    L = ArenaLayout(shapes)
    for call in range(calls):
        reps = torch.zeros(K, L.n, device=DEV)
        mask = torch.zeros(L.n, dtype=torch.uint8, device=DEV)
        for i in range(ns):
            n_i = int(np.prod(shapes[i]))
            m = np.unpackbits(z[f"K{K}_mask_{call}_{i}"])[:n_i].astype(np.uint8)
            L.views(mask)[i].copy_(torch.from_numpy(m.reshape(shapes[i])))
            for k in range(K):
                L.views(reps[k])[i].copy_(t(z[f"K{K}_before_{call}_{i}"][k]))
        cap = int(mask.sum().item())
        idx, count, work = _sparta_buffers(L.n, cap)
        vals = torch.empty(cap, device=DEV)
        ops.sparta_select(reps, L.n, cap, idx, vals, count, work, mask=mask)
        ops.sparta_scatter(vals, idx, count, cap, float(K), reps)
        for i in range(ns):
            for k in range(K):
                got = host(L.views(reps[k])[i])
                ref = z[f"K{K}_after_{call}_{i}"][k]
                if K == 2:
                    assert np.array_equal(got, ref)
                else:
                    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-9)


# ---------------------------------------------------------------- DeMo --------
DEMO_SHAPES = [(128, 128), (66, 128), (768,), (8, 4, 3, 3), (10,), (58, 29), (64, 64)]
# every chunk 64x64 or 1x64: the plan takes the wave-per-chunk encode (ga_demo_encode_sym)
DEMO_WAVE_SHAPES = [(128, 128), (768,), (64, 64), (192, 128), (320,), (64, 192)]


def _demo_setup(shapes, K, seed=0, dtype=torch.float32):
    from gym_amd.arena import ArenaLayout
    from gym_amd.demo_codec import DemoPlan
    L = ArenaLayout(shapes)
    plan = DemoPlan(L, chunk=64, topk=32)
    rng = np.random.default_rng(seed)
    arrs = {}
    for name in ("p", "g", "d"):
        host_arr = np.zeros((K, L.n), np.float32)
        for k in range(K):
            for o, nel in zip(L.offsets, L.numels):
                host_arr[k, o:o + nel] = rng.standard_normal(nel) * (0.02 if name == "p" else 1e-2)
        if name == "p":
            host_arr[:] = host_arr[0]  # DeMo keeps params identical across nodes
        arrs[name] = host_arr
    return L, plan, arrs


def _payload_host(pl, plan):
    a = pl.cpu().numpy()
    return a[:, : plan.M], a[:, plan.M: 2 * plan.M].view(np.float32)


@pytest.mark.parametrize("K,wave", [(1, False), (2, False), (3, False), (5, False), (1, True), (3, True)])
def test_demo_encode_decode_matches_oracle(K, wave):
    from gym_amd import ops
    shapes = DEMO_WAVE_SHAPES if wave else DEMO_SHAPES
    L, plan, a = _demo_setup(shapes, K, seed=K)
    assert plan.wave_encode == wave
    lr, decay, wd = 0.01, 0.999, 0.1
    wdf = float(np.float32(1.0 - lr * wd))
    P, G, D = t(a["p"]), t(a["g"]), t(a["d"])
    payload = torch.zeros(K, 2 * plan.M, dtype=torch.int32, device=DEV)
    ops.demo_encode(plan, P, G, D, payload, lr, decay, wdf)
    gidx, gval = _payload_host(payload, plan)
    grad_out = torch.zeros_like(G)
    ops.demo_decode(plan, payload, P, grad_out, lr)
    gP, gD, gS = host(P), host(D), host(grad_out)
    tally = demo_checks.SignTally()
    for ti, (shape, off, nel) in enumerate(zip(L.shapes, L.offsets, L.numels)):
        R, C, n1, n2 = odemo.tensor_view(shape, 64)
        p0 = a["p"][0, off:off + nel].reshape(shape)
        deltas = [a["d"][k, off:off + nel].reshape(shape) for k in range(K)]
        grads = [a["g"][k, off:off + nel].reshape(shape) for k in range(K)]
        want_p, want_d, want_s, sent, g_hat, margins = odemo.demo_step(p0, deltas, grads, lr, decay, 32, 64, wd,
                                                                       detail=True)
        e0 = sum(plan.entries_per_tensor[:ti])
        ne = plan.entries_per_tensor[ti]
        kk = max(1, min(32, n1 * n2))
        for k in range(K):
            idx_k = gidx[k, e0:e0 + ne].reshape(R // n1, C // n2, kk)
            val_k = gval[k, e0:e0 + ne].reshape(R // n1, C // n2, kk)
            oidx, oval = sent[k]
            # index sets exact where the k-th magnitude is not (nearly) tied
            d64 = np.asarray(deltas[k], np.float64) * decay + lr * np.asarray(grads[k], np.float64)
            margin = odemo.kth_margin(odemo.encode(d64, shape, 64), 32).reshape(R // n1, C // n2)
            scale = np.abs(oval).max()
            for y in range(R // n1):
                for x in range(C // n2):
                    if margin[y, x] > 1e-5 * scale:
                        assert np.array_equal(idx_k[y, x], oidx[y, x]), (shape, y, x)
                        np.testing.assert_allclose(val_k[y, x], oval[y, x], rtol=0, atol=1e-5 * scale)
            # residual compared in the chunks whose selected set is unambiguous
            okc = margin > 1e-5 * scale
            okel = np.repeat(np.repeat(okc, n1, axis=0), n2, axis=1).reshape(shape)
            np.testing.assert_allclose(gD[k, off:off + nel].reshape(shape)[okel], want_d[k][okel], rtol=0,
                                       atol=1e-5 * max(np.abs(d64).max(), 1e-12))
        # sign-SGD apply: exact signs wherever the sign is decided (tests/demo_checks.py)
        s = gS[0, off:off + nel].reshape(shape)
        tally.check(s, want_s, demo_checks.firm(g_hat, margins, shape), what=str(shape))
        ok = s == want_s
        np.testing.assert_allclose(gP[0, off:off + nel].reshape(shape)[ok], want_p[ok], rtol=0, atol=1e-6)
        for k in range(1, K):
            assert np.array_equal(gP[k, off:off + nel], gP[0, off:off + nel])
    # a near-tied chunk is excluded whole (one 64x64 chunk = 13% of these ~31.7k
    # elements; K=3 gives 3x the chances), so on these few-chunk tensors the floor
    # is lower than at full size (test_gpu_fullsize)
    tally.done(min_firm=0.8)
    # padding between tensors stays exactly zero in every arena
    for arr in (gP, gD, gS):
        for o, nel, o2 in zip(L.offsets, L.numels, L.offsets[1:] + [L.n]):
            assert (arr[:, o + nel:o2] == 0).all()


def test_demo_matches_reference_golden_steps(golden):
    """Three DeMo.step()s of the reference (K=2 nodes over gloo) replayed with
    the 2 nodes as replicas."""
    from gym_amd import ops
    from gym_amd.arena import ArenaLayout
    from gym_amd.demo_codec import DemoPlan
    z = golden("demo_steps.npz")
    K, steps, ns = int(z["K"]), int(z["steps"]), int(z["nshapes"])
    lr, wd, decay = float(z["lr"]), float(z["wd"]), float(z["decay"])
    shapes = [z[f"p_before_0_{i}"].shape for i in range(ns)]
    L = ArenaLayout(shapes)
    plan = DemoPlan(L, chunk=int(z["chunk"]), topk=int(z["topk"]))
    assert plan.reference_bytes() == int(z["tx_0"])
    P = torch.zeros(K, L.n, device=DEV)
    D = torch.zeros(K, L.n, device=DEV)
    G = torch.zeros(K, L.n, device=DEV)
    payload = torch.zeros(K, 2 * plan.M, dtype=torch.int32, device=DEV)
    wdf = float(np.float32(1.0 - lr * wd))
    tally = demo_checks.SignTally()
    for step in range(steps):
        for i in range(ns):  # start each step from the reference state
            for k in range(K):
                L.views(P[k])[i].copy_(t(z[f"p_before_{step}_{i}"]))
                L.views(D[k])[i].copy_(t(z[f"delta_before_{step}_{i}"][k]))
                L.views(G[k])[i].copy_(t(z[f"grad_{step}_{i}"][k]))
        ops.demo_encode(plan, P, G, D, payload, lr, decay, wdf)
        ops.demo_decode(plan, payload, P, G, lr)
        for i in range(ns):
            ref_s = z[f"sign_{step}_{i}"]
            s = host(L.views(G[0])[i])
            # where the reference's sign is decided (oracle g_hat and top-k margins on the same inputs)
            _, _, _, _, g_hat, margins = odemo.demo_step(
                z[f"p_before_{step}_{i}"], list(z[f"delta_before_{step}_{i}"]), list(z[f"grad_{step}_{i}"]), lr,
                decay, int(z["topk"]), int(z["chunk"]), wd, detail=True)
            tally.check(s, ref_s, demo_checks.firm(g_hat, margins, shapes[i], int(z["chunk"])),
                        what=f"step {step} tensor {i}")
            ok = s == ref_s
            np.testing.assert_allclose(host(L.views(P[0])[i])[ok], z[f"p_after_{step}_{i}"][ok], rtol=0, atol=1e-6)
            for k in range(K):  # 1e-6 x the chunk's scale wherever the node's top-k set is firm
                x = decay * z[f"delta_before_{step}_{i}"][k].astype(np.float64) + lr * z[f"grad_{step}_{i}"][k]
                demo_checks.residual_close(host(L.views(D[k])[i]), z[f"delta_after_{step}_{i}"][k], x, margins[k],
                                           shapes[i], int(z["chunk"]), what=f"step {step} tensor {i} node {k}")
    tally.done()


def test_demo_bf16_vs_reference_bf16_golden(golden):
    """Three DeMo.step()s of the reference on bf16 parameters (K=2 over gloo,
    tests/golden/demo_steps_bf16.npz) replayed as 2 replicas.  The reference runs
    its DCT in bf16 (bases cast to bf16, every einsum stage rounded) and breaks the
    many bf16 top-k ties in torch's CPU selection order, so bit-parity is not
    defined for bf16; the bars are the statistical ones of
    demo_checks.bf16_agreement, which the fp64 oracle also meets on the same
    inputs (test_oracle_golden.py::test_oracle_vs_reference_bf16_golden)."""
    from gym_amd import ops
    from gym_amd.arena import ArenaLayout
    from gym_amd.demo_codec import DemoPlan
    z = golden("demo_steps_bf16.npz")
    K, steps, ns = int(z["K"]), int(z["steps"]), int(z["nshapes"])
    lr, wd, decay = float(z["lr"]), float(z["wd"]), float(z["decay"])
    shapes = [z[f"p_before_0_{i}"].shape for i in range(ns)]
    L = ArenaLayout(shapes)
    plan = DemoPlan(L, chunk=int(z["chunk"]), topk=int(z["topk"]))
    assert plan.reference_bytes(2) == int(z["tx_0"])
    P, D, G = (torch.zeros(K, L.n, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    payload = torch.zeros(K, 2 * plan.M, dtype=torch.int32, device=DEV)
    wdf = float(np.float32(1.0 - lr * wd))
    agree = demo_checks.Bf16Agreement()
    for step in range(steps):
        for i in range(ns):
            for k in range(K):
                L.views(P[k])[i].copy_(t(z[f"p_before_{step}_{i}"], torch.bfloat16))
                L.views(D[k])[i].copy_(t(z[f"delta_before_{step}_{i}"][k], torch.bfloat16))
                L.views(G[k])[i].copy_(t(z[f"grad_{step}_{i}"][k], torch.bfloat16))
        P0 = P.clone()
        ops.demo_encode(plan, P, G, D, payload, lr, decay, wdf)
        ops.demo_decode(plan, payload, P, G, lr)
        # the reference's own update ops (demo.py:159-160, torch SGD p.add_(grad, alpha=-lr)) as torch
        # runs them on this GPU in bf16, fed our signs: bit-identical to the kernel's update
        want = P0.mul_(1.0 - lr * wd).add_(G, alpha=-lr)
        assert torch.equal(want, P), "bf16 p update differs from torch's bf16 mul_/add_ on the GPU"
        for i in range(ns):
            agree.check(host(L.views(G[0])[i]), host(L.views(P[0])[i]), [host(L.views(D[k])[i]) for k in range(K)],
                        z, step, i)
    agree.done()


def _bf16_golden_step(z, step, L, plan, alpha):
    """One G4b step through the codec kernels from the step's recorded state:
    (P, G = sign, D per node) of replica 0 / every node, as bf16 tensors."""
    from gym_amd import ops
    K, ns = int(z["K"]), int(z["nshapes"])
    lr, wd, decay = float(z["lr"]), float(z["wd"]), float(z["decay"])
    P, D, G = (torch.zeros(K, L.n, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    for i in range(ns):
        for k in range(K):
            L.views(P[k])[i].copy_(t(z[f"p_before_{step}_{i}"], torch.bfloat16))
            L.views(D[k])[i].copy_(t(z[f"delta_before_{step}_{i}"][k], torch.bfloat16))
            L.views(G[k])[i].copy_(t(z[f"grad_{step}_{i}"][k], torch.bfloat16))
    payload = torch.zeros(K, 2 * plan.M, dtype=torch.int32, device=DEV)
    P0 = P.clone()
    ops.demo_encode(plan, P, G, D, payload, alpha, decay, float(np.float32(1.0 - lr * wd)))
    ops.demo_decode(plan, payload, P, G, alpha)
    return P0, P, G, D


def test_demo_bf16_reference_transform_is_torch_on_gpu(golden):
    """DeMo(bf16_transform="reference") -- GA_BF16_REF: bf16 bases, every einsum
    stage rounded to bf16 in the reference's contraction order, the delta rounded
    after the decay and after the add -- against the reference's op sequence as
    torch runs it on this GPU (oracle/demo_bf16.py with device cuda: bf16 einsums
    on the GPU's GEMMs, torch.topk on the GPU, fp32 alpha), from each of G4b's
    recorded states: parameters, signs and both nodes' deltas BIT-IDENTICAL."""
    from gym_amd.arena import ArenaLayout
    from gym_amd.demo_codec import DemoPlan
    from oracle import demo_bf16 as ob
    z = golden("demo_steps_bf16.npz")
    K, steps, ns = int(z["K"]), int(z["steps"]), int(z["nshapes"])
    lr, wd, decay = float(z["lr"]), float(z["wd"]), float(z["decay"])
    shapes = [z[f"p_before_0_{i}"].shape for i in range(ns)]
    L = ArenaLayout(shapes)
    plan = DemoPlan(L, chunk=int(z["chunk"]), topk=int(z["topk"]), bf16_transform="reference")
    assert not plan.wave_encode
    for step in range(steps):
        P0, P, G, D = _bf16_golden_step(z, step, L, plan, lr)
        # the update is torch's own bf16 ops on this GPU, fed the kernel's signs
        assert torch.equal(P0.mul_(1.0 - lr * wd).add_(G, alpha=-lr), P)
        for i in range(ns):
            rp, rd, rs = ob.demo_step(z[f"p_before_{step}_{i}"], list(z[f"delta_before_{step}_{i}"]),
                                      list(z[f"grad_{step}_{i}"]), lr, decay, int(z["topk"]), int(z["chunk"]), wd,
                                      device=DEV)
            assert np.array_equal(host(L.views(G[0])[i]), rs), (step, i)
            assert np.array_equal(host(L.views(P[0])[i]), rp), (step, i)
            for k in range(K):
                assert np.array_equal(host(L.views(D[k])[i]), rd[k]), (step, i, k)


def test_demo_bf16_reference_transform_vs_cpu_golden(golden):
    """The same path against G4b itself (the reference's bf16 run on the CPU),
    alpha rounded to bf16 as torch's CPU add_ does.  What still differs is the
    CPU topk's order among tied bf16 magnitudes -- the reference run on the GPU
    differs from its own CPU run by the same amount (tools/bf16_agreement.py:
    sign agreement 0.939 worst tensor / 0.977 overall) -- so the bar is
    demo_checks.Bf16Agreement's for signs and p, and the deltas bit-identical in
    >= 60% of elements (the ones outside tie-affected chunks)."""
    from gym_amd.arena import ArenaLayout
    from gym_amd.demo_codec import DemoPlan
    z = golden("demo_steps_bf16.npz")
    K, steps, ns = int(z["K"]), int(z["steps"]), int(z["nshapes"])
    lr, wd = float(z["lr"]), float(z["wd"])
    shapes = [z[f"p_before_0_{i}"].shape for i in range(ns)]
    L = ArenaLayout(shapes)
    plan = DemoPlan(L, chunk=int(z["chunk"]), topk=int(z["topk"]), bf16_transform="reference")
    alpha = float(torch.tensor(lr).bfloat16().float())
    agree = demo_checks.Bf16Agreement(delta_rel=float("inf"))
    same = total = 0
    for step in range(steps):
        _, P, G, D = _bf16_golden_step(z, step, L, plan, alpha)
        for i in range(ns):
            ds = [host(L.views(D[k])[i]) for k in range(K)]
            agree.check(host(L.views(G[0])[i]), host(L.views(P[0])[i]), ds, z, step, i)
            same += sum(int((d == z[f"delta_after_{step}_{i}"][k]).sum()) for k, d in enumerate(ds))
            total += sum(d.size for d in ds)
    agree.done()
    assert same / total >= 0.6, same / total


@pytest.mark.parametrize("kernel", ["wave", "block"])
def test_demo_all_zero_chunk_tie_rule(monkeypatch, kernel):
    from gym_amd import ops
    from gym_amd.arena import ArenaLayout
    from gym_amd.demo_codec import DemoPlan
    if kernel == "block":
        monkeypatch.setenv("GA_DEMO_ENCODE", "block")
    L = ArenaLayout([(128, 128)])
    plan = DemoPlan(L)
    assert plan.wave_encode
    P = torch.zeros(1, L.n, device=DEV)
    payload = torch.full((1, 2 * plan.M), -1, dtype=torch.int32, device=DEV)
    ops.demo_encode(plan, P, P.clone(), P.clone(), payload, 0.01, 0.999, 1.0)
    idx, val = _payload_host(payload, plan)
    assert (val == 0).all()
    assert all(np.array_equal(idx[0, c * 32:(c + 1) * 32], np.arange(32)) for c in range(4))


@pytest.mark.parametrize("topk,chunk,wave", [(300, 64, False), (8, 16, False), (64, 32, False), (1, 64, True),
                                             (8, 64, True), (48, 64, True), (64, 64, True), (65, 64, False)])
def test_demo_topk_and_chunk_variants(topk, chunk, wave):
    """k > 256 (radix-select path), small chunks, k == chunk; the wave kernel's
    k range (k <= 64; k > 32 mostly takes its all-keys selection)."""
    from gym_amd import ops
    from gym_amd.arena import ArenaLayout
    from gym_amd.demo_codec import DemoPlan
    shapes = [(128, 128), (192,), (64, 128)] if chunk == 64 and topk <= 65 else [(128, 128), (96,), (32, 48)]
    L = ArenaLayout(shapes)
    plan = DemoPlan(L, chunk=chunk, topk=topk)
    assert plan.wave_encode == wave
    rng = np.random.default_rng(topk + chunk)
    D = np.zeros((1, L.n), np.float32)
    for o, nel in zip(L.offsets, L.numels):
        D[0, o:o + nel] = rng.standard_normal(nel)
    P, G, Dt = t(np.zeros_like(D)), t(np.zeros_like(D)), t(D)
    payload = torch.zeros(1, 2 * plan.M, dtype=torch.int32, device=DEV)
    ops.demo_encode(plan, P, G, Dt, payload, 0.01, 1.0 - 1e-9, 1.0)
    gidx, gval = _payload_host(payload, plan)
    gD = host(Dt)
    e0 = 0
    for ti, (shape, off, nel) in enumerate(zip(L.shapes, L.offsets, L.numels)):
        R, C, n1, n2 = odemo.tensor_view(shape, chunk)
        kk = max(1, min(topk, n1 * n2))
        Y = odemo.encode(D[0, off:off + nel].reshape(shape), shape, chunk)
        oidx, oval = odemo.topk_chunks(Y, topk)
        margin = odemo.kth_margin(Y, topk).reshape(R // n1, C // n2)
        ne = plan.entries_per_tensor[ti]
        gi = gidx[0, e0:e0 + ne].reshape(R // n1, C // n2, kk)
        for y in range(R // n1):
            for x in range(C // n2):
                if margin[y, x] > 1e-5:
                    assert np.array_equal(gi[y, x], oidx[y, x]), (shape, y, x)
        # residual delta - IDCT(top-k) (odd k: the synthesis lists' one zero entry),
        # in the chunks whose selected set is unambiguous
        gy, gx = R // n1, C // n2
        Ym = np.zeros_like(Y).reshape(gy * gx, n1 * n2)
        np.put_along_axis(Ym, oidx.reshape(gy * gx, kk), oval.reshape(gy * gx, kk), axis=1)
        want_d = D[0, off:off + nel].reshape(shape) - odemo.decode(Ym.reshape(Y.shape), shape, chunk)
        okel = np.repeat(np.repeat((margin > 1e-5).reshape(gy, gx), n1, axis=0), n2, axis=1).reshape(shape)
        np.testing.assert_allclose(gD[0, off:off + nel].reshape(shape)[okel], want_d[okel], rtol=0, atol=2e-5)
        e0 += ne


@pytest.mark.parametrize("shapes", [[(128, 128), (768,), (66, 128)], [(128, 128), (768,)]])
def test_demo_bf16_matches_oracle(shapes):
    from gym_amd import ops
    L, plan, a = _demo_setup(shapes, 2, seed=11)
    lr = 0.01
    P = t(a["p"], torch.bfloat16)
    G = t(a["g"], torch.bfloat16)
    D = t(a["d"], torch.bfloat16)
    p0 = P.float().cpu().numpy()
    d0 = D.float().cpu().numpy()
    g0 = G.float().cpu().numpy()
    payload = torch.zeros(2, 2 * plan.M, dtype=torch.int32, device=DEV)
    ops.demo_encode(plan, P, G, D, payload, lr, 0.999, 1.0)
    Gs = torch.zeros_like(G)
    ops.demo_decode(plan, payload, P, Gs, lr)
    gP, gD = host(P), host(D)
    tally = demo_checks.SignTally()
    for shape, off, nel in zip(L.shapes, L.offsets, L.numels):
        want_p, want_d, want_s, _, g_hat, margins = odemo.demo_step(
            p0[0, off:off + nel].reshape(shape), [d0[k, off:off + nel].reshape(shape) for k in range(2)],
            [g0[k, off:off + nel].reshape(shape) for k in range(2)], lr, detail=True)
        s = host(Gs)[0, off:off + nel].reshape(shape)
        # the codec reads the bf16 values and computes in fp32 (payload values fp32),
        # so the decided signs are the fp32 ones
        tally.check(s, want_s, demo_checks.firm(g_hat, margins, shape), what=str(shape))
        np.testing.assert_allclose(gP[0, off:off + nel].reshape(shape)[s == want_s], want_p[s == want_s],
                                   rtol=1e-2, atol=1e-3)
        for k in range(2):
            np.testing.assert_allclose(gD[k, off:off + nel].reshape(shape), want_d[k], rtol=0,
                                       atol=1e-2 * np.abs(want_d[k]).max())
    tally.done()


def test_sparta_bf16_and_many_replicas():
    from gym_amd import ops
    n, p = 200_003, 0.02
    for K, dtype in ((4, torch.bfloat16), (64, torch.float32)):
        x = np.random.default_rng(K).standard_normal((K, n)).astype(np.float32)
        src = t(x, dtype)
        xs = src.float().cpu().numpy()
        m = osparta.philox_mask(n, 5, 6, p)
        ops.sparta_average_local(src, n, float(K), seed=5, iteration=6, p=p)
        want = osparta.sparse_average(list(xs), m)
        got = host(src)
        tol = 1e-2 if dtype == torch.bfloat16 else 0
        for k in range(K):
            np.testing.assert_allclose(got[k], want[k], rtol=tol, atol=tol)


@pytest.mark.parametrize("K,dtype,ld", [(8, torch.bfloat16, 8), (32, torch.bfloat16, 32), (12, torch.float32, 16),
                                         (12, torch.float32, 14)])
def test_sparta_element_major_vector_rows(K, dtype, ld):
    """Element-major sets whose rows take 4-replica vector loads (K and the row
    stride multiples of 4; bf16 and fp32) and one whose stride (14) does not:
    the same selections and ascending-replica means either way."""
    from gym_amd import ops
    n, p = 150_001, 0.02
    x = np.random.default_rng(K + ld).standard_normal((K, n)).astype(np.float32)
    buf = torch.full((n, ld), 7.0, device=DEV, dtype=dtype)
    buf[:, :K] = t(np.ascontiguousarray(x.T), dtype)
    xs = buf[:, :K].float().cpu().numpy().T
    m = osparta.philox_mask(n, 21, 4, p)
    cap = int(m.sum()) + 8
    idx, count, work = _sparta_buffers(n, cap)
    vals = torch.empty(cap, device=DEV, dtype=dtype)
    ops.sparta_average_local(buf[:, :K], n, float(K), seed=21, iteration=4, p=p, idx=idx, vals=vals, cap=cap,
                             count=count, work=work, layout="elem")
    c = int(count[0].item())
    assert c == int(m.sum()) and np.array_equal(idx[:c].cpu().numpy(), np.flatnonzero(m))
    want = osparta.sparse_average(list(xs), m)
    got = buf.float().cpu().numpy()
    tol = 1e-2 if dtype == torch.bfloat16 else 0
    np.testing.assert_allclose(got[:, :K].T, np.stack(want), rtol=tol, atol=tol)
    assert (got[:, K:] == 7.0).all()
    # the multi-rank form: select + gather into the packed list, scatter back
    buf2 = torch.full((n, ld), 7.0, device=DEV, dtype=dtype)
    buf2[:, :K] = t(np.ascontiguousarray(x.T), dtype)
    ops.sparta_select(buf2[:, :K], n, cap, idx, vals, count, work, seed=21, iteration=4, p=p, layout="elem")
    ops.sparta_scatter(vals, idx, count, cap, float(K), buf2[:, :K], layout="elem")
    got2 = buf2.float().cpu().numpy()
    np.testing.assert_allclose(got2[:, :K].T, np.stack(want), rtol=tol, atol=tol)
    assert (got2[:, K:] == 7.0).all()


def test_replica_mean_edge_sizes():
    from gym_amd import ops
    empty = torch.zeros(0, device=DEV)
    ops.replica_mean(empty.view(1, 0), empty.view(1, 0), n=0)
    x = torch.arange(6, dtype=torch.float32, device=DEV).view(2, 3)  # ld 3: scalar path
    out = torch.empty(3, device=DEV)
    ops.replica_mean(x, out)
    assert host(out).tolist() == [1.5, 2.5, 3.5]


@pytest.mark.parametrize("S,kernel", [(1, "wave"), (2, "wave"), (3, "wave"), (8, "wave"), (15, "wave"), (16, "wave"),
                                      (8, "block")])
def test_demo_decode_sources_with_collisions(monkeypatch, S, kernel):
    """Decode of S hand-made payloads whose entries collide heavily (every chunk
    draws its k indices from a pool of 40-48 coefficients): scatter-mean over the
    hitters, inverse DCT, sign, p -= lr*sign on 2 replicas, vs the oracle.  S <= 15
    takes ga_demo_decode_sym (S = 16 falls back to ga_demo_decode)."""
    from gym_amd import ops
    if kernel == "block":
        monkeypatch.setenv("GA_DEMO_DECODE", "block")
    L, plan, a = _demo_setup(DEMO_WAVE_SHAPES, 2, seed=100 + S)
    assert plan.wave_encode
    rng = np.random.default_rng(S)
    lr = 0.01
    idx = np.zeros((S, plan.M), np.int32)
    val = np.zeros((S, plan.M), np.float32)
    e0 = 0
    per_tensor = []
    for shape in L.shapes:
        R, C, n1, n2 = odemo.tensor_view(shape, 64)
        kk = max(1, min(32, n1 * n2))
        gy, gx = R // n1, C // n2
        pool = min(n1 * n2, 40 if n1 > 1 else 48)
        ti = np.sort(np.stack([np.stack([rng.choice(pool, kk, replace=False) for _ in range(gy * gx)])
                               for _ in range(S)]), axis=-1).astype(np.int32)
        tv = rng.standard_normal(ti.shape).astype(np.float32)
        idx[:, e0:e0 + gy * gx * kk] = ti.reshape(S, -1)
        val[:, e0:e0 + gy * gx * kk] = tv.reshape(S, -1)
        per_tensor.append((ti.reshape(S, gy, gx, kk), tv.reshape(S, gy, gx, kk)))
        e0 += gy * gx * kk
    payload = torch.from_numpy(np.concatenate([idx, val.view(np.int32)], axis=1)).to(DEV)
    P = t(a["p"])
    Gs = torch.full_like(P, 7.0)
    ops.demo_decode(plan, payload, P, Gs, lr)
    gP, gS = host(P), host(Gs)
    for (shape, off, nel), (ti, tv) in zip(zip(L.shapes, L.offsets, L.numels), per_tensor):
        R, C, n1, n2 = odemo.tensor_view(shape, 64)
        Y = odemo.scatter_mean(list(ti), list(tv), n1, n2)
        g = odemo.decode(Y, shape, 64)
        want_s = np.sign(g).astype(np.float32)
        firm = np.abs(g) > 1e-5 * np.abs(g).max()
        p0 = a["p"][0, off:off + nel].reshape(shape)
        for k in range(2):
            s = gS[k, off:off + nel].reshape(shape)
            assert np.array_equal(s[firm], want_s[firm]), (shape, k)
            assert np.isin(s, (-1.0, 0.0, 1.0)).all()
            np.testing.assert_allclose(gP[k, off:off + nel].reshape(shape), p0 - lr * s, rtol=0, atol=1e-7)
    for o, nel, o2 in zip(L.offsets, L.numels, L.offsets[1:] + [L.n]):  # padding untouched
        assert (gS[:, o + nel:o2] == 7.0).all()


@pytest.mark.parametrize("K,dtype,ld,p", [(32, torch.float32, 32, 0.005), (32, torch.float32, 36, 0.3),
                                          (4, torch.float32, 4, 1.0), (64, torch.float32, 64, 0.02),
                                          (68, torch.float32, 68, 0.02), (32, torch.bfloat16, 32, 0.05),
                                          (8, torch.bfloat16, 12, 0.5)])
def test_sparta_average_local_own_groups(K, dtype, ld, p):
    """ga_sparta_average_local without the packed list on a 4-aligned element-major
    set (each lane averages its own 64-element group's selections in registers,
    K <= 64; K = 68 takes the tile-gather kernel): the Philox selection with skip
    ranges, p from sparse to every element (several rounds of two elements per
    lane), bit-identical to the tile-gather form with the list and to the oracle."""
    from gym_amd import ops
    n = 100_003
    x = np.random.default_rng(K * 7 + ld).standard_normal((K, n)).astype(np.float32)
    skip = [(0, 3), (640, 700), (50_000, 50_064), (99_990, 100_003)]
    sk = torch.tensor(skip, dtype=torch.int64, device=DEV)
    seed, it = 5, 11
    m = osparta.philox_mask(n, seed, it, p, skip=skip)
    bufs = []
    for with_list in (False, True):
        buf = torch.full((n, ld), 3.0, device=DEV, dtype=dtype)
        buf[:, :K] = t(np.ascontiguousarray(x.T), dtype)
        kw = {}
        if with_list:
            cap = int(m.sum()) + 8
            idx, count, work = _sparta_buffers(n, cap)
            kw = dict(idx=idx, vals=torch.empty(cap, device=DEV, dtype=dtype), cap=cap, count=count, work=work)
        ops.sparta_average_local(buf[:, :K], n, float(K), seed=seed, iteration=it, p=p, skip=sk, layout="elem", **kw)
        bufs.append(host(buf))
    assert np.array_equal(bufs[0], bufs[1])
    xs = bufs[0]  # untouched elements keep their (dtype-rounded) inputs
    want = osparta.sparse_average(list(t(np.ascontiguousarray(x.T), dtype).float().cpu().numpy().T), m)
    tol = 1e-2 if dtype == torch.bfloat16 else 0
    np.testing.assert_allclose(xs[:, :K].T, np.stack(want), rtol=tol, atol=tol)
    assert (xs[:, K:] == 3.0).all()


@pytest.mark.parametrize("n", [1, 63, 64, 65, 300_001, 16384 * 3])
def test_sparta_pack_mask(n):
    """ga_sparta_pack_mask against oracle.sparta.pack_mask, bit for bit,
    including the ragged last word (bits past n zero) and non-0/1 mask bytes."""
    from gym_amd import ops
    rng = np.random.default_rng(n)
    m = (rng.random(n) < 0.3).astype(np.uint8) * rng.integers(1, 256, n).astype(np.uint8)
    mask_t = torch.zeros(n + 64, dtype=torch.uint8, device=DEV)
    mask_t[:n] = torch.from_numpy(m).to(DEV)
    mask_t[n:] = 1  # past n: never packed
    bits = torch.full((ops.sparta_mask_words(n) + 1,), -1, dtype=torch.int64, device=DEV)
    ops.sparta_pack_mask(mask_t, n, bits)
    got = bits.cpu().numpy()
    assert np.array_equal(got[:-1], osparta.pack_mask(m)) and got[-1] == -1
    assert np.array_equal(osparta.unpack_mask(got[:-1], n), m != 0)


@pytest.mark.parametrize("layout,K", [("rows", 3), ("elem", 32)])
def test_sparta_packed_mask_equals_byte_mask(layout, K):
    """The packed mask selects exactly what the byte mask selects: select
    (idx, vals, count) and the fused average, both layouts."""
    from gym_amd import ops
    n = 300_001
    rng = np.random.default_rng(11)
    x = rng.standard_normal((K, n)).astype(np.float32)
    m = rng.random(n) < 0.01
    mask_t = torch.zeros(n + 15, dtype=torch.uint8, device=DEV)
    mask_t[:n] = torch.from_numpy(m.astype(np.uint8)).to(DEV)
    bits = torch.empty(ops.sparta_mask_words(n), dtype=torch.int64, device=DEV)
    ops.sparta_pack_mask(mask_t, n, bits)
    mk = (lambda a: t(np.ascontiguousarray(a.T))) if layout == "elem" else t
    cap = int(m.sum()) + 16
    outs = []
    for mk_mask in (mask_t, bits):
        idx, count, work = _sparta_buffers(n, cap)
        vals = torch.empty(cap, device=DEV)
        ops.sparta_select(mk(x), n, cap, idx, vals, count, work, mask=mk_mask, layout=layout)
        c = int(count[0].item())
        outs.append((c, idx[:c].cpu().numpy(), host(vals)[:c]))
        src = mk(x)
        ops.sparta_average_local(src, n, float(K), mask=mk_mask, layout=layout)
        got = host(src).T if layout == "elem" else host(src)
        want = osparta.sparse_average(list(x), m)
        for k in range(K):
            assert np.array_equal(got[k], want[k])
    assert outs[0][0] == outs[1][0] == int(m.sum())
    assert np.array_equal(outs[0][1], np.flatnonzero(m)) and np.array_equal(outs[1][1], outs[0][1])
    assert np.array_equal(outs[0][2], outs[1][2])


@pytest.mark.parametrize("mode", ["fused", "graph", "eager"])
def test_sparta_inplace_bernoulli_is_the_reference_draw(mode):
    """draw_masks' RandomIndexSelector path (view.bernoulli_(cached full(p))
    into the uint8 arena; from the second call one HIP graph replay of the
    whole sequence) gives the reference's torch.bernoulli(torch.full(shape,
    p)).bool() bits (sparta.py:80-85) and leaves the generator where the
    reference leaves it, step after step, on GPT-2-like shapes with a
    grad-less tensor skipped."""
    from gym_amd import ops
    from gym_amd.arena import ArenaLayout
    from gym_amd.strategy.sparta import MaskDraw, RandomIndexSelector, draw_masks
    shapes = [(50304, 768), (1024, 768), (768,), (2304, 768), (2304,), (3072, 768), (66, 128), (3, 5, 7), (1,)]
    L = ArenaLayout(shapes)
    params = [torch.zeros(s, device=DEV) for s in shapes]
    sel = RandomIndexSelector(0.005)
    skip = {3}
    mask = torch.full((L.n,), 7, dtype=torch.uint8, device=DEV)
    state = MaskDraw()
    saved = (MaskDraw.fused, MaskDraw.use_graphs)
    MaskDraw.fused, MaskDraw.use_graphs = mode == "fused", mode == "graph"
    torch.manual_seed(1234)
    for step in range(4):  # eager, capture + replay, replay, replay
        gen = torch.cuda.get_rng_state()
        want = [None if i in skip else sel.get_indices(p, step) for i, p in enumerate(params)]
        after_ref = torch.cuda.get_rng_state()
        torch.cuda.set_rng_state(gen)
        mask.fill_(7)
        bits = torch.full((ops.sparta_mask_words(L.n),), -1, dtype=torch.int64, device=DEV)
        bits[-(-(L.offsets[-1] + L.numels[-1]) // 64):] = 0  # the arena's trailing words (zero from allocation)
        packed = draw_masks(sel, params, L.views(mask), skip, step, state, bits=bits if step % 2 else None)
        assert torch.equal(torch.cuda.get_rng_state(), after_ref), step
        if packed is not None:  # the fused draw wrote the packed words instead of the bytes
            assert mode == "fused"
            mask.copy_(torch.from_numpy(osparta.unpack_mask(packed.cpu().numpy(), L.n).astype(np.uint8)))
            pad = np.ones(L.n, bool)
            for o, nn in zip(L.offsets, L.numels):
                pad[o:o + nn] = False
            assert not mask.cpu().numpy()[pad].any()
        for i, v in enumerate(L.views(mask)):
            if i in skip:
                assert int(v.sum()) == 0
            else:
                assert torch.equal(v.bool(), want[i]), (step, i)
        torch.rand(5, device=DEV)  # other consumers of the generator between steps
    MaskDraw.fused, MaskDraw.use_graphs = saved
    assert (state.graph is not None) == (mode == "graph")


# p edges for the kernels' integer threshold (tb_threshold): none / every
# element, p = 2^-32 (only a zero word qualifies), p below 2^-32, the largest
# float below 1 (the top words round to a uniform of 1.0 and are not selected)
@pytest.mark.parametrize("numel,p", [(1, 0.5), (7, 0.3), (4096 * 3 + 2, 0.005), (2_000_003, 0.005), (100_000, 0.9),
                                     (4096 + 70, 0.0), (4096 + 70, 1.0), (50_000, 2.0 ** -32), (50_000, 1e-10),
                                     (300_001, 0.99999994)])
def test_torch_gpu_bernoulli_oracle_and_kernel(numel, p):
    """oracle.sparta.torch_gpu_bernoulli restates ATen's HIP bernoulli kernel
    (pinned here against torch.bernoulli(torch.full(...)) on this GPU), and
    ga_sparta_torch_bernoulli equals both, at a ragged numel and a tensor that
    starts inside the mask arena."""
    from gym_amd import ops
    gen = torch.cuda.default_generators[0]
    torch.manual_seed(777)
    torch.rand(3, device=DEV)  # a non-zero starting offset
    seed, off = gen.initial_seed(), gen.get_offset()
    want = torch.bernoulli(torch.full((numel,), p, device=DEV)).bool().cpu().numpy()
    assert gen.get_offset() == off + 12  # the offset step draw_masks assumes
    assert np.array_equal(osparta.torch_gpu_bernoulli(numel, p, seed, off), want)
    mask = torch.full((64 + numel + 64,), 9, dtype=torch.uint8, device=DEV)
    table, nb = ops.sparta_bernoulli_table([64], [numel], DEV)
    ops.sparta_torch_bernoulli(table, nb, p, seed, off, 12, mask)
    got = mask.cpu().numpy()
    assert np.array_equal(got[64:64 + numel] != 0, want) and set(np.unique(got[64:64 + numel])) <= {0, 1}
    assert (got[:64] == 9).all() and (got[64 + numel:] == 9).all()
    # packed output: the tensor's words (tail bits past numel zero); neighbours untouched
    words = ops.sparta_mask_words(64 + numel + 64)
    bits = torch.full((words,), -1, dtype=torch.int64, device=DEV)
    ops.sparta_torch_bernoulli(table, nb, p, seed, off, 12, bits)
    gb = bits.cpu().numpy()
    assert gb[0] == -1 and all(gb[w] == -1 for w in range(1 + -(-numel // 64), words))
    assert np.array_equal(gb[1:1 + -(-numel // 64)], osparta.pack_mask(want))


@pytest.mark.parametrize("layout,K,p", [("elem", 32, 0.05), ("rows", 3, 0.05), ("elem", 32, 0.3), ("elem", 8, 0.9)])
def test_sparta_in_kernel_reference_draw(layout, K, p):
    """GA_MASK_TORCH: the average kernel draws the reference's masks itself
    (draw_masks(defer=True) -> ops.TorchDraw) -- the same averages as with the
    fused draw's packed mask and the oracle's restatement of torch's stream,
    and the generator advanced identically; a grad-less tensor is skipped and
    tensor ends fall inside 64-element groups; p = 0.3 / 0.9 list several
    windows per wave tile."""
    from gym_amd import ops
    from gym_amd.arena import ArenaLayout
    from gym_amd.strategy.sparta import MaskDraw, RandomIndexSelector, draw_masks
    shapes = [(300, 77), (768,), (5, 9), (1000, 64), (3,)]
    L = ArenaLayout(shapes)
    params = [torch.zeros(s, device=DEV) for s in shapes]
    sel = RandomIndexSelector(p)
    skip = {2}
    rng = np.random.default_rng(K)
    x = rng.standard_normal((K, L.n)).astype(np.float32)
    mk = (lambda a: t(np.ascontiguousarray(a.T))) if layout == "elem" else t
    mask = torch.zeros(L.n, dtype=torch.uint8, device=DEV)
    outs, gens = [], []
    for defer in (False, True):
        torch.manual_seed(99)
        torch.rand(7, device=DEV)
        gen = torch.cuda.default_generators[0]
        seed, off0 = gen.initial_seed(), gen.get_offset()
        bits = torch.zeros(ops.sparta_mask_words(L.n), dtype=torch.int64, device=DEV)
        m = draw_masks(sel, params, L.views(mask), skip, 0, MaskDraw(), bits=bits, defer=defer)
        assert isinstance(m, ops.TorchDraw) == defer
        gens.append(torch.cuda.get_rng_state())
        src = mk(x)
        ops.sparta_average_local(src, L.n, float(K), mask=m, layout=layout)
        outs.append(host(src).T if layout == "elem" else host(src))
    assert torch.equal(gens[0], gens[1])
    # the oracle: torch's stream per drawn tensor, offset + 12 per tensor
    want_mask = np.zeros(L.n, bool)
    i = 0
    for j, (o, nn) in enumerate(zip(L.offsets, L.numels)):
        if j in skip:
            continue
        want_mask[o:o + nn] = osparta.torch_gpu_bernoulli(nn, p, seed, off0 + 12 * i)
        i += 1
    want = osparta.sparse_average(list(x), want_mask)
    for k in range(K):
        assert np.array_equal(outs[0][k], want[k]) and np.array_equal(outs[1][k], want[k]), k


def test_fused_draw_self_check():
    """The one-time probe draw_masks runs before using the fused draw agrees
    with this torch build (and leaves the caller's generator untouched)."""
    from gym_amd.strategy import sparta as sp
    sp._FUSED_OK.clear()
    torch.manual_seed(5)
    before = torch.cuda.get_rng_state()
    assert sp.fused_draw_matches_torch(DEV)
    assert torch.equal(torch.cuda.get_rng_state(), before)


@pytest.mark.parametrize("K,n,p,src_kind", [(32, 1_000_003, 0.005, "philox"), (4, 3 * 16384 + 77, 0.3, "philox"),
                                            (8, 2_000_000, 0.01, "torch"), (64, 16384 * 5, 0.6, "bits")])
def test_sparta_select_repeated_launches_overflow(K, n, p, src_kind):
    """The exchange path's select on an element-major set (count -> scan ->
    select) against the oracle, launched repeatedly on one workspace: the same
    packed index list, the same K-replica sums and count every launch, with a
    cap that overflows on the last launch (count[1] set, the list truncated)."""
    from gym_amd import ops
    rng = np.random.default_rng(K + n)
    x = rng.standard_normal((n, K)).astype(np.float32)  # [n, K] element-major
    src = t(x)
    seed = 0xABCDEF
    ws = None
    for it in range(3):
        if src_kind == "philox":
            m = osparta.philox_mask(n, seed, it, p)
            kw = dict(seed=seed, iteration=it, p=p)
        elif src_kind == "bits":
            m = rng.random(n) < p
            bits = torch.from_numpy(osparta.pack_mask(m).view(np.int64)).to(DEV)
            kw = dict(mask=bits)
        else:  # the in-kernel reference draw (GA_MASK_TORCH)
            L = __import__("gym_amd.arena", fromlist=["ArenaLayout"]).ArenaLayout([(n,)])
            table, nb = ops.sparta_bernoulli_table(L.offsets, L.numels, DEV)
            m = osparta.torch_gpu_bernoulli(n, p, 1234, 12 * it)
            kw = dict(mask=ops.TorchDraw(table, p, 1234, 12 * it, 12))
        want = np.flatnonzero(m)
        cap = len(want) + 16 if it < 2 else max(1, len(want) - 5)  # the last launch overflows
        if ws is None:
            ws = _sparta_buffers(n, len(want) + 4096)
        idx, count, work = ws
        vals = torch.empty(cap, device=DEV)
        ops.sparta_select(src, n, cap, idx, vals, count, work, layout="elem", **kw)
        c = host(count).astype(np.int64)
        assert c[0] == len(want) and c[1] == int(len(want) > cap), (it, c, len(want))
        k = min(cap, len(want))
        assert np.array_equal(idx.cpu().numpy()[:k], want[:k]), it
        sums = oreduce.mean_reduce(list(x[want[:k]].T), divisor=1)
        assert np.array_equal(host(vals)[:k], sums), it


@pytest.mark.parametrize("K,n,p,src_kind,dtype", [(32, 1_000_003, 0.005, "philox", "f32"),
                                                  (40, 3 * 4096 + 77, 0.3, "philox", "f32"),
                                                  (5, 200_000, 0.02, "bits", "bf16"),
                                                  (128, 4096 * 9, 0.9, "bits", "f32"),
                                                  (8, 2_000_000, 0.01, "torch", "f32"),
                                                  (1, 70_001, 0.05, "philox", "f32")])
def test_sparta_rows_local_average(K, n, p, src_kind, dtype):
    """The replica loop's [K, ld] rows local average (the wave form: one lane
    per listed element, every replica's word in flight) against the oracle:
    bit-identical replicas, dense tiles (several list windows, more than 64
    elements per batch), K > 32 (several load batches), bf16, each mask source."""
    from gym_amd import ops
    rng = np.random.default_rng(K + n)
    ld = n + 61
    x = np.zeros((K, ld), np.float32)
    x[:, :n] = rng.standard_normal((K, n))
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    if src_kind == "philox":
        m = osparta.philox_mask(n, 0xABC, 5, p)
        kw = dict(seed=0xABC, iteration=5, p=p)
    elif src_kind == "bits":
        m = rng.random(n) < p
        kw = dict(mask=torch.from_numpy(osparta.pack_mask(m).view(np.int64)).to(DEV))
    else:
        L = __import__("gym_amd.arena", fromlist=["ArenaLayout"]).ArenaLayout([(n,)])
        table, _ = ops.sparta_bernoulli_table(L.offsets, L.numels, DEV)
        m = osparta.torch_gpu_bernoulli(n, p, 1234, 24)
        kw = dict(mask=ops.TorchDraw(table, p, 1234, 24, 12))
    src = torch.from_numpy(x).to(DEV).to(tdt)
    ops.sparta_average_local(src, n, float(K), layout="rows", **kw)
    got = {"1": src.float().cpu().numpy()}
    if dtype == "f32":
        want = osparta.sparse_average(list(x[:, :n]), m)
        for k in range(K):
            assert np.array_equal(got["1"][k, :n], want[k])
    else:  # bf16: the fp32 sums of the bf16 inputs, rounded once
        xb = torch.from_numpy(x).to(tdt).float().numpy()
        want = osparta.sparse_average(list(xb[:, :n]), m)
        w = torch.from_numpy(np.stack(want)).to(tdt).float().numpy()
        assert np.array_equal(got["1"][:, :n], w)
    assert (got["1"][:, n:] == 0).all()


class _LoopColl:
    """A world-1 'exchange' without a process group (collectives are identities):
    the Sparta engine takes its multi-rank select -> all-reduce -> scatter path."""
    world, rank, backend, exchange, rccl = 1, 0, "loop", True, False

    def all_reduce_(self, t, async_op=False):
        return t

    def broadcast_(self, t, src=0):
        return t


def test_sparta_engine_overflow_raised_two_steps_later():
    """The exchange path's overflow flag is read back without a host wait in
    the step: a step polls only the flag of the step before the previous one,
    so an overflow raises two steps later, and check() raises at once."""
    from gym_amd.engine import Sparta
    n, K, p = 100_000, 2, 0.3
    reps = torch.randn(K, n, device=DEV)

    def small(eng):
        eng.cap = 8
        eng.idx = torch.empty(8, dtype=torch.int32, device=DEV)
        eng.vals = torch.empty(8, device=DEV)

    eng = Sparta(_LoopColl(), K, n, DEV, torch.float32, p)
    small(eng)
    eng(reps, seed=1, iteration=0)  # overflows
    eng(reps, seed=1, iteration=1)  # step 0's flag still pending
    with pytest.raises(RuntimeError, match="capacity"):
        eng(reps, seed=1, iteration=2)
    eng2 = Sparta(_LoopColl(), K, n, DEV, torch.float32, p)
    small(eng2)
    eng2(reps, seed=1, iteration=0)
    with pytest.raises(RuntimeError, match="capacity"):
        eng2.check()
    ok = Sparta(_LoopColl(), K, n, DEV, torch.float32, 0.001)
    for it in range(4):
        ok(reps, seed=1, iteration=it)
    ok.check()


def test_empty_inputs_every_kernel():
    """n = 0 through every entry point on the device: nothing launched or an
    empty launch, no error, counts written as zero, buffers untouched."""
    from gym_amd import ops
    K = 3
    reps = torch.full((K, 64), 5.0, device=DEV)
    master, mom = torch.full((64,), 2.0, device=DEV), torch.zeros(64, device=DEV)
    ops.replica_mean(reps, reps, n=0)
    ops.diloco_outer(reps, master, mom, reps, 0, float(K), 0.7, 0.9, 0.0, 0.0, True, True)
    cap = 16
    idx = torch.full((cap,), -1, dtype=torch.int32, device=DEV)
    vals = torch.full((cap,), 9.0, device=DEV)
    count = torch.full((2,), 7, dtype=torch.int64, device=DEV)
    work = ops.sparta_workspace(1, DEV)
    ops.sparta_select(reps, 0, cap, idx, vals, count, work, seed=1, iteration=0, p=0.5)
    assert host(count).tolist() == [0, 0]
    ops.sparta_scatter(vals, idx, count, cap, float(K), reps)
    ops.sparta_average_local(reps, 0, float(K), seed=1, iteration=0, p=0.5)
    g = torch.zeros_like(reps)
    ops.adam_step(reps, g, torch.zeros_like(reps), torch.zeros_like(reps), 0.1, 0.999, 0.001, 1e-8, 1.0, 0.0,
                  -1e-3, 1.0, n=0)
    torch.cuda.synchronize()
    assert (host(reps) == 5.0).all() and (host(master) == 2.0).all() and (host(vals) == 9.0).all()
    assert (host(idx) == -1).all()


def test_demo_optimizer_bf16_transform_option():
    """DeMo(bf16_transform=...) on bf16 parameters picks the plan (reference:
    the GA_BF16_REF block kernels) and steps; fp32 parameters ignore it;
    a bad value is rejected."""
    from gym_amd.strategy.demo_impl.demo import DeMo
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(128, 64), torch.nn.Linear(64, 32)).to(DEV).to(torch.bfloat16)
    opt = DeMo(m.parameters(), lr=1e-3, compression_topk=8, bf16_transform="reference", placement=False)
    assert opt.codec.plan.bf16_reference and not opt.codec.plan.wave_encode
    for _ in range(2):
        opt.zero_grad()
        m(torch.randn(16, 128, device=DEV, dtype=torch.bfloat16)).float().square().mean().backward()
        opt.step()
    assert all(torch.isfinite(p.float()).all() for p in m.parameters())
    f = torch.nn.Linear(64, 64).to(DEV)
    assert not DeMo(f.parameters(), bf16_transform="reference").codec.plan.bf16_reference
    with pytest.raises(ValueError):
        DeMo(f.parameters(), bf16_transform="bf8")


def test_demo_bf16_reference_decode_three_hitters():
    """GA_BF16_REF decode with 3 and 4 nodes sending IDENTICAL payloads, so every
    selected position has 3-4 hitters: the scatter-mean's running sum is rounded
    to bf16 after every add (torch's bf16 scatter_reduce), then divided --
    parameters and signs bit-identical to the reference's op sequence as torch
    runs it on this GPU (oracle/demo_bf16.py, device cuda; identical values make
    torch's atomic add order irrelevant)."""
    from gym_amd import ops
    from gym_amd.arena import ArenaLayout
    from gym_amd.demo_codec import DemoPlan
    from oracle import demo_bf16 as ob
    shapes = [(128, 64), (64,)]
    L = ArenaLayout(shapes)
    plan = DemoPlan(L, chunk=64, topk=8, bf16_transform="reference")
    g = torch.Generator().manual_seed(11)
    p = [torch.randn(*s, generator=g) * 0.02 for s in shapes]
    d = [torch.randn(*s, generator=g) * 1e-3 for s in shapes]
    gr = [torch.randn(*s, generator=g) * 1e-2 for s in shapes]
    lr, decay = 1e-3, 0.999
    for K in (3, 4):
        P, D, G = (torch.zeros(K, L.n, device=DEV, dtype=torch.bfloat16) for _ in range(3))
        for i in range(len(shapes)):
            for k in range(K):
                L.views(P[k])[i].copy_(p[i].to(torch.bfloat16))
                L.views(D[k])[i].copy_(d[i].to(torch.bfloat16))
                L.views(G[k])[i].copy_(gr[i].to(torch.bfloat16))
        payload = torch.zeros(K, 2 * plan.M, dtype=torch.int32, device=DEV)
        ops.demo_encode(plan, P, G, D, payload, lr, decay, 1.0)
        assert all(torch.equal(payload[0], payload[k]) for k in range(K))  # every node sends the same
        ops.demo_decode(plan, payload, P, G, lr)
        for i, s in enumerate(shapes):
            bf = lambda x: x.to(torch.bfloat16).float().numpy()  # noqa: E731
            rp, rd, rs = ob.demo_step(bf(p[i]), [bf(d[i])] * K, [bf(gr[i])] * K, lr, decay, 8, 64, 0.0, device=DEV)
            assert np.array_equal(host(L.views(G[0])[i]), rs), (K, i)
            assert np.array_equal(host(L.views(P[0])[i]), rp), (K, i)
