"""Assertions shared by the CPU (oracle stand-in) and GPU (real kernel) runs of
tests/strategy_scenarios.py: every rank's final state against the reference's
golden fixtures or the oracle."""
import os
import random

import numpy as np

from oracle import demo as odemo
from oracle import reduce as oreduce
from oracle import sparta as osparta


def check_simple(res, world, golden_dir):
    z = np.load(os.path.join(golden_dir, "mean_reduce.npz"))
    for r in range(world):
        for si in range(4):
            got, ref = res[r][f"grad_{si}"], z[f"K{world}_out_{si}"]
            if world == 2:
                assert np.array_equal(got, ref)
            else:
                np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-7)


def check_diloco(res, world, golden_dir):
    z = np.load(os.path.join(golden_dir, "diloco.npz"))
    ns, calls = int(z["nshapes"]), int(z["calls"])
    for call in range(calls):
        for i in range(ns):
            for r in range(world):
                # no chaining here: three outer steps run end to end on our state
                np.testing.assert_allclose(res[r][f"after_{call}_{i}"], z[f"after_{call}_{i}"][r], rtol=2e-6,
                                           atol=2e-8)


def check_sparta(res, world, golden_dir):
    z = np.load(os.path.join(golden_dir, "sparta.npz"))
    ns, calls = int(z["nshapes"]), int(z["calls"])
    for call in range(calls):
        for i in range(ns):
            for r in range(world):
                got, ref = res[r][f"after_{call}_{i}"], z[f"K{world}_after_{call}_{i}"][r]
                if world == 2:
                    assert np.array_equal(got, ref)
                else:
                    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-9)


def check_sparta_philox(res, world, golden_dir):
    seed = int(res[0]["seed"])
    n = int(res[0]["n"])
    assert all(int(res[r]["seed"]) == seed for r in range(world))  # rank 0's seed everywhere
    reps = [res[r]["before"] for r in range(world)]
    for it in (0, 1):
        reps = osparta.sparse_average(reps, osparta.philox_mask(n, seed, it, 0.05))
    for r in range(world):
        np.testing.assert_array_equal(res[r]["after"], reps[r]) if world == 2 else \
            np.testing.assert_allclose(res[r]["after"], reps[r], rtol=1e-6, atol=1e-9)


def _torch_masks(kind, device, steps):
    """Rank 0's masks for `steps` calls, re-derived from the generator calls the
    reference selectors make (sparta.py:80-85, :95-136, :146-193) on `device`
    after torch.manual_seed(42), through the oracle's restatements (the draws
    are inputs, as torch's randperm/argsort order is the generator's)."""
    import torch
    import strategy_scenarios as S
    p = S.SEL_P[kind]
    live = [i for i in range(len(S.SEL_SHAPES)) if i != S.SEL_FROZEN]
    numel = {i: int(np.prod(S.SEL_SHAPES[i])) for i in live}
    torch.manual_seed(42)
    masks, perms, orders, calls = [], {}, {i: [] for i in live}, 0
    for it in range(steps):
        m = {}
        for i in live:
            if kind == "random":
                m[i] = torch.bernoulli(torch.full(S.SEL_SHAPES[i], p, device=device)).bool().cpu().numpy().reshape(-1)
            elif kind == "shuffled":
                if i not in perms:
                    perms[i] = torch.randperm(numel[i], device=device).cpu().numpy()
                m[i] = osparta.shuffled_sequential_mask(numel[i], p, perms[i], it)
            else:  # partitioned: a new argsort at the first call and after each full cycle
                nparts = max(1, min(int(np.ceil(1.0 / p)), numel[i]))
                if it % nparts == 0:
                    orders[i].append(torch.rand(numel[i], device=device).argsort().cpu().numpy())
                m[i] = osparta.partitioned_masks(numel[i], p, orders[i], it + 1)[-1]
        masks.append(m)
    return masks


def check_sparta_sel(res, world, golden_dir, kind="random", device="cpu", rank_seeds=False):
    import strategy_scenarios as S
    nt = len(S.SEL_SHAPES)
    # the draw that ran, as the strategy's __config__ records it (no silent fallback)
    want_draw = "philox" if kind == "philox" else ("fused" if kind == "random" and device != "cpu" else "torch")
    for r in range(world):
        assert str(res[r]["mask_draw_0"]) == want_draw, (r, str(res[r]["mask_draw_0"]), want_draw)
    if kind == "random" and "gen_0" in res[0]:  # every rank's generator advanced by its own draws
        draws = S.SEL_STEPS * (nt - 1)
        for r in range(world):
            seed, off = (int(v) for v in res[r]["gen_0"])
            assert seed == 42 + (r if rank_seeds else 0) and off == 12 * draws, (r, seed, off)
    if kind == "philox":
        seed = int(res[0]["seed_0"])
        offs = res[0]["offsets_0"]
        n_tot = int(offs[-1]) + int(np.prod(S.SEL_SHAPES[-1]))
        skip = [(int(offs[S.SEL_FROZEN]), int(offs[S.SEL_FROZEN]) + int(np.prod(S.SEL_SHAPES[S.SEL_FROZEN])))]
        masks = []
        for it in range(S.SEL_STEPS):
            full = osparta.philox_mask(n_tot, seed, it, S.SEL_P[kind], skip=skip)
            masks.append({i: full[int(offs[i]):int(offs[i]) + int(np.prod(S.SEL_SHAPES[i]))]
                          for i in range(nt) if i != S.SEL_FROZEN})
    else:
        masks = _torch_masks(kind, device, S.SEL_STEPS)
    for step in range(S.SEL_STEPS):
        for i in range(nt):
            before = [res[r][f"before_{step}_{i}"] for r in range(world)]
            if i == S.SEL_FROZEN:
                want = before
            else:
                assert masks[step][i].any() or kind in ("random", "philox")
                want = osparta.sparse_average(before, masks[step][i].reshape(S.SEL_SHAPES[i]))
            for r in range(world):
                got = res[r][f"after_{step}_{i}"]
                if world == 2:
                    assert np.array_equal(got, want[r]), f"{kind} step {step} tensor {i} rank {r}"
                else:
                    np.testing.assert_allclose(got, want[r], rtol=1e-6, atol=1e-9)


def check_eval_avg(res, world, golden_dir):
    for i in range(3):
        own = [res[r][f"own_{i}"] for r in range(world)]
        want = oreduce.mean_reduce(own)
        for r in range(world):
            assert np.array_equal(res[r][f"after_{i}"], own[r])  # the node's model is not touched
            if world == 2:
                assert np.array_equal(res[r][f"avg_{i}"], want)
            else:  # gloo's ring order: a few ulp of the summands where they cancel
                scale = max(np.abs(x).max() for x in own)
                np.testing.assert_allclose(res[r][f"avg_{i}"], want, rtol=1e-6, atol=1e-7 * scale)


def check_mnist_diloco(res, world, golden_dir):
    """Each outer step = oracle.diloco.outer_step over the nodes' parameters as
    they entered it (master chained from the shared start, momentum from the
    previous outer step); every node leaves it holding the new master."""
    from oracle import diloco as odiloco
    n = res[0]["pre_0"].size
    master = res[0]["init"][:n].copy()
    assert all(np.array_equal(res[r]["init"], res[0]["init"]) for r in range(world))
    mom = None
    outer = 0
    for t in range(5):
        if t % 2 == 0 and t > 0:  # the gate sees local_step = t before its increment (diloco.py:62)
            pre = [res[r][f"pre_{outer}"] for r in range(world)]
            assert not np.array_equal(pre[0], pre[1])  # the nodes trained on different data
            master, mom, _ = odiloco.outer_step(master, mom, pre)
            for r in range(world):
                got = res[r][f"after_{t}"][:n]
                np.testing.assert_allclose(got, master, rtol=1e-6, atol=1e-9)
            outer += 1
    assert outer == 2


def check_fedavg(res, world, golden_dir, island_size=None, max_groups=None):
    """Averaging steps (rank 0's island draws from random.seed(1234)): every
    node ends at the ascending-rank fp32 mean of its island, bit-exact (the
    reference's sum(island_tensors) / len, federated_averaging.py:61-69),
    whether the round ran in cached island sub-communicators or in the world
    all-gather; the sub-communicator cache stays within its bound."""
    nt = 3
    rounds = int(res[0]["rounds"])
    if max_groups is not None:
        for r in range(world):
            assert int(res[r]["ngroups"].max()) <= max_groups, res[r]["ngroups"]
    state = [[res[r][f"before_{i}"] for i in range(nt)] for r in range(world)]
    for r in range(world):
        for i in range(nt):
            assert np.array_equal(res[r][f"after0_{i}"], state[r][i])  # local_step 0: no averaging
    rng = random.Random(1234)
    for step in range(1, rounds + 1):
        if island_size is None or island_size >= world:
            islands = [set(range(world))]
        else:
            ranks = list(range(world))
            rng.shuffle(ranks)
            islands = [set(ranks[j:j + island_size]) for j in range(0, world, island_size)]
        new = []
        for r in range(world):
            isl = next(s for s in islands if r in s)
            new.append([oreduce.mean_reduce([state[m][i] for m in sorted(isl)]) for i in range(nt)])
            for i in range(nt):
                got = res[r][f"after{step}_{i}"]
                if island_size is None or island_size >= world:
                    np.testing.assert_allclose(got, new[r][i], rtol=1e-6, atol=1e-9)  # all-reduce order
                else:
                    assert np.array_equal(got, new[r][i]), (step, r, i)
        state = [[res[r][f"after{step}_{i}"] for i in range(nt)] for r in range(world)]


def check_demo(res, world, golden_dir):
    import demo_checks
    z = np.load(os.path.join(golden_dir, "demo_steps.npz"))
    ns, steps = int(z["nshapes"]), int(z["steps"])
    lr = float(z["lr"])
    tally = demo_checks.SignTally()
    for step in range(steps):
        assert int(res[0][f"tx_{step}"]) == int(z[f"tx_{step}"])
        assert int(res[0][f"rx_{step}"]) == int(z[f"rx_{step}"])
        for i in range(ns):
            ref_s = z[f"sign_{step}_{i}"]
            _, _, _, _, g_hat, margins = odemo.demo_step(
                z[f"p_before_{step}_{i}"], list(z[f"delta_before_{step}_{i}"]), list(z[f"grad_{step}_{i}"]), lr,
                float(z["decay"]), int(z["topk"]), int(z["chunk"]), float(z["wd"]), detail=True)
            firm = demo_checks.firm(g_hat, margins, ref_s.shape, int(z["chunk"]))
            for r in range(world):
                s = res[r][f"sign_{step}_{i}"]
                tally.check(s, ref_s, firm, what=f"rank {r} step {step} tensor {i}")
                ok = s == ref_s
                np.testing.assert_allclose(res[r][f"p_{step}_{i}"][ok], z[f"p_after_{step}_{i}"][ok], rtol=0,
                                           atol=1e-6)
                assert np.array_equal(res[r][f"p_{step}_{i}"], res[0][f"p_{step}_{i}"])  # nodes stay in sync
                ref_d = z[f"delta_after_{step}_{i}"][r]
                scale = max(np.abs(ref_d).max(), lr * np.abs(z[f"grad_{step}_{i}"][r]).max())
                np.testing.assert_allclose(res[r][f"delta_{step}_{i}"], ref_d, rtol=0, atol=2e-5 * scale)
    tally.done()


def check_demo_pipe(res, world, golden_dir, **_):
    """The pipelined codec ends exactly where the one-exchange codec ends
    (params, signs, residual deltas) on every rank, in more than one piece."""
    for r in range(world):
        assert int(res[r]["pipe_pieces"]) > 1
        for what in ("p", "g", "d"):
            assert np.array_equal(res[r][f"pipe_pipe_{what}"], res[r][f"pipe_plain_{what}"]), (r, what)


def check_engine(res, world, golden_dir, K_local=3, **_):
    """Every node of every rank ends equal to the oracle over all K_total nodes
    (reordered fp32 sums: RCCL/gloo ring order, 1e-6 relative)."""
    import strategy_scenarios as S
    from oracle import diloco as odiloco
    from oracle import reduce as oreduce
    KT = world * K_local
    n = world * 64 * 10
    x = [S.engine_node(j, n) for j in range(KT)]
    m1, b1, _ = odiloco.outer_step(S.engine_node(0, n), None, x)
    x2 = [m1 + S.engine_node(j, n, salt=1) * np.float32(0.05) for j in range(KT)]
    m2, _, _ = odiloco.outer_step(m1, b1, x2)
    avg = oreduce.mean_reduce([S.engine_node(j, n, salt=2) for j in range(KT)])
    for r in range(world):
        for k in range(K_local):
            np.testing.assert_allclose(res[r]["d1"][k], m1, rtol=1e-6, atol=2e-8)
            np.testing.assert_allclose(res[r]["d2"][k], m2, rtol=1e-6, atol=2e-8)
            np.testing.assert_allclose(res[r]["m_shard"][k], avg, rtol=1e-6, atol=2e-8)
            np.testing.assert_allclose(res[r]["m_plain"][k], avg, rtol=1e-6, atol=2e-8)
    if "sparta" in res[0]:  # forced-exchange run (world 1): exact orders, bit-exact
        x3 = [S.engine_node(j, n, salt=3) for j in range(KT)]
        want = osparta.sparse_average(x3, osparta.philox_mask(n, 77, 5, 0.05))
        for k in range(KT):
            assert np.array_equal(res[0]["sparta"][k], want[k])
        import demo_checks
        from gym_amd.arena import ArenaLayout
        L = ArenaLayout([(128, 128), (768,)])
        g = res[0]["demo_g"]
        tally = demo_checks.SignTally()
        for shape, off, m in zip(L.shapes, L.offsets, L.numels):
            grads = [g[k, off:off + m].reshape(shape) for k in range(KT)]
            zeros = [np.zeros(shape, np.float32)] * KT
            want_p, _, want_s, _, g_hat, margins = odemo.demo_step(zeros[0], zeros, grads, 0.01, detail=True)
            for k in range(KT):
                tally.check(res[0]["demo_sign"][k, off:off + m].reshape(shape), want_s,
                            demo_checks.firm(g_hat, margins, shape), what=f"demo {shape} node {k}")
                ok = res[0]["demo_sign"][k, off:off + m].reshape(shape) == want_s
                np.testing.assert_allclose(res[0]["demo_p"][k, off:off + m].reshape(shape)[ok], want_p[ok],
                                           rtol=0, atol=1e-7)
        tally.done()
        check_demo_pipe(res, 1, golden_dir)


def check_simple_adamw(res, world, golden_dir, steps=3):
    """torch's own pipeline on CPU: mean of the nodes' grads (true division),
    clip_grad_norm_(0.5), AdamW(lr=3e-3, wd=0.05)."""
    import torch
    import strategy_scenarios as S
    model = S.ShapeModel(S.ADAMW_SHAPES, seed=11)
    opt = torch.optim.AdamW(model.parameters(), lr=3e-3, weight_decay=0.05)
    for step in range(steps):
        per = [S._adamw_grads(r, step, S.ADAMW_SHAPES) for r in range(world)]
        for i, p in enumerate(model.parameters()):
            acc = per[0][i].clone()
            for r in range(1, world):
                acc += per[r][i]
            p.grad = acc / world
        torch.nn.utils.clip_grad_norm_(model.parameters(), 0.5)
        opt.step()
    for r in range(world):
        assert bool(res[r]["fused"]), "the default AdamW should run fused on the arena"
        for i, p in enumerate(model.parameters()):
            np.testing.assert_allclose(res[r][f"p_{i}"], p.detach().numpy(), rtol=1e-5, atol=1e-7)


CHECKS = {"simple_adamw": check_simple_adamw, "engine": check_engine, "simple": check_simple, "diloco": check_diloco, "sparta": check_sparta,
          "sparta_philox": check_sparta_philox, "sparta_sel": check_sparta_sel,
          "eval_avg": check_eval_avg, "mnist_diloco": check_mnist_diloco, "fedavg": check_fedavg, "demo": check_demo,
          "demo_pipe": check_demo_pipe}
