"""Inner optimizer on the flat arena.

The reference's strategies run `clip_grad_norm_(model.parameters(), max_norm)`
and `self.optim.step()` with the default inner optimizer torch.optim.AdamW
(exogym/strategy/strategy.py:135-140, diloco.py:52-59,
communicate_optimize_strategy.py:69-74; OptimSpec default optim.py:11).
ArenaAdam is a torch.optim.Optimizer (schedulers such as LambdaLR drive its
param_groups[0]["lr"] as usual) whose step() is ONE fused kernel over the
node's parameter arena (ga_adam_step: read p, g, m, v; write p, m, v) and,
with clipping, one norm reduction (ga_grad_clip_coef) whose coefficient the
step kernel applies on the device -- no host synchronisation.

Exactness: parameters whose .grad is None at step time are skipped, as torch
does (the kernel runs over the contiguous arena ranges that have gradients).
The per-parameter state (exp_avg, exp_avg_sq, step) are views of the flat
state buffers, so state_dict() has torch's layout, and load_state_dict()
(of an ArenaAdam or a torch.optim.Adam/AdamW state dict) copies the loaded
moments into those buffers, so a resumed run continues where it stopped.
"""
import math
import time

import torch

from . import ops

_UNSUPPORTED = ("amsgrad", "maximize", "capturable", "differentiable")

# physical placement of the moments (gym_amd.placement), chosen on the first step
PLACEMENT_CANDIDATES = 48
PLACEMENT_MAX_FRAC = 0.3
PLACEMENT_MIN_BYTES = 32 << 20
# K > 1 replicas: each replica's moments are placed on their own (probed against that
# replica's parameter / gradient rows), with fewer candidates per replica and a budget:
# a replica's search stops after ROW_PATIENCE candidates unless the best beats its
# ordinary rows by > 2%, and the whole search stops at PLACEMENT_ROW_BUDGET_S
PLACEMENT_ROW_CANDIDATES = 16
PLACEMENT_ROW_PATIENCE = 3
PLACEMENT_ROW_BUDGET_S = 0.25


def fusable(spec_cls, kwargs, arena):
    """True when OptimSpec(spec_cls, **kwargs) can run as ArenaAdam on this arena."""
    if spec_cls not in (torch.optim.AdamW, torch.optim.Adam):
        return False
    grads = getattr(arena, "grad_set", None) if hasattr(arena, "grad_set") else getattr(arena, "grad_flat", None)
    if arena is None or grads is None or arena.dtype != torch.float32:
        return False
    kw = dict(kwargs or {})
    if any(kw.get(k) for k in _UNSUPPORTED):
        return False
    if spec_cls is torch.optim.Adam and kw.get("decoupled_weight_decay"):
        return False
    allowed = {"lr", "betas", "eps", "weight_decay", "foreach", "fused"} | set(_UNSUPPORTED)
    if set(kw) - allowed:
        return False
    lr = kw.get("lr", 1e-3)
    return not isinstance(lr, torch.Tensor)


def place_moment_rows(P, G, Mr, Vr, max_candidates=None, max_frac=None, patience=None, budget_s=None):
    """Per-replica placement of Adam moments (ArenaAdam, K > 1): for each
    replica k, fresh allocations of its two moment rows are timed with
    ga_probe_adam_placement against P[k], G[k] (values unchanged) beside Mr[k],
    Vr[k] where they are; the fastest keeps them.  Budget: up to max_candidates
    per replica, stopping after `patience` unless the best beats the rows' own
    time by > 2% (placement.choose), and the whole search ends by budget_s (each
    replica gets an equal share of what is left).  Rows not moved stay where
    they were probed (views of the caller's buffers).  Returns (new rows M, new
    rows V, per replica the chosen buffer or None, the record)."""
    from . import placement
    max_candidates = PLACEMENT_ROW_CANDIDATES if max_candidates is None else max_candidates
    max_frac = PLACEMENT_MAX_FRAC if max_frac is None else max_frac
    patience = PLACEMENT_ROW_PATIENCE if patience is None else patience
    budget_s = PLACEMENT_ROW_BUDGET_S if budget_s is None else budget_s
    watch = placement.Stopwatch()
    t_end = watch.t0 + budget_s
    K, ld = P.shape[0], Mr[0].numel()
    bufs, probe_ms, chosen = [], [], []
    for k in range(K):
        Pk, Gk = P[k, :ld], G[k, :ld]

        def probe(M, V):
            return placement.time_probe(lambda: ops.probe_adam_placement(Pk, Gk, M, V), reps=2)

        def split(buf):
            t = buf.tensor()
            return t[:ld], t[ld:2 * ld]

        now = time.perf_counter()
        deadline = now + max(0.0, t_end - now) / (K - k)
        best, times = placement.choose(2 * ld * 4, P.device, lambda b: probe(*split(b)), probe(Mr[k], Vr[k]),
                                       max_candidates, max_frac, patience=patience, deadline=deadline)
        bufs.append(best)
        probe_ms.append([round(t, 4) for t in times])
        chosen.append(min(range(len(times)), key=lambda i: times[i]) if best is not None else 0)
    outM, outV = [], []
    for k, b in enumerate(bufs):
        if b is None:  # kept where they were probed
            m, v = Mr[k], Vr[k]
        else:
            t = b.tensor()
            m, v = t[:ld], t[ld:2 * ld]
            m.copy_(Mr[k])
            v.copy_(Vr[k])
        outM.append(m)
        outV.append(v)
    rec = {"per_replica": True, "candidates_per_replica": max_candidates, "patience": patience,
           "budget_s": budget_s, "candidates_probed": sum(len(t) - 1 for t in probe_ms), "chosen": chosen,
           "placed_rows": sum(b is not None for b in bufs),
           "probe_ms_ordinary_sum": round(sum(t[0] for t in probe_ms), 4),
           "probe_ms_chosen_sum": round(sum(min(t) for t in probe_ms), 4), "probe_ms": probe_ms}
    return outM, outV, bufs, watch.stamp(rec)


class ArenaAdam(torch.optim.Optimizer):
    """Adam/AdamW over one node's ParamArena, or over a ReplicaArena (K nodes of
    one process, [K, ld] parameter/gradient sets: one launch for all of them,
    each replica clipped by its own gradient norm)."""

    def __init__(self, params, arena, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=None, decoupled=True,
                 placement=True, **ignored):
        if weight_decay is None:
            weight_decay = 1e-2 if decoupled else 0.0  # torch's AdamW / Adam defaults
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        for i, b in enumerate(betas):
            if not 0.0 <= b < 1.0:
                raise ValueError(f"Invalid beta parameter at index {i}: {b}")
        if not 0.0 <= weight_decay:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=None, capturable=False, differentiable=False, fused=None,
                        decoupled_weight_decay=bool(decoupled))
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("ArenaAdam: one parameter group (the node's arena)")
        self.arenas = list(getattr(arena, "arenas", [arena]))
        self._arena = arena  # P and G are read from it at every use: the sets may be relocated
        self.K, self.ld = self.P.shape
        dev = self.P.device
        self._M = torch.zeros_like(self.P, dtype=torch.float32)
        self._V = torch.zeros_like(self.P, dtype=torch.float32)
        # per replica [ld] rows of the moments: views of _M / _V, or (after a per-replica
        # placement) each in its own candidate buffer, when _M / _V are None
        self._Mr, self._Vr = list(self._M.unbind(0)), list(self._V.unbind(0))
        self.exp_avg, self.exp_avg_sq = self._M.view(-1), self._V.view(-1)  # flat views (single-arena users)
        self._step_t = torch.tensor(0.0)
        where = {}
        for k, ar in enumerate(self.arenas):
            for i, p in enumerate(ar.params):
                where[id(p)] = (k, ar.layout.offsets[i], ar.layout.numels[i])
        self._spans = [[] for _ in self.arenas]  # per replica: (param, offset, numel) in arena order
        self._where = where
        for p in self.param_groups[0]["params"]:
            if id(p) not in where:
                raise ValueError("ArenaAdam: every parameter must live in the arena")
            k, o, n = where[id(p)]
            self._spans[k].append((p, o, n))
            self._bind_state(p)
        for sp in self._spans:
            sp.sort(key=lambda t: t[1])
        self._partials = ops.sumsq_partials(dev, self.K)
        self._clip = torch.ones(2 * self.K, dtype=torch.float32, device=dev)
        self._placed = None  # the candidate buffer holding M and V once _place chose one
        self._placed_for = None  # (P, G) data pointers the moments were placed against
        self._placements = 0  # searches run (a relocated P / G set is searched again)
        self.placement = None  # the placement record (probe times, or why it was skipped)
        self.place_opt = placement  # False: never probe / move the moments (gym_amd.placement.policy)

    @property
    def P(self):
        """The parameter set [K, ld] (the replica arena's rows, or the node's arena as one row)."""
        a = self._arena
        return a.flat_set if hasattr(a, "flat_set") else a.flat.view(1, -1)

    @property
    def G(self):
        """The gradient set, read from the arena like P."""
        a = self._arena
        return a.grad_set if hasattr(a, "grad_set") else a.grad_flat.view(1, -1)

    @property
    def M(self):
        """exp_avg as [K, ld] (a stacked copy once the rows were placed apart)."""
        return self._M if self._M is not None else torch.stack(self._Mr)

    @property
    def V(self):
        return self._V if self._V is not None else torch.stack(self._Vr)

    def _bind_state(self, p):
        k, o, n = self._where[id(p)]
        self.state[p] = {"step": self._step_t, "exp_avg": self._Mr[k][o:o + n].view(p.shape),
                         "exp_avg_sq": self._Vr[k][o:o + n].view(p.shape)}

    def load_state_dict(self, state_dict):
        """torch's Optimizer.load_state_dict, then the loaded per-parameter
        moments are copied into the flat state buffers the kernel reads and the
        state is re-pointed at those views.  The kernel keeps one step count
        for the arena, so every parameter must carry the same `step`."""
        super().load_state_dict(state_dict)
        steps = set()
        with torch.no_grad():
            for r in self._Mr + self._Vr:
                r.zero_()
            for p in self.param_groups[0]["params"]:
                st = self.state.get(p, {})
                k, o, n = self._where[id(p)]
                if "exp_avg" in st:
                    self._Mr[k][o:o + n].copy_(st["exp_avg"].reshape(-1))
                    self._Vr[k][o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                if "step" in st:
                    steps.add(float(st["step"]))
        if len(steps) > 1:
            raise ValueError(f"ArenaAdam: parameters carry different step counts {sorted(steps)}; "
                             "the fused step keeps one count per arena")
        self._step_t = torch.tensor(steps.pop() if steps else 0.0)
        for p in self.param_groups[0]["params"]:
            self._bind_state(p)

    def _place(self):
        """Choose the physical memory of the moments, once, before the first
        step: the fused step's rate depends on where exp_avg / exp_avg_sq sit
        physically relative to the parameters and gradients (0.553-0.625 ms at
        GPT-2 124M, profiles/r04k_adam_placement.txt; gym_amd.placement), so
        fresh device allocations are timed with ga_probe_adam_placement (the
        step's access pattern, values unchanged) beside the ordinary ones and
        the fastest keeps the moments.  One replica (K = 1): up to
        PLACEMENT_CANDIDATES buffers for both moments.  K > 1: replica by
        replica, up to PLACEMENT_ROW_CANDIDATES buffers of one replica's two
        moment rows each, probed against that replica's parameter / gradient
        rows (the kernel's replica-major grid streams one replica's four rows
        at a time; a [K, ld] candidate at K = 32 x 124M would be 32 GB, so the
        memory budget would leave no choice); the step then runs one launch
        per replica.  When the parameter / gradient set is later moved (the
        outer step's own placement relocates the replica set at step H), the
        search runs again against the new rows, so the moments' placement
        always describes the step that runs."""
        self._placed_for = (self.P.data_ptr(), self.G.data_ptr())
        self._placements += 1
        nb = 2 * self.K * self.ld * 4
        if (self.P.device.type != "cuda" or nb < PLACEMENT_MIN_BYTES or PLACEMENT_CANDIDATES < 2
                or self.ld % 4 or self.P.stride(-1) != 1):
            return
        from . import placement
        ok, why = placement.policy(self.place_opt)
        if not ok:
            self.placement = {"placed": False, "why": why}
            return
        watch = placement.Stopwatch()
        if self.K == 1:
            self._place_whole(placement, nb)
        else:
            self._place_rows(placement)
        watch.stamp(self.placement)
        self.placement["searches"] = self._placements

    def _place_whole(self, placement, nb):
        KL = self.K * self.ld

        def probe(M, V):
            return placement.time_probe(lambda: ops.probe_adam_placement(self.P, self.G, M, V))

        def split(buf):
            t = buf.tensor()
            return t[:KL].view(self.K, self.ld), t[KL:2 * KL].view(self.K, self.ld)

        best, times = placement.choose(nb, self.P.device, lambda b: probe(*split(b)), probe(self._M, self._V),
                                       PLACEMENT_CANDIDATES, PLACEMENT_MAX_FRAC)
        chosen = 0
        if best is not None:
            chosen = min(range(len(times)), key=lambda i: times[i])
            M, V = split(best)
            M.copy_(self._M)
            V.copy_(self._V)
            self._M, self._V, self._placed = M, V, best
            self._Mr, self._Vr = list(M.unbind(0)), list(V.unbind(0))
            self.exp_avg, self.exp_avg_sq = M.view(-1), V.view(-1)
            for p in self.param_groups[0]["params"]:
                self._bind_state(p)
        self.placement = {"candidates": len(times), "probe_ms": [round(t, 4) for t in times], "chosen": chosen}

    def _place_rows(self, placement):
        Mr, Vr, bufs, rec = place_moment_rows(self.P, self.G, self._Mr, self._Vr)
        if any(b is not None for b in bufs):
            self._Mr, self._Vr, self._placed = Mr, Vr, bufs
            self._M = self._V = None
            self.exp_avg = self.exp_avg_sq = None
            for p in self.param_groups[0]["params"]:
                self._bind_state(p)
            torch.cuda.empty_cache()
        self.placement = rec

    def _ranges(self, k):
        """Contiguous ranges [a, b) of replica k's arena whose parameters have a
        gradient now (the whole row when all do: the padding stays 0)."""
        live = [(o, n) for p, o, n in self._spans[k] if p.grad is not None]
        if len(live) == len(self._spans[k]):
            return [(0, self.ld)]
        out = []
        for o, n in live:
            if out and o - out[-1][1] < 64:  # adjacent tensors (the alignment gap is zero padding)
                out[-1][1] = o + n
            else:
                out.append([o, o + n])
        return [(a, b) for a, b in out]

    @torch.no_grad()
    def step(self, closure=None, max_norm=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        ranges = [self._ranges(k) for k in range(self.K)]
        for ar in self.arenas:
            ar.sync_grads()
        if self._placed_for != (self.P.data_ptr(), self.G.data_ptr()):
            self._place()
        g = self.param_groups[0]
        lr, (b1, b2), eps, wd = float(g["lr"]), g["betas"], float(g["eps"]), float(g["weight_decay"])
        decoupled = g["decoupled_weight_decay"]
        self._step_t += 1
        t = float(self._step_t)
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        hp = dict(lerp_w=1 - b1, beta2=b2, one_m_beta2=1 - b2, eps=eps,
                  wd_factor=(1 - lr * wd) if (decoupled and wd != 0) else 1.0,
                  l2_wd=wd if (not decoupled and wd != 0) else 0.0, step_size=-(lr / bc1), bc2_sqrt=math.sqrt(bc2))
        clip = None
        if max_norm:
            ops.grad_clip_coef(self.G, self.ld, max_norm, self._partials, self._clip)
            clip = self._clip
        if self._M is not None and all(r == [(0, self.ld)] for r in ranges):
            ops.adam_step(self.P, self.G, self._M, self._V, clip_coef=clip, **hp)
            return loss
        for k in range(self.K):  # per replica (its moments placed apart, or partial ranges)
            ck = clip[2 * k:2 * k + 2] if clip is not None else None
            for a, b in ranges[k]:
                ops.adam_step(self.P[k, a:b], self.G[k, a:b], self._Mr[k][a:b], self._Vr[k][a:b], clip_coef=ck, **hp)
        return loss
