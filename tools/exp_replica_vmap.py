"""Replica mode's forward/backward: K model copies in a Python loop (today's
ReplicaTrainNode) vs one torch.func.vmap over the K parameter rows (diagnostic,
round 5).  A nanoGPT-shaped GPT (example/nanogpt/nanogpt.py:
SDPA causal attention, GELU MLP, tied head; dropout 0) with K replicas whose
parameters are views of one [K, ld] set; per replica one minibatch of B x T
tokens.  Prints ms per inner step (zero_grad excluded) for both forms and the
largest relative gradient difference between them.  One JSON line per config.
Under vmap SDPA runs as gym_amd.replica's folded call (VMAP_SDPA=FOLD, the
default: the nodes folded into the fused kernel's batch dim) or on the backend
VMAP_SDPA names (MATH; FLASH_ATTENTION / EFFICIENT_ATTENTION fail in backward
on this stack: no batching rule).
Usage: python tools/exp_replica_vmap.py [n_layer,d_model,heads,T,B,K,chunk[,vocab]]..."""
import copy
import json
import sys
import time

import os

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.func import functional_call, vmap


class Attn(nn.Module):
    def __init__(s, d, nh):
        super().__init__()
        s.nh = nh
        s.c_attn = nn.Linear(d, 3 * d)
        s.c_proj = nn.Linear(d, d)

    def forward(s, x):
        B, T, C = x.shape
        q, k, v = s.c_attn(x).split(C, dim=2)
        q, k, v = (t.view(B, T, s.nh, C // s.nh).transpose(1, 2) for t in (q, k, v))
        y = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        return s.c_proj(y.transpose(1, 2).contiguous().view(B, T, C))


class Block(nn.Module):
    def __init__(s, d, nh):
        super().__init__()
        s.ln_1, s.attn, s.ln_2 = nn.LayerNorm(d), Attn(d, nh), nn.LayerNorm(d)
        s.c_fc, s.c_proj = nn.Linear(d, 4 * d), nn.Linear(4 * d, d)

    def forward(s, x):
        x = x + s.attn(s.ln_1(x))
        return x + s.c_proj(F.gelu(s.c_fc(s.ln_2(x))))


class GPT(nn.Module):
    def __init__(s, n_layer, d, nh, T, V=50304):
        super().__init__()
        s.wte, s.wpe = nn.Embedding(V, d), nn.Embedding(T, d)
        s.h = nn.ModuleList([Block(d, nh) for _ in range(n_layer)])
        s.ln_f = nn.LayerNorm(d)

    def forward(s, idx):
        x, y = idx[..., :-1], idx[..., 1:]
        T = x.shape[-1]
        h = s.wte(x) + s.wpe(torch.arange(T, device=x.device))
        for b in s.h:
            h = b(h)
        logits = F.linear(s.ln_f(h), s.wte.weight)
        return F.cross_entropy(logits.reshape(-1, logits.shape[-1]), y.reshape(-1))


def timeit(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return 1e3 * sorted(ts)[len(ts) // 2]


def run(n_layer, d, nh, T, B, K, chunk, V=50304):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    base = GPT(n_layer, d, nh, T + 1, V).to(dev)
    names = [n for n, _ in base.named_parameters()]
    shapes = [p.shape for _, p in base.named_parameters()]
    sizes = [p.numel() for _, p in base.named_parameters()]
    offs = [0]
    for n in sizes:
        offs.append(offs[-1] + n)
    ld = offs[-1]
    Pset = torch.empty(K, ld, device=dev)
    Gset = torch.zeros(K, ld, device=dev)
    with torch.no_grad():
        flat = torch.cat([p.reshape(-1) for p in base.parameters()])
        Pset.copy_(flat.expand(K, ld))
    # loop form: K modules whose params are row views
    models = []
    for k in range(K):
        m = copy.deepcopy(base)
        for (n, p), o, sz, sh in zip(m.named_parameters(), offs, sizes, shapes):
            p.data = Pset[k, o:o + sz].view(sh)
            p.grad = Gset[k, o:o + sz].view(sh)
        models.append(m)
    data = torch.randint(0, V, (K, B, T + 1), device=dev)

    def loop():
        Gset.zero_()
        for k, m in enumerate(models):
            m(data[k]).backward()

    t_loop = timeit(loop)
    g_loop = Gset.clone()
    meta = copy.deepcopy(base).to("meta")
    bufs = dict(base.named_buffers())

    def f(ps, idx):
        return functional_call(meta, ({n: p for n, p in zip(names, ps)}, bufs), (idx,))

    vf = vmap(f, in_dims=(0, 0), randomness="different")

    from torch.nn.attention import SDPBackend, sdpa_kernel
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from gym_amd.replica import _vmappable_attention
    mode = os.environ.get("VMAP_SDPA", "FOLD")
    ctx = _vmappable_attention if mode == "FOLD" else (lambda: sdpa_kernel(getattr(SDPBackend, mode)))

    def vm():
        Gset.zero_()
        for c0 in range(0, K, chunk):
            c1 = min(K, c0 + chunk)
            leaves = []
            for o, sz, sh in zip(offs, sizes, shapes):
                w = Pset[c0:c1, o:o + sz].view(c1 - c0, *sh).detach().requires_grad_()
                w.grad = Gset[c0:c1, o:o + sz].view(c1 - c0, *sh)
                leaves.append(w)
            with ctx():
                vf(leaves, data[c0:c1]).sum().backward()

    t_vmap = timeit(vm)
    rel = float(((Gset - g_loop).abs().max() / g_loop.abs().max().clamp_min(1e-30)).item())
    tokens = K * B * T
    flops = 6.0 * ld * tokens
    return {"n_layer": n_layer, "d": d, "vocab": V, "T": T, "B": B, "K": K, "chunk": chunk, "params_M": round(ld / 1e6, 1),
            "loop_ms": round(t_loop, 2), "vmap_ms": round(t_vmap, 2), "speedup": round(t_loop / t_vmap, 3),
            "loop_TFLOPs": round(flops / t_loop / 1e9, 1), "vmap_TFLOPs": round(flops / t_vmap / 1e9, 1),
            "grad_max_rel_diff": rel, "vmap_sdpa": mode, "mem_GB": round(torch.cuda.max_memory_allocated() / 1e9, 1)}


if __name__ == "__main__":
    cfgs = [list(map(int, a.split(","))) for a in sys.argv[1:]] or [
        [4, 256, 4, 128, 4, 32, 32], [12, 768, 12, 256, 2, 32, 8], [12, 768, 12, 1024, 8, 32, 4]]
    for c in cfgs:
        torch.cuda.reset_peak_memory_stats()
        print(json.dumps(run(*c)), flush=True)
        torch.cuda.empty_cache()
