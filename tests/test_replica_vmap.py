"""replica_forward="vmap" (gym_amd.replica.BatchedForward): the K local nodes'
forward/backward as one torch.func.vmap over the replica arena's rows gives
each node the gradients, losses and BatchNorm statistics of its own
forward/backward (the default per-node loop) up to fp32 rounding, accumulates
in place into the arena across minibatches, and trains end to end through
ReplicaTrainNode to the loop's parameters.  CPU; tests/test_gpu_replica.py
repeats the end-to-end case with the kernels."""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from test_replica_mode import fake  # noqa: F401  (fixture)


class TinyNet(nn.Module):
    """Linear -> BatchNorm -> causal SDPA attention -> mean-pool head; the
    forward takes the (x, y) minibatch and returns the loss (TrainNode's
    contract, exogym/train_node.py:145-175)."""

    def __init__(self, seed=3, masked=False, norm="bn"):
        super().__init__()
        self.masked = masked  # an explicit mask: the math-backend path of BatchedForward's attention
        self.norm = norm
        torch.manual_seed(seed)
        self.lin = nn.Linear(8, 16, bias=False)  # BatchNorm follows: a bias would get ~0 gradients that AdamW amplifies
        self.bn = nn.BatchNorm1d(16) if norm == "bn" else nn.LayerNorm(16)
        self.qkv = nn.Linear(16, 48, bias=False)  # (a key bias gets ~0 gradients too: softmax is shift-invariant)
        self.head = nn.Linear(16, 4)

    def forward(self, batch):
        x, y = batch
        B, T, _ = x.shape
        h = self.lin(x)
        h = self.bn(h.transpose(1, 2)).transpose(1, 2) if self.norm == "bn" else self.bn(h)
        q, k, v = (t.reshape(B, T, 2, 8).transpose(1, 2) for t in self.qkv(h).split(16, dim=-1))
        if self.masked:
            mask = torch.ones(T, T, dtype=torch.bool, device=x.device).tril()
            z = F.scaled_dot_product_attention(q, k, v, attn_mask=mask)
        else:
            z = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        h = h + z.transpose(1, 2).reshape(B, T, 16)
        return F.cross_entropy(self.head(h.mean(1)), y)


def _batches(K, n, seed):
    g = torch.Generator().manual_seed(seed)
    return [[(torch.randn(6, 5, 8, generator=g), torch.randint(0, 4, (6,), generator=g)) for _ in range(n)]
            for _ in range(K)]


def _bufs(models):
    return [[b.detach().clone() for b in m.buffers()] for m in models]


@pytest.mark.parametrize("masked", [False, True])
def test_batched_forward_matches_loop(masked):
    from gym_amd.arena import ReplicaArena
    from gym_amd.replica import BatchedForward
    K, accum = 3, 2
    models = [TinyNet(masked=masked) for _ in range(K)]
    with torch.no_grad():  # the nodes differ
        for k, m in enumerate(models):
            for p in m.parameters():
                p.add_(0.05 * k * torch.randn_like(p))
    ra = ReplicaArena(models)
    data = _batches(K, accum, seed=7)
    b0 = _bufs(models)
    ra.zero_grad()
    loop_losses = []
    for k, m in enumerate(models):
        for j in range(accum):
            loss = m(data[k][j])
            loss.backward()
            loop_losses.append(float(loss.detach()))
    ra.sync_grads()
    g_loop, b_loop = ra.grad_set.clone(), _bufs(models)
    with torch.no_grad():  # BatchNorm statistics back to the start
        for m, bs in zip(models, b0):
            for b, v in zip(m.buffers(), bs):
                b.copy_(v)
    ra.zero_grad()
    bf = BatchedForward(models, ra, chunk=2)  # chunks of 2 + 1 nodes
    vm_losses = [bf([data[k][j] for k in range(K)]) for j in range(accum)]
    ra.sync_grads()
    np.testing.assert_allclose(ra.grad_set.numpy(), g_loop.numpy(), rtol=1e-5, atol=1e-7)
    got = torch.stack(vm_losses, 1).reshape(-1).numpy()
    np.testing.assert_allclose(got, np.array(loop_losses, np.float32), rtol=1e-6, atol=1e-7)
    for bs_v, bs_l in zip(_bufs(models), b_loop):
        for v, w in zip(bs_v, bs_l):
            np.testing.assert_allclose(v.numpy(), w.numpy(), rtol=1e-6, atol=1e-7)
    # the arena rows are still every model's parameters and gradients
    ra.check_bound()
    assert F.scaled_dot_product_attention is torch._C._nn.scaled_dot_product_attention  # the patch is undone


def test_batched_forward_frozen_parameter():
    from gym_amd.arena import ReplicaArena
    from gym_amd.replica import BatchedForward
    models = [TinyNet() for _ in range(2)]
    for m in models:
        m.head.bias.requires_grad_(False)
    ra = ReplicaArena(models)
    ra.zero_grad()
    BatchedForward(models, ra)([d[0] for d in _batches(2, 1, seed=1)])
    o = ra.layout.offsets[[n for n, _ in models[0].named_parameters()].index("head.bias")]
    assert (ra.grad_set[:, o:o + 4] == 0).all() and ra.grad_set.abs().sum() > 0


def _train(forward, device="cpu", strategy="simple", seed=11):
    from torch.utils.data import TensorDataset

    from gym_amd.replica import ReplicaTrainNode
    from replica_scenarios import make_strategy
    g = torch.Generator().manual_seed(seed)
    ds = TensorDataset(torch.randn(96, 5, 8, generator=g), torch.randint(0, 4, (96,), generator=g))

    class DS(torch.utils.data.Dataset):  # (x, y) items -> one tuple per sample
        def __len__(self):
            return len(ds)

        def __getitem__(self, i):
            return ds[i]

    node = ReplicaTrainNode(TinyNet(), DS(), DS(), make_strategy(strategy), device, rank=0, num_nodes=3, K=3,
                            num_epochs=1, max_steps=3, batch_size=8, minibatch_size=4, val_size=0,
                            replica_forward=forward, replica_vmap_chunk=2)
    return node.train()


def assert_states_close(loop, vm):
    """Every node's state after a few AdamW steps: AdamW's first steps move an
    element by ~lr whatever its gradient's size, so the rare element whose
    gradient is ~0 (rounding-level) may move differently; >= 99.5% of each
    tensor within 1e-4 relative / 1e-5 absolute, none further than lr / 5."""
    for sl, sv in zip(loop, vm):
        for key in sl:
            a, b = sv[key].float().cpu().numpy(), sl[key].float().cpu().numpy()
            d = np.abs(a - b)
            assert (d <= 1e-5 + 1e-4 * np.abs(b)).mean() >= 0.995, (key, float(d.max()))
            assert d.max() <= 2e-3, (key, float(d.max()))


def test_replica_trainnode_vmap_matches_loop(fake):  # noqa: F811
    assert_states_close(_train("loop"), _train("vmap"))


def test_replica_forward_rejects_unknown_mode(fake):  # noqa: F811
    with pytest.raises(ValueError):
        _train("graph")


def test_batched_forward_under_autocast():
    """bf16 autocast around the batched forward (ReplicaTrainNode(autocast=True)):
    the folded attention's backward recomputes under the forward's autocast
    state; gradients match the per-node loop under the same autocast.  (LayerNorm:
    torch's vmap rule for batch_norm rejects autocast's mixed dtypes on this
    stack, so BatchNorm models under autocast keep the loop.)"""
    import contextlib

    from gym_amd.arena import ReplicaArena
    from gym_amd.replica import BatchedForward
    K = 2
    models = [TinyNet(norm="ln") for _ in range(K)]
    ra = ReplicaArena(models)
    data = _batches(K, 1, seed=3)
    b0 = _bufs(models)

    def ac():
        return torch.autocast(device_type="cpu", dtype=torch.bfloat16)

    ra.zero_grad()
    for k, m in enumerate(models):
        with ac():
            loss = m(data[k][0])
        loss.backward()
    ra.sync_grads()
    g_loop = ra.grad_set.clone()
    with torch.no_grad():
        for m, bs in zip(models, b0):
            for b, v in zip(m.buffers(), bs):
                b.copy_(v)
    ra.zero_grad()
    BatchedForward(models, ra)([data[k][0] for k in range(K)], ac)
    ra.sync_grads()
    assert ra.grad_set.abs().sum() > 0
    np.testing.assert_allclose(ra.grad_set.numpy(), g_loop.numpy(), rtol=2e-2, atol=2e-3)


def test_sdpa_override_is_local_to_the_batched_forward():
    """The batched forward's attention override is a torch-function mode on its
    own thread: SDPA called from a second thread while the vmap forward runs is
    torch's own (no folded autograd node), and the module attribute is never
    swapped."""
    import threading

    from gym_amd.arena import ReplicaArena
    from gym_amd.replica import BatchedForward
    seen = {}

    def other_thread():
        q = torch.randn(2, 2, 5, 8, requires_grad=True)
        out = F.scaled_dot_product_attention(q, q, q)
        seen["fn"] = F.scaled_dot_product_attention
        seen["grad_fn"] = type(out.grad_fn).__name__

    class Spy(TinyNet):
        def forward(self, batch):
            t = threading.Thread(target=other_thread)
            t.start()
            t.join()
            seen["main_sdpa"] = F.scaled_dot_product_attention
            return super().forward(batch)

    models = [Spy() for _ in range(2)]
    ra = ReplicaArena(models)
    ra.zero_grad()
    BatchedForward(models, ra)([d[0] for d in _batches(2, 1, seed=5)])
    assert seen["fn"] is torch._C._nn.scaled_dot_product_attention
    assert seen["main_sdpa"] is torch._C._nn.scaled_dot_product_attention
    assert "Folded" not in seen["grad_fn"], seen["grad_fn"]
    assert ra.grad_set.abs().sum() > 0


def test_batched_forward_unfoldable_attention_is_exact():
    """k / v broadcast over SDPA's batch (a leading 1) cannot be folded into the
    node dim: the batched forward takes the math backend and still matches the
    per-node loop."""
    from gym_amd.arena import ReplicaArena
    from gym_amd.replica import BatchedForward

    class Bcast(TinyNet):
        def forward(self, batch):
            x, y = batch
            B, T, _ = x.shape
            h = self.lin(x)
            h = self.bn(h.transpose(1, 2)).transpose(1, 2)
            q, k, v = (t.reshape(B, T, 2, 8).transpose(1, 2) for t in self.qkv(h).split(16, dim=-1))
            z = F.scaled_dot_product_attention(q, k[:1], v[:1])  # k, v broadcast over the batch
            h = h + z.transpose(1, 2).reshape(B, T, 16)
            return F.cross_entropy(self.head(h.mean(1)), y)

    K = 2
    models = [Bcast() for _ in range(K)]
    with torch.no_grad():
        for k, m in enumerate(models):
            for p in m.parameters():
                p.add_(0.05 * k * torch.randn_like(p))
    ra = ReplicaArena(models)
    data = _batches(K, 1, seed=9)
    b0 = _bufs(models)
    ra.zero_grad()
    for k, m in enumerate(models):
        m(data[k][0]).backward()
    ra.sync_grads()
    g_loop = ra.grad_set.clone()
    with torch.no_grad():
        for m, bs in zip(models, b0):
            for b, v in zip(m.buffers(), bs):
                b.copy_(v)
    ra.zero_grad()
    BatchedForward(models, ra)([data[k][0] for k in range(K)])
    ra.sync_grads()
    np.testing.assert_allclose(ra.grad_set.numpy(), g_loop.numpy(), rtol=1e-5, atol=1e-7)


def test_batched_forward_follows_the_models_mode():
    """A model put in eval() after the batched forward was built runs its
    BatchNorm on running statistics in the vmap path too (as the loop does)."""
    from gym_amd.arena import ReplicaArena
    from gym_amd.replica import BatchedForward
    K = 2
    models = [TinyNet() for _ in range(K)]
    ra = ReplicaArena(models)
    bf = BatchedForward(models, ra)
    for m in models:
        m.eval()
    data = _batches(K, 1, seed=4)
    b0 = _bufs(models)
    ra.zero_grad()
    for k, m in enumerate(models):
        m(data[k][0]).backward()
    ra.sync_grads()
    g_loop = ra.grad_set.clone()
    ra.zero_grad()
    bf([data[k][0] for k in range(K)])
    ra.sync_grads()
    assert not bf.meta.training
    np.testing.assert_allclose(ra.grad_set.numpy(), g_loop.numpy(), rtol=1e-5, atol=1e-7)
    for bs_v, bs_0 in zip(_bufs(models), b0):  # eval: running statistics untouched
        for v, w in zip(bs_v, bs_0):
            assert torch.equal(v, w)
