"""Process-group setup (LocalTrainer._build_connection, exogym/trainer.py:310-351):
RCCL ("nccl") when every process has a GPU of its own, gloo when nodes share
GPUs; device placement rank % len(devices); 127.0.0.1 rendezvous; CPU/MPS
devices refused (no CPU path).  Host logic only: torch.distributed and the
device calls are stubbed."""
import pytest
import torch

from gym_amd import trainer as T


def test_select_backend():
    assert T.select_backend(8, list(range(8))) == "nccl"
    assert T.select_backend(4, list(range(8))) == "nccl"
    assert T.select_backend(2, [0]) == "gloo"
    assert T.select_backend(16, list(range(8))) == "gloo"


@pytest.fixture
def stub(monkeypatch):
    calls = {}
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: calls.setdefault("set_device", d))
    monkeypatch.setattr(T.dist, "init_process_group",
                        lambda backend, **kw: calls.update(backend=backend, **kw))
    return calls


def _trainer(rank, num_nodes, devices=None, device="cuda", world=None):
    tr = T.LocalTrainer(torch.nn.Linear(2, 2), None, None, start_port=30000)
    tr.rank, tr.num_nodes, tr.devices, tr.device = rank, num_nodes, devices, device
    if world is not None:
        tr.world_size = world
    return tr


def test_one_gpu_per_node_is_rccl(stub):
    tr = _trainer(rank=5, num_nodes=8)
    tr._build_connection()
    assert stub["backend"] == "nccl" and stub["world_size"] == 8 and stub["rank"] == 5
    assert stub["device_id"] == torch.device("cuda:5") and stub["set_device"] == 5
    assert tr.device == torch.device("cuda:5")
    import os
    assert os.environ["MASTER_ADDR"] == "127.0.0.1" and os.environ["MASTER_PORT"] == "30000"


def test_shared_gpus_are_gloo(stub):
    tr = _trainer(rank=3, num_nodes=4, devices=[0, 1])
    tr._build_connection()
    assert stub["backend"] == "gloo" and "device_id" not in stub
    assert stub["set_device"] == 1 and tr.device == torch.device("cuda:1")


def test_replica_processes_use_rccl(stub):
    """16 nodes on 8 GPUs: 8 processes hosting 2 nodes each, RCCL between them."""
    tr = _trainer(rank=7, num_nodes=16, world=8)
    tr._build_connection()
    assert stub["backend"] == "nccl" and stub["world_size"] == 8 and stub["device_id"] == torch.device("cuda:7")


@pytest.mark.parametrize("device", ["cpu", "mps"])
def test_cpu_devices_are_refused(stub, device):
    with pytest.raises(ValueError, match="Invalid device"):
        _trainer(rank=0, num_nodes=2, device=device)._build_connection()


def test_exchange_sharding_follows_arena_size():
    """RCCL across processes: arenas of >= 32 MB take the reduce-scatter ->
    shard kernel -> all-gather pipeline (bandwidth-bound, outer state / world),
    smaller ones one all-reduce (latency-bound, e.g. the char-level model of
    configs[1]: 3.7 MB); gloo and world size 1 never shard."""
    from types import SimpleNamespace

    from gym_amd.engine import SHARD_MIN_BYTES, default_shard
    from gym_amd.shapes import MODELS, numel
    rccl8 = SimpleNamespace(rccl=True, exchange=True)
    assert default_shard(rccl8, numel(MODELS["gpt2-124m"]()), torch.float32)
    assert not default_shard(rccl8, numel(MODELS["gpt2-char"]()), torch.float32)
    assert default_shard(rccl8, SHARD_MIN_BYTES // 4, torch.float32)
    assert not default_shard(rccl8, SHARD_MIN_BYTES // 4, torch.bfloat16)
    assert not default_shard(SimpleNamespace(rccl=False, exchange=True), 1 << 30, torch.float32)
    assert not default_shard(SimpleNamespace(rccl=True, exchange=False), 1 << 30, torch.float32)


def test_exchange_chunks_follow_world():
    """The sharded exchange's chunks: ~64 MB up to world 4, and each rank's piece
    at least PIECE_BYTES beyond (GPT-2 124M at world 8: 4 chunks of ~128 MB,
    ~16 MB per rank); the pieces tile the arena and each rank's shard."""
    from gym_amd.engine import PIECE_BYTES, ShardPlan
    from gym_amd.shapes import MODELS, numel
    n0 = numel(MODELS["gpt2-124m"]())
    for world, want in [(1, 8), (2, 8), (4, 8), (8, 4)]:
        n = -(-n0 // (8 * 64)) * 8 * 64
        plans = [ShardPlan(n, world, r, 4) for r in range(world)]
        assert len(plans[0].bounds) == want, world
        assert plans[0].bounds[0][0] == 0 and plans[0].bounds[-1][1] == n
        for p in plans:
            assert p.per * world == n
            assert all(b - a == (c1 - c0) // world for (a, b), (c0, c1) in zip(p.own, p.bounds))
        if world == 8:
            assert min(b - a for a, b in plans[0].own) * 4 >= PIECE_BYTES * 0.9
