"""The RCCL ("nccl" backend) code paths on a one-GPU box: a world-size-1 RCCL
process group with Collective(force_exchange=True), so the engines take their
multi-rank paths -- the chunk-pipelined reduce_scatter_tensor /
all_gather_into_tensor(async_op=True) exchange with Work.wait() stream
ordering (engine.ShardPlan.run), SPARTA's all-reduce of the packed values and
DeMo's all-gather -- and the results are checked against the oracle.
Multi-rank gloo runs of the same scenario: test_strategies_gloo.py /
test_gpu_strategies.py."""
import pytest
import torch

import strategy_scenarios as S
from conftest import GOLDEN
from scenario_checks import check_engine

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("chunks", [1, 4])
def test_rccl_world1_engines(tmp_path, chunks):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = S.run("engine", 1, "cuda:0", False, str(tmp_path), GOLDEN, backend="nccl", force=True, chunks=chunks)
    check_engine(res, 1, GOLDEN)
