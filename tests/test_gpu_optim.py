"""Fused inner optimizer on the MI355X (ga_adam_step, ga_grad_clip_coef through
the C ABI) against torch.optim.AdamW / Adam + clip_grad_norm_ running on the
same GPU (the reference's inner optimizer).  fp32 tolerance: reordered norm
sums and FMA contraction differ at the ulp level; 1e-5 relative after 5 steps."""
import pytest
import torch

import optim_cases as C

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,cls,kw,max_norm,skip", C.CASES, ids=[c[0] for c in C.CASES])
def test_arena_adam_matches_torch_on_gpu(name, cls, kw, max_norm, skip):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ours, ref = C.run_pair("cuda:0", cls, kw, max_norm=max_norm, skip=skip)
    C.assert_close(ours, ref)


def test_clip_coef_kernel():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gym_amd import ops
    g = torch.randn(1_000_003, device="cuda") * 0.01
    part, out = ops.sumsq_partials(g.device), torch.zeros(2, device="cuda")
    ops.grad_clip_coef(g, g.numel(), 0.5, part, out)
    ref = torch.linalg.vector_norm(g.double()).item()
    assert abs(out[1].item() - ref) <= 1e-5 * ref
    assert abs(out[0].item() - min(1.0, 0.5 / (ref + 1e-6))) <= 1e-5

