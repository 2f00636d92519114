"""Probe: does Tensor.bernoulli_(p_tensor) on a uint8 (or bool) destination draw
the same bits, and leave the generator in the same state, as the reference's
torch.bernoulli(torch.full(shape, p)).bool() (sparta.py:80-85)?  Run on the GPU
box; prints one JSON line."""
import json

import torch

dev = torch.device("cuda:0")
shapes = [(50304, 768), (1024, 768), (768,), (2304, 768), (2304,), (3072, 768), (66, 128), (3, 5, 7), (1,)]
p = 0.005
out = {}
for dst_dtype in (torch.uint8, torch.bool, torch.float32):
    ok_bits, ok_state = True, True
    for sh in shapes:
        torch.manual_seed(42)
        ref = torch.bernoulli(torch.full(sh, p, device=dev)).bool()
        s_ref = torch.cuda.get_rng_state()
        after_ref = torch.rand(4, device=dev)
        torch.manual_seed(42)
        P = torch.full(sh, p, device=dev)
        d = torch.empty(sh, dtype=dst_dtype, device=dev)
        d.bernoulli_(P)
        s_new = torch.cuda.get_rng_state()
        after_new = torch.rand(4, device=dev)
        ok_bits &= bool(torch.equal(ref, d.bool()))
        ok_state &= bool(torch.equal(s_ref, s_new)) and bool(torch.equal(after_ref, after_new))
    out[str(dst_dtype)] = {"bits_equal": ok_bits, "rng_state_equal": ok_state}
print(json.dumps(out), flush=True)
