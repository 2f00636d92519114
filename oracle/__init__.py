"""oracle — CPU restatement of the reference's strategy-communication-step
arithmetic (satoutahhaithem/gym @ 2025-07-11), in numpy.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package, and only as the checker (or, for the
baseline, as the thing timed on the host).  The product path (gym_amd) never
imports it and has no CPU fallback: without the HIP library it raises.

Parity pinning: every function here is checked against the golden fixtures in
tests/golden/*.npz, which tests/golden/gen_golden.py produced by running the
reference's own code (exogym.strategy.*, CPU/gloo) in the build container —
see tests/test_oracle_golden.py.  Functions with no reference counterpart (the
in-kernel Philox mask of gym_amd's fast SPARTA mode) are pinned by the
published Philox4x32-10 known-answer vectors instead.

Modules:
  reduce    mean over nodes                 strategy.py:130-133, diloco.py:34-37
  diloco    fused outer SGD/Nesterov step   diloco.py:43-76 + torch sgd.py
  sparta    masked gather/average/scatter   sparta.py:24-44; Philox4x32-10 mask
  demo      DCT codec + DeMo step           demo_impl/demo.py:142-498
  schedule  lambda_cosine LR                strategy.py:65-95
"""
