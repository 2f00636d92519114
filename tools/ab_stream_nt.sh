#!/bin/bash
# Same-box A/B of the streaming kernels with and without non-temporal hints
# (VARIANTS: base = gym_amd/_lib, others = build/libgym_amd_<V>.so): ga_diloco_outer
# at K = 8 over GPT-2 124M (tools/prof_kernels.py diloco) and the bench's headline
# line without extras (its copy_GBps uses ga_stream_copy from the same library).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_nt
VARIANTS=${VARIANTS:-"base nt0"}
for r in 1 2 3; do
  for V in $VARIANTS; do
    L=$GRAFT_REPO_ROOT/build/libgym_amd_$V.so; [ $V = base ] && L=$GRAFT_REPO_ROOT/gym_amd/_lib/libgym_amd.so
    GYM_AMD_LIB=$L timeout -k 10 120 python tools/prof_kernels.py diloco 20 > gpurun_out/ab_nt/diloco_${V}_$r.txt 2>&1 || { tail -5 gpurun_out/ab_nt/diloco_${V}_$r.txt; exit 1; }
    GYM_AMD_LIB=$L timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-pmc > gpurun_out/ab_nt/bench_${V}_$r.txt 2>&1 || { tail -5 gpurun_out/ab_nt/bench_${V}_$r.txt; exit 1; }
    python - $V $r <<'PY'
import json, sys
V, r = sys.argv[1], sys.argv[2]
g = lambda f: [json.loads(l) for l in open(f"gpurun_out/ab_nt/{f}_{V}_{r}.txt") if l.startswith("{")]
b = g("bench")[-1]
print(V, "diloco_kernel_ms", g("diloco")[0]["ms"], "bench_ms", b["ms_per_step"], "kernel_ms", b["roofline"]["kernel_ms"],
      "copy_GBps", b["roofline"].get("copy_GBps"), "frac", b["roofline"]["frac"])
PY
  done
done
