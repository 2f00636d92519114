#!/bin/bash
# Same-box A/B of the reference-draw kernels (VARIANTS: base = gym_amd/_lib, others =
# build/libgym_amd_<V>.so): ga_sparta_torch_bernoulli into the packed mask
# (prof_kernels torch_draw), the average kernel drawing in-kernel (sparta_torch),
# and draw_masks' fused byte draw with its check against the per-tensor torch draws.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_tw
VARIANTS=${VARIANTS:-"base old"}
for r in 1 2 3; do
  for V in $VARIANTS; do
    L=$GRAFT_REPO_ROOT/build/libgym_amd_$V.so; [ $V = base ] && L=$GRAFT_REPO_ROOT/gym_amd/_lib/libgym_amd.so
    for M in ${MODES:-torch_draw sparta_torch}; do
      GYM_AMD_LIB=$L timeout -k 10 120 python tools/prof_kernels.py $M 50 > gpurun_out/ab_tw/${M}_${V}_$r.txt 2>&1 || { tail -5 gpurun_out/ab_tw/${M}_${V}_$r.txt; exit 1; }
    done
    GYM_AMD_LIB=$L timeout -k 10 120 python tools/time_mask_draw.py > gpurun_out/ab_tw/fused_${V}_$r.txt 2>&1 || { tail -5 gpurun_out/ab_tw/fused_${V}_$r.txt; exit 1; }
    python - $V $r <<'PY'
import json, sys
V, r = sys.argv[1], sys.argv[2]
g = lambda f: [json.loads(l) for l in open(f"gpurun_out/ab_tw/{f}_{V}_{r}.txt") if l.startswith("{")]
d = g("fused")
import os
ms = {m: g(m)[0]["ms"] for m in os.environ.get("MODES", "torch_draw sparta_torch").split()}
print(V, ms, "fused_byte_draw_ms", round(d[0]["fused"]["gpu_ms"], 4), d[1])
PY
  done
done
