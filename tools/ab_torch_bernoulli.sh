#!/bin/bash
# Same-box A/B of Philox variants (VARIANTS: base = gym_amd/_lib, others =
# build/libgym_amd_<V>.so): the fused reference draw (tools/time_mask_draw.py, with its
# check against the per-tensor torch draws over GPT-2 124M) and the Philox-mode SPARTA
# average (tools/prof_kernels.py sparta_elem, K = 32).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_tb
VARIANTS=${VARIANTS:-"base oldxor"}
for r in 1 2 3; do
  for V in $VARIANTS; do
    L=$GRAFT_REPO_ROOT/build/libgym_amd_$V.so; [ $V = base ] && L=$GRAFT_REPO_ROOT/gym_amd/_lib/libgym_amd.so
    GYM_AMD_LIB=$L timeout -k 10 120 python tools/time_mask_draw.py > gpurun_out/ab_tb/${V}_$r.txt 2>&1 || { tail -5 gpurun_out/ab_tb/${V}_$r.txt; exit 1; }
    GYM_AMD_LIB=$L timeout -k 10 120 python tools/prof_kernels.py sparta_elem 20 > gpurun_out/ab_tb/sp_${V}_$r.txt 2>&1 || { tail -5 gpurun_out/ab_tb/sp_${V}_$r.txt; exit 1; }
    python - gpurun_out/ab_tb/${V}_$r.txt gpurun_out/ab_tb/sp_${V}_$r.txt $V <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
s = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")]
print(sys.argv[3], "fused_draw_ms", round(d[0]["fused"]["gpu_ms"], 4), d[1], "sparta_elem_ms", s[0]["ms"])
PY
  done
done
