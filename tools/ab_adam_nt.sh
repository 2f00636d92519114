#!/bin/bash
# Same-box A/B of the inner AdamW + clip step (bench.py --only adamw) with and
# without non-temporal hints (VARIANTS: base = gym_amd/_lib, others = build/libgym_amd_<V>.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_adam
VARIANTS=${VARIANTS:-"base nt0"}
for r in 1 2 3; do
  for V in $VARIANTS; do
    L=$GRAFT_REPO_ROOT/build/libgym_amd_$V.so; [ $V = base ] && L=$GRAFT_REPO_ROOT/gym_amd/_lib/libgym_amd.so
    GYM_AMD_LIB=$L timeout -k 10 200 python bench.py --only adamw --no-cpu-baseline --no-pmc > gpurun_out/ab_adam/${V}_$r.txt 2>&1 || { tail -5 gpurun_out/ab_adam/${V}_$r.txt; exit 1; }
    echo "$V $(grep '^{' gpurun_out/ab_adam/${V}_$r.txt | tail -1 | cut -c1-400)"
  done
done
