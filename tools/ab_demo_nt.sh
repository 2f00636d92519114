#!/bin/bash
# Same-box A/B of the DeMo codec kernels with and without non-temporal hints on the
# chunk loads/stores (VARIANTS: base = gym_amd/_lib, others = build/libgym_amd_<V>.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_demo_nt
VARIANTS=${VARIANTS:-"base nt0"}
for r in 1 2 3; do
  for V in $VARIANTS; do
    L=$GRAFT_REPO_ROOT/build/libgym_amd_$V.so; [ $V = base ] && L=$GRAFT_REPO_ROOT/gym_amd/_lib/libgym_amd.so
    line="$V"
    for M in demo_encode demo_decode1 demo_decode8; do
      GYM_AMD_LIB=$L timeout -k 10 150 python tools/prof_kernels.py $M 10 > gpurun_out/ab_demo_nt/${M}_${V}_$r.txt 2>&1 || { tail -5 gpurun_out/ab_demo_nt/${M}_${V}_$r.txt; exit 1; }
      line="$line $M $(python -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]['ms'])" gpurun_out/ab_demo_nt/${M}_${V}_$r.txt)"
    done
    echo $line
  done
done
