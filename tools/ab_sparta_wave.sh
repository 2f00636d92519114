#!/bin/bash
# Same-box A/B of the wave-granular SPARTA average (K = 32, GPT-2 124M), interleaved:
# w4 = gym_amd/_lib (4 waves per workgroup), others = build/libgym_amd_<V>.so built
# from variants of gym_amd/csrc/sparta.hip (e.g. -DGA_SP_WAVES=1/2/8); round-2 records
# in profiles/r02q_ab_sparta_wave.txt.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/ab_wave
mkdir -p $O
VARIANTS=${VARIANTS:-"w4 w1 w2 w8"}
for r in 1 2 3; do
  for V in $VARIANTS; do
    L=$GRAFT_REPO_ROOT/build/libgym_amd_$V.so
    [ $V = w4 ] && L=$GRAFT_REPO_ROOT/gym_amd/_lib/libgym_amd.so
    GYM_AMD_LIB=$L timeout -k 10 120 python tools/prof_kernels.py sparta_elem 20 > $O/${V}_$r.json || exit 1
    echo "$V $(python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['ms'])" $O/${V}_$r.json)"
  done
done
