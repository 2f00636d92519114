#!/bin/bash
# Same-box A/B of the in-kernel reference draw's tensor lookup (base = gym_amd/_lib:
# wave-uniform search + per-lane forward walk; bsearch = build/libgym_amd_bsearch.so:
# a per-lane binary search in global memory): parity tests, then timings.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_st
for V in base bsearch; do
  L=$GRAFT_REPO_ROOT/build/libgym_amd_$V.so; [ $V = base ] && L=$GRAFT_REPO_ROOT/gym_amd/_lib/libgym_amd.so
  GYM_AMD_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "in_kernel_reference_draw or bernoulli" > gpurun_out/ab_st/tests_$V.log 2>&1 || { echo "$V TESTS FAILED"; tail -20 gpurun_out/ab_st/tests_$V.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/ab_st/tests_$V.log)"
done
for r in 1 2 3; do
  for V in base bsearch; do
    L=$GRAFT_REPO_ROOT/build/libgym_amd_$V.so; [ $V = base ] && L=$GRAFT_REPO_ROOT/gym_amd/_lib/libgym_amd.so
    GYM_AMD_LIB=$L timeout -k 10 120 python tools/prof_kernels.py sparta_torch 20 > gpurun_out/ab_st/st_${V}_$r.txt 2>&1 || exit 1
    echo "$V sparta_torch_ms $(python -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]['ms'])" gpurun_out/ab_st/st_${V}_$r.txt)"
  done
done
