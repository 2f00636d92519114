#!/bin/bash
# Same-box A/B of the wave kernel's gather batch: base = gym_amd/_lib (register-only
# batch: DPP lane walk for the ascending sum, 8 passes in flight), np4 = the same with 4
# passes (-DGA_SP_DPP_PASSES=4), lds = the LDS-staged batch (-DGA_SP_LDS_STAGE).
# SPARTA parity tests under each library, then K=32 timings (Philox and in-kernel torch draw).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_batch
VARIANTS=${VARIANTS:-"base np4 lds"}
for V in $VARIANTS; do
  L=$GRAFT_REPO_ROOT/build/libgym_amd_$V.so; [ $V = base ] && L=$GRAFT_REPO_ROOT/gym_amd/_lib/libgym_amd.so
  GYM_AMD_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread -k "sparta" > gpurun_out/ab_batch/tests_$V.log 2>&1 || { echo "$V TESTS FAILED"; tail -20 gpurun_out/ab_batch/tests_$V.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/ab_batch/tests_$V.log)"
done
for r in 1 2 3; do
  for V in $VARIANTS; do
    L=$GRAFT_REPO_ROOT/build/libgym_amd_$V.so; [ $V = base ] && L=$GRAFT_REPO_ROOT/gym_amd/_lib/libgym_amd.so
    for M in sparta_elem sparta_torch; do
      GYM_AMD_LIB=$L timeout -k 10 120 python tools/prof_kernels.py $M 20 > gpurun_out/ab_batch/${M}_${V}_$r.txt 2>&1 || exit 1
    done
    echo "$V sparta_elem_ms $(python -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]['ms'])" gpurun_out/ab_batch/sparta_elem_${V}_$r.txt) sparta_torch_ms $(python -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]['ms'])" gpurun_out/ab_batch/sparta_torch_${V}_$r.txt)"
  done
done
