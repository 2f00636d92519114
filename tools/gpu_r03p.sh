#!/bin/bash
# r03p: AdamW sc1 stores (r03o), then the reference-draw SPARTA step with 2 / 4 64-element
# groups per lane (8192 / 16384-element wave tiles; build variants spg2 / spg4) against the
# in-tree library (4096-element wave tiles).
set -o pipefail
cd $GRAFT_REPO_ROOT

O=gpurun_out/r03p
mkdir -p $O
for VN in spg2 spg4; do
  GYM_AMD_LIB=$GRAFT_REPO_ROOT/build/libgym_amd_$VN.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "reference_draw or in_kernel or average_local" > $O/tests_$VN.log 2>&1 || { echo "TESTS $VN FAILED"; tail -30 $O/tests_$VN.log; exit 1; }
  tail -1 $O/tests_$VN.log
  VNAME=$VN MODES="sparta_torch sparta_elem" TAG=r03p/ab_$VN bash tools/ab_lib.sh || exit 1
done
echo DONE
