#!/bin/bash
# r03w: DeMo synthesis batch size (entry pairs per batch of LDS reads ahead of the MFMAs): 2 and 8
# against 4 (build variants synb2 / synb8): parity under each, then same-box A/Bs.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03w
mkdir -p $O
export TMPDIR=/tmp
for VN in synb2 synb8; do
  GYM_AMD_LIB=$GRAFT_REPO_ROOT/build/libgym_amd_$VN.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "demo" > $O/tests_$VN.log 2>&1 || { echo "TESTS $VN FAILED"; tail -30 $O/tests_$VN.log; exit 1; }
  tail -1 $O/tests_$VN.log
  VNAME=$VN MODES="demo_encode demo_decode1" TAG=r03w/ab_$VN bash tools/ab_lib.sh || exit 1
done
echo DONE
