#!/bin/bash
# r03ac: DeMo chunk streams with non-temporal loads / stores / both (build variants) against the
# in-tree library: parity under each, then same-box A/Bs of the encode and both decodes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ac
mkdir -p $O
export TMPDIR=/tmp
for VN in nt_ld nt_st nt_both; do
  GYM_AMD_LIB=$GRAFT_REPO_ROOT/build/libgym_amd_$VN.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "demo" > $O/tests_$VN.log 2>&1 || { echo "TESTS $VN FAILED"; tail -30 $O/tests_$VN.log; exit 1; }
  tail -1 $O/tests_$VN.log
  VNAME=$VN MODES="demo_encode demo_decode1 demo_decode8" TAG=r03ac/ab_$VN bash tools/ab_lib.sh || exit 1
done
echo DONE
