#!/bin/bash
# r03v: DeMo encode with registers holding no candidate skipped in the top-k compaction (build
# variant skip): parity under the variant, then the same-box A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03v
mkdir -p $O
export TMPDIR=/tmp
GYM_AMD_LIB=$GRAFT_REPO_ROOT/build/libgym_amd_skip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -x -v --timeout 120 --timeout-method thread -k "demo" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
VNAME=skip MODES="demo_encode" TAG=r03v/ab bash tools/ab_lib.sh || exit 1
echo DONE
