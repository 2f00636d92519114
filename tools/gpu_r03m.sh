#!/bin/bash
# r03m: DeMo kernels with device-scope (sc1) buffer stores (build variant demosc1): parity under the
# variant, then the same-box A/B against the in-tree library.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03m
mkdir -p $O
export TMPDIR=/tmp
GYM_AMD_LIB=$GRAFT_REPO_ROOT/build/libgym_amd_demosc1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "demo" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
VNAME=demosc1 MODES="demo_encode demo_decode8 demo_decode1" TAG=r03m/ab bash tools/ab_lib.sh || exit 1

timeout -k 10 120 python tools/demo_stamps.py --wave > gpurun_out/r03m/stamps.txt 2>&1 || { echo "STAMPS FAILED"; tail -5 gpurun_out/r03m/stamps.txt; exit 1; }
cat gpurun_out/r03m/stamps.txt
echo DONE
