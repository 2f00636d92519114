#!/bin/bash
# r03ae: DeMo encode with the next chunk prefetched by LDS-DMA dword touches
# (GA_DEMO_PREFETCH=1 variant, build/libgym_amd_demopf.so): parity of the variant, then
# interleaved same-box A/B against the in-tree library.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ae
mkdir -p $O
export TMPDIR=/tmp
GYM_AMD_LIB=$GRAFT_REPO_ROOT/build/libgym_amd_demopf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "demo and encode" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
VNAME=demopf MODES="demo_encode" TAG=r03ae/ab bash tools/ab_lib.sh || exit 1
echo DONE
