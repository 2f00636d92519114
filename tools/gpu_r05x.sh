#!/bin/bash
# r05x: the multi-source decode scales by 2^-k for power-of-two hit counts (mean_pow2; in-tree)
# vs build/libgym_amd_base.so: DeMo kernel parity, then interleaved decode timing.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05x
mkdir -p $O
export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/build/libgym_amd_base.so
N=$GRAFT_REPO_ROOT/gym_amd/_lib/libgym_amd.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -k "demo" -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/exp_demo_ablate.py --decode 8 $B $N > $O/ab_decode8.txt 2>&1 || { echo "AB FAILED"; tail -20 $O/ab_decode8.txt; exit 1; }
cat $O/ab_decode8.txt
timeout -k 10 300 python tools/exp_demo_ablate.py --decode 8 $N $B > $O/ab_decode82.txt 2>&1 || { echo "AB2 FAILED"; tail -20 $O/ab_decode82.txt; exit 1; }
cat $O/ab_decode82.txt
timeout -k 10 300 python tools/exp_demo_ablate.py --decode 2 $B $N > $O/ab_decode2src.txt 2>&1 || { echo "AB3 FAILED"; tail -20 $O/ab_decode2src.txt; exit 1; }
cat $O/ab_decode2src.txt
