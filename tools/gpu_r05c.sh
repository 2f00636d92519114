#!/bin/bash
# r05c: DeMo encode with the next chunk's first half prefetched (GA_DW_PF variant) vs the
# in-tree library: parity of the variant (DeMo kernel tests through GYM_AMD_LIB), then
# interleaved timing of both builds in one process (tools/exp_demo_ablate.py).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/build/libgym_amd_dwpf.so
GYM_AMD_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -k "demo" -x -q --timeout 240 --timeout-method thread > $O/tests_variant.log 2>&1 || { echo "VARIANT TESTS FAILED"; tail -30 $O/tests_variant.log; exit 1; }
tail -2 $O/tests_variant.log
timeout -k 10 300 python tools/exp_demo_ablate.py --codec 3 gym_amd/_lib/libgym_amd.so $V > $O/ab_encode.txt 2>&1 || { echo "AB FAILED"; tail -20 $O/ab_encode.txt; exit 1; }
cat $O/ab_encode.txt
timeout -k 10 300 python tools/exp_demo_ablate.py --codec 3 $V gym_amd/_lib/libgym_amd.so > $O/ab_encode2.txt 2>&1 || { echo "AB2 FAILED"; tail -20 $O/ab_encode2.txt; exit 1; }
cat $O/ab_encode2.txt
