#!/bin/bash
# r03u: persistent pipelined reference-draw SPARTA average (GA_SP_PIPE=1): parity, then the
# same-box interleaved A/B against the wave kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "pipelined or reference_draw or in_kernel" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for V in 0 1; do
    GA_SP_PIPE=$V timeout -k 10 120 python tools/prof_kernels.py sparta_torch 20 > $O/sp_${V}_$r.txt 2>&1 || { echo "SPARTA $V FAILED"; tail -5 $O/sp_${V}_$r.txt; exit 1; }
    echo "PIPE=$V run $r $(grep '^{' $O/sp_${V}_$r.txt)"
  done
done
echo DONE
