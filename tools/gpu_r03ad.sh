#!/bin/bash
# r03ad: non-temporal grad stores in the multi-source DeMo decode (GA_DEMO_NT_GRAD): parity, then
# same-box interleaved A/B of both decodes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ad
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread -k "demo" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for V in 0 1; do
    line="NT_GRAD=$V run $r"
    for M in demo_decode8 demo_decode1; do
      GA_DEMO_NT_GRAD=$V timeout -k 10 120 python tools/prof_kernels.py $M 20 > $O/${M}_${V}_$r.txt 2>&1 || { echo "$M $V FAILED"; tail -5 $O/${M}_${V}_$r.txt; exit 1; }
      line="$line $M $(python -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]['ms'])" $O/${M}_${V}_$r.txt)"
    done
    echo $line
  done
done
echo DONE
