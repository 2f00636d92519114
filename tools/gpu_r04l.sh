#!/bin/bash
# r04l: optimizer + DiLoCo GPU tests with the placement probes; AdamW / DiLoCo bench lines, 2 processes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "optim or replica or placed or diloco or trainer or dropin" > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for p in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --only adamw > $O/adamw_p$p.json 2> $O/adamw_p$p.err || { echo "ADAMW $p FAILED"; tail -20 $O/adamw_p$p.err; exit 1; }
  cat $O/adamw_p$p.json
done
echo DONE
