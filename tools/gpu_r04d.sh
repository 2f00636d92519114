#!/bin/bash
# r04d: new GPU tests (fused AdamW+SPARTA, 350M four-node decode, pruned kernels) and the
# DiLoCo headline with the placement probe in three fresh processes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "adam_sparta or four_nodes or replica or repeated_launches or rows_local_average or gpu_optim" > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
for p in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --only diloco > $O/bench_p$p.json 2> $O/bench_p$p.err || { echo "BENCH $p FAILED"; tail -20 $O/bench_p$p.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_p$p.json'))['roofline']; print('p$p kernel_ms', d['kernel_ms'], 'frac', d['frac'], 'sustained', d['sustained']['kernel_ms'], d['sustained']['frac'], 'placement', d['placement'])"
done
echo DONE
