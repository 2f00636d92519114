#!/bin/bash
# r05f: reduce kernels with finer workgroup chunks for small arenas: parity + the SimpleReduce leg
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "replica_mean or diloco" -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do timeout -k 10 120 python bench.py --only simple --steps 50 > $O/simple_$r.json 2> $O/simple_$r.err || { echo "SIMPLE FAILED"; tail -20 $O/simple_$r.err; exit 1; }; cat $O/simple_$r.json; done
