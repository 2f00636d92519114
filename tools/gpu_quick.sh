#!/bin/bash
# GPU-box check of a change: the GPU tests (optionally a -k filter), the bench line,
# optional 2-rank gloo rehearsal.  Usage: bash tools/gpu_quick.sh <tag> [pytest -k expr] [rehearse]
set -o pipefail
TAG=${1:-quick}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
fi
tail -2 $O/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
if [ "${3:-}" = rehearse ]; then
  GA_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { echo "REHEARSAL FAILED"; tail -30 $O/bench_gloo2.err; exit 1; }
  cat $O/bench_gloo2.json
fi
echo DONE
