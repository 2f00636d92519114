#!/bin/bash
# r05a: placement opt-out test, then the self-launched 2-rank gloo bench (no torchrun).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -k "placement" -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -8 $O/tests.log
GA_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_gloo2_selflaunch.json 2> $O/bench_gloo2_selflaunch.err || { echo "GLOO2 SELF-LAUNCH FAILED"; tail -30 $O/bench_gloo2_selflaunch.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_gloo2_selflaunch.json'))
print('n_gpus', d['n_gpus'], 'cpu', d['cpu_baseline'] and d['cpu_baseline']['value'], 'launch', d.get('launch'))
print('xgmi', 'xgmi' in d, {k: ('xgmi' in v) for k, v in d.get('extras', {}).items()})
"
echo DONE
