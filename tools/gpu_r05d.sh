#!/bin/bash
# r05d: (1) placed-buffer VA ranges vs the caching allocator's segments;
# (2) the whole bench with 8 ranks over gloo sharing this one GPU, self-launched (world-8 code
# paths: shard plans, 32 SPARTA nodes / 8, pipelined DeMo, xgmi blocks -- a rehearsal, not xGMI).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "demo" -x -q --timeout 240 --timeout-method thread > $O/demo_tests.log 2>&1 || { echo "DEMO TESTS FAILED"; tail -30 $O/demo_tests.log; exit 1; }
tail -2 $O/demo_tests.log
GA_BENCH_BACKEND=gloo GA_BENCH_WATCHDOG=120 timeout -k 10 900 python bench.py --gpus 8 --steps 3 --warmup 1 > $O/bench_gloo8_selflaunch.json 2> $O/bench_gloo8_selflaunch.err || { echo "GLOO8 FAILED"; tail -40 $O/bench_gloo8_selflaunch.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_gloo8_selflaunch.json'))
print('n_gpus', d['n_gpus'], 'value', d['value'], 'ms', d['ms_per_step'], 'cpu', d['cpu_baseline'] and d['cpu_baseline']['value'])
print({k: (v.get('error') or v.get('ms_per_step')) for k, v in d.get('extras', {}).items()})
"
echo DONE
