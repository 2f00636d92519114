#!/bin/bash
# SPARTA exchange-path select: parity, same-box A/B of the one-pass select (GA_SP_SELECT1=1)
# against the three passes, and the
# forced-exchange step's kernel breakdown.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-select1_ab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "sparta" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for V in 0 1; do
    GA_SP_SELECT1=$V GA_BENCH_FORCE_EXCHANGE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --only sparta --steps 20 --warmup 3 > $O/sp_${V}_$r.json 2> $O/sp_${V}_$r.err || { echo "SPARTA FX $V FAILED"; tail -20 $O/sp_${V}_$r.err; exit 1; }
    echo "SELECT1=$V run $r $(grep '^{' $O/sp_${V}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("kernel_ms"))')"
  done
done
for V in 0 1; do
  GA_SP_SELECT1=$V GA_BENCH_FORCE_EXCHANGE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/spx$V -o run --output-format csv -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 bench.py --only sparta --steps 20 --warmup 3 > $O/spx$V.log 2>&1 || { echo "SPX PROF FAILED"; tail -20 $O/spx$V.log; exit 1; }
  python tools/prof_summary.py $O/spx$V/run_kernel_stats.csv "forced-exchange SPARTA K=32 step, GA_SP_SELECT1=$V, rocprofv3 --kernel-trace --stats" > $O/spx${V}_stats.txt; head -14 $O/spx${V}_stats.txt
  rm -f $O/spx$V/run_kernel_trace.csv
done
echo DONE
