#!/bin/bash
# r03n: the count pass with the scan folded into its last workgroup: SPARTA parity (every
# select path), then the forced-exchange step A/B (GA_SP_FUSED_SCAN=0/1) with its kernel breakdown.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_rccl.py tests/test_gpu_strategies.py -x -v --timeout 120 --timeout-method thread -k "sparta or rccl" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for V in 0 1; do
    GA_SP_FUSED_SCAN=$V GA_BENCH_FORCE_EXCHANGE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --only sparta --steps 20 --warmup 3 > $O/sp_${V}_$r.json 2> $O/sp_${V}_$r.err || { echo "SPARTA FX $V FAILED"; tail -20 $O/sp_${V}_$r.err; exit 1; }
    echo "FUSED_SCAN=$V run $r $(grep '^{' $O/sp_${V}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("kernel_ms"))')"
  done
done
GA_BENCH_FORCE_EXCHANGE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/spx -o run --output-format csv -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 bench.py --only sparta --steps 20 --warmup 3 > $O/spx.log 2>&1 || { echo "SPX PROF FAILED"; tail -20 $O/spx.log; exit 1; }
python tools/prof_summary.py $O/spx/run_kernel_stats.csv "forced-exchange SPARTA K=32 step, fused count+scan, rocprofv3 --kernel-trace --stats" > $O/spx_stats.txt; head -16 $O/spx_stats.txt
rm -f $O/spx/run_kernel_trace.csv
echo DONE
