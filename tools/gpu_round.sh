#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel stats, PMC traffic passes.
# Usage (via gpurun): bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -30 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > $O/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $O/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --no-extras --no-cpu-baseline --no-pmc --steps 3 --warmup 1 > $O/pmc_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; tail -20 $O/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --no-extras --no-cpu-baseline --no-pmc --steps 3 --warmup 1 > $O/pmc_write.log 2>&1 || { echo "PMC WRITE FAILED"; tail -20 $O/pmc_write.log; exit 1; }
grep '^{"metric"' $O/prof.log > $O/bench_under_rocprof.json || echo "no bench line in prof.log"
python tools/prof_summary.py $O/prof/run_kernel_stats.csv "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc (box $TAG)" > $O/rocprof_stats.txt
rm -f $O/prof/run_kernel_trace.csv
python tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write diloco_outer $O/pmc_traffic_diloco.json 9958072320 > $O/pmc_traffic.log 2>&1 || echo "PMC SUMMARY FAILED"
# multi-GPU code paths on this one GPU: the whole bench under a world-1 RCCL group with every
# exchange forced (rehearsal), and 2 ranks over gloo sharing the GPU (REHEARSE=0 skips both)
if [ "${REHEARSE:-1}" != "0" ]; then
  GA_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29613 bench.py --steps 10 --warmup 2 > $O/bench_rccl1_rehearsal.json 2> $O/bench_rccl1_rehearsal.err || { echo "RCCL1 REHEARSAL FAILED"; tail -20 $O/bench_rccl1_rehearsal.err; exit 1; }
  GA_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_gloo2_rehearsal.json 2> $O/bench_gloo2_rehearsal.err || { echo "GLOO2 REHEARSAL FAILED"; tail -20 $O/bench_gloo2_rehearsal.err; exit 1; }
  tail -c 400 $O/bench_gloo2_rehearsal.json
fi
# the driver's N > 1 form (torchrun around bench.py; rank 0 times the CPU baseline first; TORCHRUN=1)
if [ "${TORCHRUN:-0}" = "1" ]; then
  GA_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_gloo2_torchrun.json 2> $O/bench_gloo2_torchrun.err || { echo "GLOO2 TORCHRUN REHEARSAL FAILED"; tail -20 $O/bench_gloo2_torchrun.err; exit 1; }
  tail -c 300 $O/bench_gloo2_torchrun.json
fi
echo DONE
