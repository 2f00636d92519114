#!/bin/bash
# Copy one tools/gpu_round.sh session's judged outputs from gpurun_out/<tag>/ into profiles/<tag>_*.
# Usage: bash tools/save_round.sh <tag>
set -e
T=$1
O=gpurun_out/$T
for f in bench.json bench_gloo2_rehearsal.json bench_rccl1_rehearsal.json bench_under_rocprof.json pmc_traffic_diloco.json rocprof_stats.txt smoke.log; do
  [ -f $O/$f ] && cp $O/$f profiles/${T}_$f
done
grep -E "PASSED|FAILED|passed|failed" $O/gpu_tests.log | tail -40 > profiles/${T}_gpu_tests_tail.txt
ls profiles/${T}_*
