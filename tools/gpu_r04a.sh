#!/bin/bash
# r04a: DiLoCo layout experiment (tools/ubench_diloco_layout.cpp): 4 fresh processes in a row,
# each timing the library kernel under 10 placements interleaved over 3 rounds; then one under
# rocprofv3 --kernel-trace (does the profiler's own allocations shift the placement?), then
# bench.py --only diloco.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04a
mkdir -p $O
export TMPDIR=/tmp
for p in 1 2 3 4; do
  timeout -k 10 60 ./build/ubench_diloco_layout 3 20 > $O/layout_p$p.txt 2>&1 || { echo "LAYOUT $p FAILED"; tail -5 $O/layout_p$p.txt; exit 1; }
  grep -E "round 2" $O/layout_p$p.txt
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- ./build/ubench_diloco_layout 3 20 > $O/layout_rocprof.txt 2>&1 || { echo "ROCPROF FAILED"; tail -5 $O/layout_rocprof.txt; exit 1; }
grep -E "round 2" $O/layout_rocprof.txt
rm -f $O/prof/run_kernel_trace.csv
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --only diloco > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"
echo DONE
