#!/bin/bash
# r03h: SPARTA kernel tests, one-pass select A/B (two-level look-back, polls every 8 s_sleep units),
# the DeMo memory-pattern ubench (chunk vs row-band access), then the full default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03h
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_select1_ab.sh r03h/sel || exit 1
timeout -k 10 300 ./tools/ubench_demo_mem > $O/ubench_demo_mem.txt 2>&1 || { echo "UBENCH FAILED"; tail -5 $O/ubench_demo_mem.txt; exit 1; }
cat $O/ubench_demo_mem.txt
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -30 $O/bench.err; exit 1; }
tail -c 6000 $O/bench.json
echo DONE
