#!/bin/bash
# r03ag: per-launch drift of the DiLoCo kernel over a sustained run (3000 back-to-back
# launches, ~6 s), with amd-smi sampling socket power / clocks / HBM temperature; then a
# bench.py run right after a 20 s idle pause.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ag
mkdir -p $O
export TMPDIR=/tmp
( for i in $(seq 1 300); do echo "T $(date +%s.%N)"; timeout -k 2 10 amd-smi metric -g 0 -c -p -t --json 2>&1; sleep 0.2; done ) > $O/smi.log 2>&1 &
SMI=$!
for r in 1 2; do
  echo "S $r $(date +%s.%N)" >> $O/runs.log
  GA_PROF_DUMP=$O/launches_$r.txt timeout -k 10 120 python tools/prof_kernels.py diloco 3000 > $O/diloco_$r.txt 2>&1 || { echo "DILOCO $r FAILED"; tail -5 $O/diloco_$r.txt; kill $SMI; exit 1; }
  echo "E $r $(date +%s.%N) $(grep '^{' $O/diloco_$r.txt)" >> $O/runs.log
  tail -1 $O/runs.log
done
sleep 20
echo "S bench $(date +%s.%N)" >> $O/runs.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --only diloco > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; kill $SMI; exit 1; }
echo "E bench $(date +%s.%N)" >> $O/runs.log
python -c "import json; d=json.load(open('$O/bench.json')); print('bench kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"
kill $SMI
echo DONE
