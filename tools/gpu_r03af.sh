#!/bin/bash
# r03af: does the DiLoCo kernel's process-to-process spread follow a
# clock, power or temperature change?  8 processes in a row, each timing 1500 back-to-back
# ga_diloco_outer launches (K = 8, GPT-2 124M; ~3 s of kernel), while amd-smi samples the
# GPU's clocks / power / temperature in the background.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03af
mkdir -p $O
export TMPDIR=/tmp
( for i in $(seq 1 400); do echo "T $(date +%s.%N)"; timeout -k 2 10 amd-smi metric -g 0 -c -p -t --json 2>&1; sleep 0.2; done ) > $O/smi.log 2>&1 &
SMI=$!
sleep 2
for r in 1 2 3 4 5 6 7 8; do
  echo "S $r $(date +%s.%N)" >> $O/runs.log
  timeout -k 10 120 python tools/prof_kernels.py diloco 1500 > $O/diloco_$r.txt 2>&1 || { echo "DILOCO $r FAILED"; tail -5 $O/diloco_$r.txt; kill $SMI; exit 1; }
  echo "E $r $(date +%s.%N) $(grep '^{' $O/diloco_$r.txt)" >> $O/runs.log
  tail -1 $O/runs.log
done
sleep 1
kill $SMI
echo DONE
