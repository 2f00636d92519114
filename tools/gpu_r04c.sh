#!/bin/bash
# r04c: DiLoCo placement sweep (tools/ubench_diloco_layout.cpp sweep) in two fresh processes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04c
mkdir -p $O
for p in 1 2; do
  timeout -k 10 150 ./build/ubench_diloco_layout 0 10 sweep > $O/sweep_p$p.txt 2>&1 || { echo "SWEEP $p FAILED"; tail -5 $O/sweep_p$p.txt; exit 1; }
done
paste -d'|' $O/sweep_p1.txt $O/sweep_p2.txt | awk -F'|' '{print $1 "  ||  " substr($2, index($2, ":"))}'
echo DONE
