#!/bin/bash
# r04i: DiLoCo placement map (tools/ubench_diloco_layout.cpp map) in two fresh processes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04i
mkdir -p $O
for p in 1 2; do
  timeout -k 10 250 ./build/ubench_diloco_layout 0 5 map > $O/map_p$p.txt 2>&1 || { echo "MAP $p FAILED"; tail -5 $O/map_p$p.txt; exit 1; }
  cat $O/map_p$p.txt
done
echo DONE
