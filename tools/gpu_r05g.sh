#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05g
mkdir -p $O
timeout -k 10 300 ./tools/ubench_demo_occupancy > $O/occupancy.txt 2>&1 || { echo "UBENCH FAILED"; tail -20 $O/occupancy.txt; exit 1; }
cat $O/occupancy.txt
