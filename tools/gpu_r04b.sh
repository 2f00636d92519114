#!/bin/bash
# r04b: DiLoCo placement search (tools/ubench_diloco_layout.cpp search): the replica set packed
# at the start of a 24 GiB pool, master/momentum at 40 seeded random offsets; three fresh
# processes with the same seed (same virtual offsets) -- is a fast placement fast in every process?
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04b
mkdir -p $O
for p in 1 2 3; do
  timeout -k 10 100 ./build/ubench_diloco_layout 0 10 search 7 40 > $O/search_p$p.txt 2>&1 || { echo "SEARCH $p FAILED"; tail -5 $O/search_p$p.txt; exit 1; }
  grep -E "^best|^worst" $O/search_p$p.txt | sort | head -8
done
echo DONE
