#!/bin/bash
# r05p: DiLoCo placement with the replica-set stage -- GPU tests touching placement / DiLoCo /
# the fused AdamW / replica mode, then the headline across fresh processes, stage on vs off.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_replica.py tests/test_gpu_optim.py tests/test_gpu_strategies.py -k "placement or diloco or replica or adam" -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python -u tools/exp_diloco_replica_placement.py 4 > $O/procs.txt 2>&1 || { echo "EXP FAILED"; tail -20 $O/procs.txt; exit 1; }
cat $O/procs.txt
