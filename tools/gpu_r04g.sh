#!/bin/bash
# r04g: replica tests (FedAvg islands) on the GPU; DeMo delta-placement experiment
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "replica or gpu_optim" > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python tools/exp_demo_placement.py > $O/demo_placement.txt 2>&1 || { echo "DEMO PLACEMENT FAILED"; tail -20 $O/demo_placement.txt; exit 1; }
cat $O/demo_placement.txt
echo DONE
