#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/exp_sparta_overlap.py > $O/overlap.json 2> $O/overlap.err || { echo "OVERLAP FAILED"; tail -20 $O/overlap.err; exit 1; }
cat $O/overlap.json
