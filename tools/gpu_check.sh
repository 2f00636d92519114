#!/bin/bash
# A focused GPU check: the selected GPU tests, then bench.py --only legs.
# Usage (via gpurun): bash tools/gpu_check.sh <tag> "<pytest selection>" "<only leg> [<only leg> ...]"
set -o pipefail
TAG=$1
SEL=$2
LEGS=$3
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$SEL" ]; then
  eval timeout -k 10 900 python -u -m pytest $SEL -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
for leg in $LEGS; do
  timeout -k 10 300 python bench.py --only $leg > $O/only_$leg.json 2> $O/only_$leg.err || { echo "LEG $leg FAILED"; tail -20 $O/only_$leg.err; exit 1; }
  cat $O/only_$leg.json
done
echo DONE
