#!/bin/bash
# r04h: DiLoCo headline with spaced placement candidates, four fresh processes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04h
mkdir -p $O
export TMPDIR=/tmp
for p in 1 2 3 4; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --only diloco > $O/bench_p$p.json 2> $O/bench_p$p.err || { echo "BENCH $p FAILED"; tail -20 $O/bench_p$p.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_p$p.json'))['roofline']; print('p$p kernel_ms', d['kernel_ms'], 'frac', d['frac'], 'sustained', d['sustained']['kernel_ms'], d['sustained']['frac'], 'placement', d['placement'])"
done
echo DONE
