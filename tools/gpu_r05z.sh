#!/bin/bash
# r05z: placement of the set the replica mean averages (MeanReduce._place, ga_probe_mean_placement):
# replica-loop relocation tests, then the 124M x 8 mean in fresh processes with placement on / off.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_replica.py tests/test_gpu_fullsize.py -k "relocation or placement or replicas_match" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
  for mode in on off; do
    if [ $mode = off ]; then E=0; else E=1; fi
    GA_PLACEMENT=$E timeout -k 10 120 python bench.py --only simple_reduce_124m_k8 --no-cpu-baseline --no-pmc > $O/simple_${mode}_$i.json 2> $O/simple_${mode}_$i.err || { echo "BENCH $mode FAILED"; tail -10 $O/simple_${mode}_$i.err; exit 1; }
    python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], d['kernel_ms'], d['kernel_frac_hbm'], d.get('placement'))" $O/simple_${mode}_$i.json $mode
  done
done | tee $O/ab.txt
