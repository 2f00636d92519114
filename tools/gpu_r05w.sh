#!/bin/bash
# r05w: SPARTA averages divide by a power-of-two node count as an exact reciprocal multiply
# (div_nodes; in-tree) vs build/libgym_amd_base.so: SPARTA GPU tests (bit-exact), then
# interleaved per-kernel timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_strategies.py -k "sparta or torch or bernoulli" -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for V in base new; do
    line="$V run $r"
    for M in sparta_torch sparta_elem; do
      if [ $V = base ]; then L=$GRAFT_REPO_ROOT/build/libgym_amd_base.so; else L=""; fi
      GYM_AMD_LIB=$L timeout -k 10 120 python tools/prof_kernels.py $M 20 > $O/${M}_${V}_$r.txt 2>&1 || { echo "$M $V FAILED"; tail -5 $O/${M}_${V}_$r.txt; exit 1; }
      line="$line $M $(python -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]['ms'])" $O/${M}_${V}_$r.txt)"
    done
    echo $line
  done
done | tee $O/ab.txt
