#!/bin/bash
# r05t: the reference-draw SPARTA step as a producer / consumer workgroup (GA_SP_PC variant,
# build/libgym_amd_sppc.so) vs the in-tree wave-per-tile kernel: SPARTA GPU tests through the
# variant (bit-exact), then interleaved per-kernel timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05t
mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/build/libgym_amd_sppc.so
GYM_AMD_LIB=$V timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_strategies.py -k "sparta or torch" -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for V2 in base pc; do
    line="$V2 run $r"
    for M in sparta_torch probe_philox; do
      if [ $V2 = base ]; then L=""; else L=$V; fi
      GYM_AMD_LIB=$L timeout -k 10 120 python tools/prof_kernels.py $M 20 > $O/${M}_${V2}_$r.txt 2>&1 || { echo "$M $V2 FAILED"; tail -5 $O/${M}_${V2}_$r.txt; exit 1; }
      line="$line $M $(python -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]['ms'])" $O/${M}_${V2}_$r.txt)"
    done
    echo $line
  done
done | tee $O/ab.txt
