#!/bin/bash
# r03l: sc1 (device-scope) buffer stores in the DiLoCo kernel: parity, same-box interleaved A/B
# (GA_STORE_SC1=0/1), the bench headline per mode, and the store-policy ubench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -x -v --timeout 120 --timeout-method thread -k "diloco or mean or replica" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for V in 0 1; do
    GA_STORE_SC1=$V timeout -k 10 120 python tools/prof_kernels.py diloco 20 > $O/dl_${V}_$r.txt 2>&1 || { echo "DILOCO $V FAILED"; tail -5 $O/dl_${V}_$r.txt; exit 1; }
    echo "SC1=$V run $r $(grep '^{' $O/dl_${V}_$r.txt)"
  done
done
for V in 0 1; do
  GA_STORE_SC1=$V timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline --no-pmc > $O/bench_$V.json 2> $O/bench_$V.err || { echo "BENCH $V FAILED"; tail -20 $O/bench_$V.err; exit 1; }
  echo "SC1=$V bench $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['kernel_ms'], r['frac'], r['copy_GBps'], r['frac_of_copy'])" $O/bench_$V.json)"
done
timeout -k 10 200 ./tools/ubench_ldsdma > $O/ubench.txt 2>&1 || { echo "UBENCH FAILED"; tail -5 $O/ubench.txt; exit 1; }
grep -E "copy|dl" $O/ubench.txt
echo DONE
