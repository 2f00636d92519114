#!/bin/bash
# r03o: AdamW + clip with device-scope (sc1) buffer stores (build variant adamsc1): parity under the
# variant, then bench.py --only adamw interleaved against the in-tree library.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03o
mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/build/libgym_amd_adamsc1.so
GYM_AMD_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_optim.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for L in base adamsc1; do
    if [ $L = base ]; then LP=""; else LP=$V; fi
    GYM_AMD_LIB=$LP timeout -k 10 200 python bench.py --only adamw --steps 20 --warmup 3 > $O/ad_${L}_$r.json 2> $O/ad_${L}_$r.err || { echo "ADAM $L FAILED"; tail -20 $O/ad_${L}_$r.err; exit 1; }
    echo "$L run $r $(grep '^{' $O/ad_${L}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("kernel_ms"), d.get("kernel_frac_hbm"))')"
  done
done
echo DONE
