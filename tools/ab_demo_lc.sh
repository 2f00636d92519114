#!/bin/bash
# Same-box A/B of the DeMo codec's 64x64-chunk kernels: one wave per chunk
# (GA_DEMO_ENCODE_LC=0 / GA_DEMO_DECODE_LC=0) vs the loader/consumer and
# consumer/updater kernels (1), interleaved runs of tools/prof_kernels.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_demo_lc}
mkdir -p $O
MODES=${MODES:-"demo_encode demo_decode8 demo_decode1"}
for r in 1 2 3; do
  for V in 0 1; do
    line="LC=$V run $r"
    for M in $MODES; do
      GA_DEMO_ENCODE_LC=$V GA_DEMO_DECODE_LC=$V timeout -k 10 120 python tools/prof_kernels.py $M 20 > $O/${M}_${V}_$r.txt 2>&1 || { echo "$M LC=$V FAILED"; tail -5 $O/${M}_${V}_$r.txt; exit 1; }
      line="$line $M $(python -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]['ms'])" $O/${M}_${V}_$r.txt)"
    done
    echo $line
  done
done
