#!/bin/bash
# Same-box A/B of the DeMo encode's 64x64-chunk kernels: all-in-one (GA_DEMO_ENCODE_LC=0)
# vs loader/consumer (1), interleaved runs of tools/prof_kernels.py demo_encode.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_demo_lc}
mkdir -p $O
for r in 1 2 3; do
  for V in 0 1; do
    GA_DEMO_ENCODE_LC=$V timeout -k 10 120 python tools/prof_kernels.py demo_encode 20 > $O/enc_${V}_$r.txt 2>&1 || { echo "LC=$V FAILED"; tail -5 $O/enc_${V}_$r.txt; exit 1; }
    echo "LC=$V run $r $(grep '^{' $O/enc_${V}_$r.txt)"
  done
done
