#!/bin/bash
# Same-box A/B of a library variant (build/libgym_amd_$VNAME.so, `make variant`) against the
# in-tree library: interleaved processes of tools/prof_kernels.py per mode.
# Usage (via gpurun): VNAME=demosc1 MODES="demo_encode demo_decode8" TAG=r03m/ab bash tools/ab_lib.sh
# (VNAMES="a b c" compares several variants, each interleaved with the base in every run)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_lib}
mkdir -p $O
for r in 1 2 3; do
  for V in base ${VNAMES:-$VNAME}; do
    line="$V run $r"
    for M in $MODES; do
      if [ $V = base ]; then L=""; else L=$GRAFT_REPO_ROOT/build/libgym_amd_$V.so; fi
      GYM_AMD_LIB=$L timeout -k 10 120 python tools/prof_kernels.py $M 20 > $O/${M}_${V}_$r.txt 2>&1 || { echo "$M $V FAILED"; tail -5 $O/${M}_${V}_$r.txt; exit 1; }
      line="$line $M $(python -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]['ms'])" $O/${M}_${V}_$r.txt)"
    done
    echo $line
  done
done
