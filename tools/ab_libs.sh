#!/bin/bash
# Same-box A/B of several library variants (build/libgym_amd_<name>.so, `make variant`)
# against the in-tree library: interleaved processes of tools/prof_kernels.py per mode.
# Usage (via gpurun): VNAMES="a b" MODES="sparta_torch" TAG=r04o/ab bash tools/ab_libs.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_libs}
mkdir -p $O
for r in 1 2 3; do
  for V in base $VNAMES; do
    line="$V run $r"
    for M in $MODES; do
      if [ $V = base ]; then L=""; else L=$GRAFT_REPO_ROOT/build/libgym_amd_$V.so; fi
      GYM_AMD_LIB=$L timeout -k 10 120 python tools/prof_kernels.py $M 20 > $O/${M}_${V}_$r.txt 2>&1 || { echo "$M $V FAILED"; tail -5 $O/${M}_${V}_$r.txt; exit 1; }
      line="$line $M $(python -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]['ms'])" $O/${M}_${V}_$r.txt)"
    done
    echo $line
  done
done
