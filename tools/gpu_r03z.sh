#!/bin/bash
# r03z: per-kernel PMC passes (HBM traffic + two SQ passes) of the final code's kernel families.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03z
bash tools/pmc_round.sh r03z/pmc demo_encode demo_decode8 sparta_torch torch_draw sparta_rows_torch sparta_elem > gpurun_out/r03z/pmc.log 2>&1 || { echo "PMC FAILED"; tail -30 gpurun_out/r03z/pmc.log; exit 1; }
grep -E "^void|^ga::|HBM read|wave-cycle|SQ_INSTS_VALU per|SQ_INSTS_MFMA per|effective clock|wall_us|LDS bank" gpurun_out/r03z/pmc.log | head -80
echo DONE
