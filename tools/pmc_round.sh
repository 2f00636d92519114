#!/bin/bash
# rocprofv3 PMC passes, one kernel family per run (tools/prof_kernels.py):
# HBM traffic (FETCH_SIZE, WRITE_SIZE: separate passes) and two SQ passes
# (wave-cycle split, instruction mix, LDS, MFMA busy).  Each pass under its own
# time limit; the script stops at the first failure.
# Usage (via gpurun): bash tools/pmc_round.sh <tag> <mode> [<mode> ...]
set -o pipefail
TAG=$1
shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
PASSES=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
)
# PMC_TRAFFIC=0: skip the FETCH_SIZE / WRITE_SIZE passes (SQ passes only)
if [ "${PMC_TRAFFIC:-1}" != "0" ]; then PASSES=("FETCH_SIZE" "WRITE_SIZE" "${PASSES[@]}"); fi
# PMC_EXTRA: one more pass (e.g. "SQ_VALU_MFMA_COEXEC_CYCLES"), allowed to fail
EXTRA=${PMC_EXTRA:-}
for MODE in "$@"; do
  timeout -k 10 120 python3 tools/prof_kernels.py $MODE 10 > $O/${MODE}_time.json 2> $O/${MODE}_time.err || { echo "TIME $MODE FAILED"; tail -20 $O/${MODE}_time.err; exit 1; }
  cat $O/${MODE}_time.json
  i=0
  for P in "${PASSES[@]}"; do
    D=$O/${MODE}_p$i
    timeout -s KILL 120 rocprofv3 --pmc $P -d $D -o run --output-format csv -- python3 tools/prof_kernels.py $MODE 5 > $D.log 2>&1 || { echo "PMC $MODE pass $i FAILED"; tail -20 $D.log; exit 1; }
    python3 tools/pmc_kernels.py --filter $D ga:: || { echo "FILTER $MODE FAILED"; exit 1; }
    i=$((i+1))
  done
  if [ -n "$EXTRA" ]; then
    D=$O/${MODE}_p$i
    if timeout -s KILL 120 rocprofv3 --pmc $EXTRA -d $D -o run --output-format csv -- python3 tools/prof_kernels.py $MODE 5 > $D.log 2>&1; then
      python3 tools/pmc_kernels.py --filter $D ga:: || echo "FILTER EXTRA FAILED"
    else
      echo "PMC EXTRA ($EXTRA) failed for $MODE (tolerated)"; tail -3 $D.log; rm -rf $D
    fi
  fi
  python3 tools/pmc_kernels.py "$O/${MODE}_p*/run_counter_collection.csv" ga:: > $O/${MODE}_pmc.txt 2>&1 || echo "SUMMARY $MODE FAILED"
  cat $O/${MODE}_pmc.txt
done
echo DONE
