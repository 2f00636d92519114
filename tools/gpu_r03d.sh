#!/bin/bash
# r03d: the round-3 kernels' parity tests (DeMo loader/consumer encode, consumer/updater
# decode, SPARTA one-pass select, drop-in replay), same-box A/B timings of both, the
# SQ counters of the DeMo kernels.  Every GPU step under its own limit, stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dropin.py -x -v --timeout 120 --timeout-method thread -k "demo or dropin or one_pass or sparta" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for V in 0 1; do
    line="ROWS_WAVE=$V run $r"
    for M in sparta_rows sparta_rows_torch; do
      GA_SP_ROWS_WAVE=$V timeout -k 10 120 python tools/prof_kernels.py $M 20 > $O/${M}_${V}_$r.txt 2>&1 || { echo "$M $V FAILED"; tail -5 $O/${M}_${V}_$r.txt; exit 1; }
      line="$line $M $(grep '^{' $O/${M}_${V}_$r.txt)"
    done
    echo $line
  done
done
timeout -k 10 120 python tools/prof_kernels.py probe_rows 20 > $O/probe_rmw.txt 2>&1 && echo "probe rmw $(cat $O/probe_rmw.txt)" || { echo "PROBE FAILED"; tail -5 $O/probe_rmw.txt; exit 1; }
GA_PROBE_WRITE=0 timeout -k 10 120 python tools/prof_kernels.py probe_rows 20 > $O/probe_rd.txt 2>&1 && echo "probe read $(cat $O/probe_rd.txt)" || { echo "PROBE FAILED"; tail -5 $O/probe_rd.txt; exit 1; }
TAG=r03d/ab bash tools/ab_demo_lc.sh || exit 1
for r in 1 2; do
  for V in 0 1; do
    GA_SP_SELECT1=$V GA_BENCH_FORCE_EXCHANGE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --only sparta --steps 20 --warmup 3 > $O/sp_${V}_$r.json 2> $O/sp_${V}_$r.err || { echo "SPARTA FX $V FAILED"; tail -20 $O/sp_${V}_$r.err; exit 1; }
    echo "SELECT1=$V run $r $(cat $O/sp_${V}_$r.json)"
  done
done
PMC_TRAFFIC=0 bash tools/pmc_round.sh r03d/pmc demo_encode demo_decode8 > $O/pmc.log 2>&1 || { echo "PMC FAILED"; tail -30 $O/pmc.log; exit 1; }
grep -E "^void|SQ_INSTS_VALU per|SQ_INSTS_MFMA per|wave-cycle|SQ_VALU_MFMA_BUSY|SQ_ACTIVE_INST_VALU|SQ_WAVES|SQ_LDS_BANK" $O/pmc.log | head -60
echo DONE
