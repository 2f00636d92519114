#!/bin/bash
# r03c: decode with the cheaper sign / collision-only divisions (parity + timing),
# SQ counters of the loader/consumer DeMo kernels and the reference-draw SPARTA
# kernels, and the forced-exchange SPARTA step's kernel breakdown.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "demo" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
MODES="demo_encode demo_decode8 demo_decode1" TAG=r03c/ab bash tools/ab_demo_lc.sh || exit 1
PMC_TRAFFIC=0 PMC_EXTRA="SQ_VALU_MFMA_COEXEC_CYCLES" bash tools/pmc_round.sh r03c/pmc demo_encode demo_decode8 torch_draw sparta_torch > $O/pmc.log 2>&1 || { echo "PMC FAILED"; tail -30 $O/pmc.log; exit 1; }
grep -E "^void|SQ_INSTS_VALU per|SQ_INSTS_MFMA per|wave-cycle|COEXEC|SQ_VALU_MFMA_BUSY|SQ_ACTIVE_INST_VALU|effective clock|wall_us|SQ_WAVES|SQ_INSTS_VALU  " $O/pmc.log | head -60
GA_SP_SELECT1=0 GA_BENCH_FORCE_EXCHANGE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/spx -o run --output-format csv -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 bench.py --only sparta --steps 20 --warmup 3 > $O/spx.log 2>&1 || { echo "SPX PROF FAILED"; tail -20 $O/spx.log; exit 1; }
python tools/prof_summary.py $O/spx/run_kernel_stats.csv "forced-exchange SPARTA K=32 step (three-pass select), rocprofv3 --kernel-trace --stats" > $O/spx_stats.txt; head -20 $O/spx_stats.txt
rm -f $O/spx/run_kernel_trace.csv
echo DONE
