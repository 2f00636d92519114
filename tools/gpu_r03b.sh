#!/bin/bash
# Round-3 step b: the new DeMo / SPARTA kernels' parity tests, the drop-in replay,
# then same-box A/B timings (DeMo one-wave vs loader/consumer; SPARTA three-pass vs one-pass).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dropin.py -x -v --timeout 120 --timeout-method thread -k "demo or dropin or one_pass or sparta" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
TAG=r03b/ab bash tools/ab_demo_lc.sh || exit 1
for r in 1 2; do
  for V in 0 1; do
    GA_SP_SELECT1=$V GA_BENCH_FORCE_EXCHANGE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --only sparta --steps 20 --warmup 3 > $O/sp_${V}_$r.json 2> $O/sp_${V}_$r.err || { echo "SPARTA FX $V FAILED"; tail -20 $O/sp_${V}_$r.err; exit 1; }
    echo "SELECT1=$V run $r $(cat $O/sp_${V}_$r.json)"
  done
done
echo DONE
