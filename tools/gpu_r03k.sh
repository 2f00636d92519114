#!/bin/bash
# r03k: SPARTA engine tests (overflow lag), forced-exchange step timing after the flag-poll change,
# store-policy / LDS-DMA streaming ubench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_rccl.py -x -v --timeout 120 --timeout-method thread -k "sparta or rccl" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  GA_BENCH_FORCE_EXCHANGE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --only sparta --steps 20 --warmup 3 > $O/sp_$r.json 2> $O/sp_$r.err || { echo "SPARTA FX FAILED"; tail -20 $O/sp_$r.err; exit 1; }
  echo "forced-exchange run $r $(grep '^{' $O/sp_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("kernel_ms"))')"
done
timeout -k 10 150 ./tools/ubench_ldsdma > $O/ubench_ldsdma2.txt 2>&1 || { echo "UBENCH FAILED"; tail -5 $O/ubench_ldsdma2.txt; exit 1; }
cat $O/ubench_ldsdma2.txt
echo DONE
