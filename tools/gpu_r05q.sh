#!/bin/bash
# r05q: the replica-loop DiLoCo relocation test, then the driver's N > 1 bench form
# (torchrun around bench.py, 2 gloo ranks sharing the GPU; rank 0 times the CPU baseline first).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_replica.py -k "relocation or vmap" -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
GA_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_gloo2_torchrun.json 2> $O/bench_gloo2_torchrun.err || { echo "TORCHRUN REHEARSAL FAILED"; tail -20 $O/bench_gloo2_torchrun.err; exit 1; }
tail -c 400 $O/bench_gloo2_torchrun.json
