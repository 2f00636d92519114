#!/bin/bash
# r03s: the full world-1 RCCL forced-exchange bench rehearsal with leg progress and a stack
# watchdog, to locate the r03q hang.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03s
mkdir -p $O
export TMPDIR=/tmp
GA_BENCH_WATCHDOG=45 GA_BENCH_FORCE_EXCHANGE=1 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29631 bench.py --steps 10 --warmup 2 > $O/rehearsal.json 2> $O/rehearsal.err
rc=$?
grep -E "^\[bench\]|File|Thread|Current" $O/rehearsal.err | head -80
echo "rc=$rc"
tail -c 300 $O/rehearsal.json
echo DONE
