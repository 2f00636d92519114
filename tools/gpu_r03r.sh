#!/bin/bash
# r03r: which leg of the world-1 RCCL forced-exchange bench rehearsal hangs: every extras
# entry on its own under its own time limit, stopping at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03r
mkdir -p $O
export TMPDIR=/tmp
P=29620
for E in diloco sparta_k32 sparta_k32_rows sparta_k32_torch_mask sparta_k32_rows_torch_mask simple_reduce_char_k8 demo_350m inner_adamw_clip_124m; do
  P=$((P+1))
  echo "== $E"
  GA_BENCH_FORCE_EXCHANGE=1 timeout -k 10 90 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $P bench.py --only $E --steps 10 --warmup 2 > $O/$E.json 2> $O/$E.err
  rc=$?
  if [ $rc != 0 ]; then echo "$E rc=$rc"; tail -15 $O/$E.err; exit 1; fi
  tail -c 300 $O/$E.json; echo
done
echo DONE
