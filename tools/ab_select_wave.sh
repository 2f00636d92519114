#!/bin/bash
# Same-box A/B of the exchange path's select kernel (VARIANTS: base = gym_amd/_lib,
# others = build/libgym_amd_<V>.so) under a world-1 RCCL group with the exchange
# forced (bench.py --only sparta: select + all-reduce + scatter, K = 32, 124M).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_sel
VARIANTS=${VARIANTS:-"base nows"}
port=29701
for r in 1 2 3; do
  for V in $VARIANTS; do
    L=$GRAFT_REPO_ROOT/build/libgym_amd_$V.so; [ $V = base ] && L=$GRAFT_REPO_ROOT/gym_amd/_lib/libgym_amd.so
    port=$((port+1))
    GYM_AMD_LIB=$L GA_BENCH_FORCE_EXCHANGE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --steps 20 --warmup 3 --only sparta --no-cpu-baseline --no-pmc > gpurun_out/ab_sel/${V}_$r.txt 2>&1 || { tail -5 gpurun_out/ab_sel/${V}_$r.txt; exit 1; }
    echo "$V $(grep '^{' gpurun_out/ab_sel/${V}_$r.txt | tail -1 | cut -c1-200)"
  done
done
