#!/bin/bash
# The N-rank bench on this one GPU over gloo, self-launched (`python bench.py --gpus N`):
# every multi-GPU leg at world N (shard plans, 32/N SPARTA nodes, pipelined DeMo, xgmi
# blocks) -- a code-path rehearsal, not an xGMI measurement (the driver's SCALE run is).
# Then the default N=1 bench line.  Usage (via gpurun): bash tools/gpu_rehearse.sh <tag> [N]
set -o pipefail
TAG=${1:-r06a}
N=${2:-8}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
GA_BENCH_BACKEND=gloo GA_BENCH_WATCHDOG=120 timeout -k 10 900 python bench.py --gpus $N --steps 3 --warmup 1 > $O/bench_gloo${N}_selflaunch.json 2> $O/bench_gloo${N}_selflaunch.err || { echo "GLOO$N FAILED"; tail -40 $O/bench_gloo${N}_selflaunch.err; exit 1; }
python tools/check_bench_line.py $O/bench_gloo${N}_selflaunch.json $N || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
python tools/check_bench_line.py $O/bench.json 1 || exit 1
echo DONE
