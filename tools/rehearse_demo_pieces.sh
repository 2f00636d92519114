set -o pipefail
cd $GRAFT_REPO_ROOT
for P in 1 2 3 4; do
  for r in 1 2; do
    GA_DEMO_PIECES=$P GA_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29550+P*2+r)) bench.py --gpus 1 --steps 10 --warmup 2 --only demo > gpurun_out/reh_demo_$P_$r.json 2>/dev/null || exit 1
    python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('pieces', sys.argv[2], 'one-exchange', d['ms_per_step'], 'pipelined', d['ms_per_step_pipelined'])" gpurun_out/reh_demo_$P_$r.json $P
  done
done
