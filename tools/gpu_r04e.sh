#!/bin/bash
# r04e: the new bench extras (replica-loop SPARTA step, DeMo 8 distinct sources) and the
# multi-rank xgmi blocks under a world-1 RCCL group (forced exchange) and 2 gloo ranks
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --only sparta_k32_replica_step > $O/replica_step.json 2> $O/replica_step.err || { echo "REPLICA STEP FAILED"; tail -20 $O/replica_step.err; exit 1; }
cat $O/replica_step.json
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --only demo > $O/demo.json 2> $O/demo.err || { echo "DEMO FAILED"; tail -20 $O/demo.err; exit 1; }
cat $O/demo.json
GA_BENCH_FORCE_EXCHANGE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29613 bench.py --steps 5 --warmup 1 > $O/rccl1.json 2> $O/rccl1.err || { echo "RCCL1 FAILED"; tail -20 $O/rccl1.err; exit 1; }
GA_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 2 --steps 3 --warmup 1 > $O/gloo2.json 2> $O/gloo2.err || { echo "GLOO2 FAILED"; tail -20 $O/gloo2.err; exit 1; }
python - <<'PY'
import json
for f in ("rccl1", "gloo2"):
    d = json.load(open(f"gpurun_out/r04e/{f}.json"))
    print(f, "xgmi head:", d.get("xgmi"))
    for k, v in d.get("extras", {}).items():
        x = v.get("xgmi") if isinstance(v, dict) else None
        print(f, k, "xgmi:", x, "error:", v.get("error") if isinstance(v, dict) else None)
PY
echo DONE
