#!/bin/bash
# Timing-consistency check: bench (HIP events) vs rocprofv3 kernel trace on one box.
O=$GRAFT_REPO_ROOT/gpurun_out/var
mkdir -p $O
export TMPDIR=/tmp
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print('bench kernel_ms',d['roofline']['kernel_ms'],'step_ms',d['ms_per_step'],'traffic',d['roofline']['traffic'])" $1; }
timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline > $O/b1.json 2> $O/b1.err || { tail -20 $O/b1.err; exit 1; }
show $O/b1.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-extras --no-cpu-baseline > $O/p.json 2> $O/p.err || { tail -20 $O/p.err; exit 1; }
show $O/p.json
grep diloco $O/prof/run_kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f1-3
timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline > $O/b3.json 2> $O/b3.err || { tail -20 $O/b3.err; exit 1; }
show $O/b3.json
ONLY_DILOCO=1 timeout -k 10 100 ./build/ubench_stream
