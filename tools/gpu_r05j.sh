#!/bin/bash
# r05j: replica_forward="vmap" -- GPU tests, then loop vs vmap forward/backward timing
# (tools/exp_replica_vmap.py) on the reference's nanoGPT presets: char-level "small"
# (4 layers, d 128, vocab 65, block 1024, minibatch 16) and GPT-2 124M.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_replica.py -k vmap -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -5 $O/tests.log
timeout -k 10 600 python -u tools/exp_replica_vmap.py 4,128,4,1024,16,8,8,65 4,128,4,1024,16,32,8,65 4,128,4,256,16,32,32,65 4,256,4,128,4,32,32 12,768,12,256,2,32,8 12,768,12,1024,8,32,4 > $O/vmap.txt 2>&1 || { echo "EXP FAILED"; tail -20 $O/vmap.txt; exit 1; }
grep -v amdgpu $O/vmap.txt | grep "{"
