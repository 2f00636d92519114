set -e
mkdir -p gpurun_out/r05aa
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_replica.py -k "relocation" -m gpu > gpurun_out/r05aa/tests.log 2>&1
timeout -k 10 300 python -u tools/exp_replica_demo_placement.py 3 > gpurun_out/r05aa/demo_placement.txt 2> gpurun_out/r05aa/demo_placement.err
