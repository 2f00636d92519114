set -e
mkdir -p gpurun_out/r05ab
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_replica.py -m gpu > gpurun_out/r05ab/tests.log 2>&1
