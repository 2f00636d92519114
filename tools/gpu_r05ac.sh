set -e
mkdir -p gpurun_out/r05ac
export PYTHONUNBUFFERED=1
timeout -k 10 800 python -u tools/exp_diloco_replica_placement.py 4 on,20 > gpurun_out/r05ac/candidates_12_vs_20.txt 2> gpurun_out/r05ac/err.txt
