set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_strategies.py tests/test_gpu_replica.py -x -v --timeout 120 --timeout-method thread -k "bernoulli or pack_mask or packed or sparta" > gpurun_out/bern_tests.log 2>&1 || { tail -30 gpurun_out/bern_tests.log; exit 1; }
tail -3 gpurun_out/bern_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/bench_u.json 2>gpurun_out/bench_u.err || { tail -20 gpurun_out/bench_u.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_u.json'))
print(d['ms_per_step'], d['roofline']['frac']); print(d['extras']['sparta_k32_torch_mask']); print(d['extras']['sparta_k32'])"
