set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist_loopback.py tests/test_gpu_dist_split_abi.py tests/test_gpu_napi.py > gpurun_out/t1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload config5 --loopback 2 --c5-owners 20000 --c5-messages 5000000 --steps 3 --warmup 1 > gpurun_out/c5lb.json 2> gpurun_out/c5lb.err &&
timeout -k 10 300 python -u bench.py --workload config5 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/c5w1.json 2> gpurun_out/c5w1.err
