set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# K5's new-leaf searches over the owner's tree codes in LDS (leaflds) vs global: server suites on the variant, then reingest A/B
EVM_LIB_PATH=_var/leaflds/libevm.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_server.py tests/test_gpu_server_segments.py tests/test_gpu_config3_oracle.py tests/test_gpu_scale.py tests/test_gpu_dist_ingest.py tests/test_gpu_adversarial.py > gpurun_out/x_pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/x_server.json 2> gpurun_out/x.err &&
EVM_LIB_PATH=_var/leaflds/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/x_server_leaflds.json 2>> gpurun_out/x.err &&
timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/x_server2.json 2>> gpurun_out/x.err &&
EVM_LIB_PATH=_var/leaflds/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/x_server2_leaflds.json 2>> gpurun_out/x.err
