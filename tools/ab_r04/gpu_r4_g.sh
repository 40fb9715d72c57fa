set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
# narrow routes as three arrays: the dist suites, then config 4; k_svo_b load batching A/B
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist_ingest.py tests/test_gpu_dist_loopback.py tests/test_gpu_dist_split_abi.py tests/test_gpu_dist_abi.py tests/test_gpu_napi.py tests/test_gpu_server.py tests/test_gpu_server_segments.py > gpurun_out/t_g.log 2>&1
rc=$?; ok $rc || exit $rc
timeout -k 10 300 python -u bench.py --workload config4 --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/g_c4.json 2> gpurun_out/g.err &&
timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/g_server.json 2>> gpurun_out/g.err &&
EVM_LIB_PATH=_var/svb1/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/g_server_b1.json 2>> gpurun_out/g.err &&
timeout -k 10 300 python -u bench.py --workload config5shape --steps 5 --warmup 1 > gpurun_out/g_c5s.json 2>> gpurun_out/g.err &&
EVM_LIB_PATH=_var/svb1/libevm.so timeout -k 10 300 python -u bench.py --workload config5shape --steps 5 --warmup 1 > gpurun_out/g_c5s_b1.json 2>> gpurun_out/g.err &&
EVM_LIB_PATH=_var/k5t512/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/g_server_t512.json 2>> gpurun_out/g.err &&
EVM_LIB_PATH=_var/k5t512/libevm.so timeout -k 10 300 python -u bench.py --workload config5shape --steps 5 --warmup 1 > gpurun_out/g_c5s_t512.json 2>> gpurun_out/g.err &&
EVM_LIB_PATH=_var/k5t512/libevm.so timeout -k 10 300 python -u bench.py --workload config4 --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/g_c4_t512.json 2>> gpurun_out/g.err
