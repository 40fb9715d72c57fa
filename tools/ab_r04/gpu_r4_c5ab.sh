set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# a test step that only failed asserts (pytest exit 1) lets the benches run; anything else ends the call
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dist_ingest.py > gpurun_out/t_ding.log 2>&1
rc=$?; ok $rc || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist_loopback.py tests/test_gpu_dist_split_abi.py tests/test_gpu_dist_abi.py tests/test_gpu_server_segments.py tests/test_gpu_server.py tests/test_gpu_config3_oracle.py > gpurun_out/t_srv2.log 2>&1
rc=$?; ok $rc || exit $rc
timeout -k 10 200 python -u bench.py --workload client --steps 20 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err &&
EVM_LIB_PATH=_var/tp_pf/libevm.so timeout -k 10 200 python -u bench.py --workload client --steps 20 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/b_c2_pf.json 2>> gpurun_out/b_c2.err &&
EVM_LIB_PATH=_var/xf_nostage/libevm.so timeout -k 10 200 python -u bench.py --workload client --steps 20 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/b_c2_xfns.json 2>> gpurun_out/b_c2.err &&
timeout -k 10 300 python -u bench.py --workload config4 --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/b_c4.json 2> gpurun_out/b_c4.err &&
timeout -k 10 300 python -u bench.py --workload config4 --steps 5 --warmup 1 --cpu-seconds 0 --c4-take > gpurun_out/b_c4_take.json 2>> gpurun_out/b_c4.err
