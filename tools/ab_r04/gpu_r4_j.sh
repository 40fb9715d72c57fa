set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
# K5's batched stored-row loads: the server suites, then reingest A/B
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_server.py tests/test_gpu_server_segments.py tests/test_gpu_config3_oracle.py > gpurun_out/t_j.log 2>&1
rc=$?; ok $rc || exit $rc
timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/j_server.json 2> gpurun_out/j.err &&
EVM_LIB_PATH=_var/sb1/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/j_server_sb1.json 2>> gpurun_out/j.err
