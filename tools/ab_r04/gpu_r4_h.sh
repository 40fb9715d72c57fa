set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
# the async status record landed by a kernel (EVM_INFO_KERNEL=1) vs the runtime's copy: async tests + config 2 A/B
EVM_LIB_PATH=_var/infok/libevm.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_async.py tests/test_gpu_tcpath.py tests/test_gpu_apply.py > gpurun_out/t_h.log 2>&1
rc=$?; ok $rc || exit $rc
timeout -k 10 200 python -u bench.py --workload client --steps 30 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/h_c2.json 2> gpurun_out/h.err &&
EVM_LIB_PATH=_var/infok/libevm.so timeout -k 10 200 python -u bench.py --workload client --steps 30 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/h_c2_infok.json 2>> gpurun_out/h.err &&
timeout -k 10 200 python -u bench.py --workload client --steps 30 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/h_c2_again.json 2>> gpurun_out/h.err &&
EVM_LIB_PATH=_var/infok/libevm.so timeout -k 10 200 python -u bench.py --workload client --steps 30 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/h_c2_infok_again.json 2>> gpurun_out/h.err
