set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# the 64-KiB cross-cell dedup set (two workgroups per CU): parity, then A/B on the headline
EVM_LIB_PATH=_var/xfsmall/libevm.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_apply.py tests/test_gpu_apply_stored.py > gpurun_out/m_t.log 2>&1 &&
timeout -k 10 200 python -u bench.py --workload client --steps 20 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/m_c2.json 2> gpurun_out/m.err &&
EVM_LIB_PATH=_var/xfsmall/libevm.so timeout -k 10 200 python -u bench.py --workload client --steps 20 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/m_c2_small.json 2>> gpurun_out/m.err &&
timeout -k 10 200 python -u bench.py --workload client --steps 20 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/m_c2b.json 2>> gpurun_out/m.err &&
EVM_LIB_PATH=_var/xfsmall/libevm.so timeout -k 10 200 python -u bench.py --workload client --steps 20 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/m_c2b_small.json 2>> gpurun_out/m.err
