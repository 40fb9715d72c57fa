set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
# the small-batch path's multi-workgroup offset scan: its tests, then the config-1 leg A/B (twice each)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_small.py tests/test_gpu_config1.py tests/test_gpu_apply.py > gpurun_out/t_k.log 2>&1
rc=$?; ok $rc || exit $rc
timeout -k 10 200 python -u tools/ab_r04/c1_probe.py > gpurun_out/k_c1.json 2> gpurun_out/k.err &&
EVM_LIB_PATH=_var/smscan1/libevm.so timeout -k 10 200 python -u tools/ab_r04/c1_probe.py > gpurun_out/k_c1_one.json 2>> gpurun_out/k.err &&
timeout -k 10 200 python -u tools/ab_r04/c1_probe.py > gpurun_out/k_c1_b.json 2>> gpurun_out/k.err &&
EVM_LIB_PATH=_var/smscan1/libevm.so timeout -k 10 200 python -u tools/ab_r04/c1_probe.py > gpurun_out/k_c1_one_b.json 2>> gpurun_out/k.err
