set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_core.py tests/test_gpu_server.py tests/test_gpu_scale.py tests/test_gpu_config3_oracle.py tests/test_gpu_dist_split_abi.py > gpurun_out/t_diff.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_r04/diff_sweep.py > gpurun_out/diff_sweep.json 2> gpurun_out/diff_sweep.err &&
EVM_LIB_PATH=_var/diff_r3/libevm.so timeout -k 10 300 python -u tools/ab_r04/diff_sweep.py 0 > gpurun_out/diff_sweep_r3.json 2>> gpurun_out/diff_sweep.err &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcd_new0 -o run -- python3 tools/ab_r04/diff_sweep.py 0 > /dev/null 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcd_new2 -o run -- python3 tools/ab_r04/diff_sweep.py 2 > /dev/null 2>&1 &&
EVM_LIB_PATH=_var/diff_r3/libevm.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcd_r3 -o run -- python3 tools/ab_r04/diff_sweep.py 0 > /dev/null 2>&1
