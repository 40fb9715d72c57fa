set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# small scans (<= 64 tiles) in one launch by look-back: the whole GPU suite, then A/B (scanbig = three launches for every scan);
# then k_seg_key messages per thread 8 / 2 (sk8, sk2) against 4
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/t_server.json 2> gpurun_out/t.err &&
EVM_LIB_PATH=_var/scanbig/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/t_server_big.json 2>> gpurun_out/t.err &&
timeout -k 10 300 python -u bench.py --workload config5shape --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/t_c5.json 2>> gpurun_out/t.err &&
EVM_LIB_PATH=_var/scanbig/libevm.so timeout -k 10 300 python -u bench.py --workload config5shape --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/t_c5_big.json 2>> gpurun_out/t.err &&
timeout -k 10 300 python -u bench.py --workload config4 --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/t_c4.json 2>> gpurun_out/t.err &&
EVM_LIB_PATH=_var/scanbig/libevm.so timeout -k 10 300 python -u bench.py --workload config4 --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/t_c4_big.json 2>> gpurun_out/t.err &&
EVM_LIB_PATH=_var/sk8/libevm.so timeout -k 10 300 python -u bench.py --workload config5shape --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/t_c5_sk8.json 2>> gpurun_out/t.err &&
EVM_LIB_PATH=_var/sk2/libevm.so timeout -k 10 300 python -u bench.py --workload config5shape --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/t_c5_sk2.json 2>> gpurun_out/t.err
