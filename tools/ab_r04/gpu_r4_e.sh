set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# K5 compiled for six waves per SIMD (EVM_K5_WPE=6) vs five: config 3 (+ reingest), config-5 shape, config 4
timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/e_server.json 2> gpurun_out/e.err &&
EVM_LIB_PATH=_var/k5wpe6/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/e_server_w6.json 2>> gpurun_out/e.err &&
timeout -k 10 300 python -u bench.py --workload config5shape --steps 5 --warmup 1 > gpurun_out/e_c5s.json 2>> gpurun_out/e.err &&
EVM_LIB_PATH=_var/k5wpe6/libevm.so timeout -k 10 300 python -u bench.py --workload config5shape --steps 5 --warmup 1 > gpurun_out/e_c5s_w6.json 2>> gpurun_out/e.err &&
timeout -k 10 300 python -u bench.py --workload config4 --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/e_c4.json 2>> gpurun_out/e.err &&
EVM_LIB_PATH=_var/k5wpe6/libevm.so timeout -k 10 300 python -u bench.py --workload config4 --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/e_c4_w6.json 2>> gpurun_out/e.err
