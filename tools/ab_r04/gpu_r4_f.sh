set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# k_svo_b with 4 rows / leaves' loads in flight per thread vs 1: reingest (config 3), config-5 shape, config 4
timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/f_server.json 2> gpurun_out/f.err &&
EVM_LIB_PATH=_var/svb1/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/f_server_b1.json 2>> gpurun_out/f.err &&
timeout -k 10 300 python -u bench.py --workload config5shape --steps 5 --warmup 1 > gpurun_out/f_c5s.json 2>> gpurun_out/f.err &&
EVM_LIB_PATH=_var/svb1/libevm.so timeout -k 10 300 python -u bench.py --workload config5shape --steps 5 --warmup 1 > gpurun_out/f_c5s_b1.json 2>> gpurun_out/f.err
