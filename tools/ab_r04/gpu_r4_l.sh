set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# the merge with fewer workgroups per CU (LDS pad): does reingest's write traffic fit L2 better?
timeout -k 10 400 python -u bench.py --workload server --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/l_server.json 2> gpurun_out/l.err &&
EVM_LIB_PATH=_var/pad40/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/l_server_pad40.json 2>> gpurun_out/l.err &&
EVM_LIB_PATH=_var/pad80/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/l_server_pad80.json 2>> gpurun_out/l.err
