set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# the round's final suite + default line (tools/gpu_full.sh), then config 3 with / without the unused run permutation (fillall)
bash tools/gpu_full.sh &&
timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/u_server.json 2> gpurun_out/u.err &&
EVM_LIB_PATH=_var/fillall/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/u_server_fillall.json 2>> gpurun_out/u.err
