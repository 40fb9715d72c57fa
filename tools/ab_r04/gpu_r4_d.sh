set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# the merge's prefix XOR by wave look-back vs the scan; the one-pass selection; the fused segment plan
timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/d_server.json 2> gpurun_out/d.err &&
EVM_LIB_PATH=_var/svb_nopfx/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/d_server_nopfx.json 2>> gpurun_out/d.err &&
timeout -k 10 300 python -u bench.py --workload config5shape --steps 5 --warmup 1 > gpurun_out/d_c5s.json 2>> gpurun_out/d.err &&
EVM_LIB_PATH=_var/svb_nopfx/libevm.so timeout -k 10 300 python -u bench.py --workload config5shape --steps 5 --warmup 1 > gpurun_out/d_c5s_nopfx.json 2>> gpurun_out/d.err &&
timeout -k 10 300 python -u bench.py --workload config4 --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/d_c4.json 2>> gpurun_out/d.err &&
EVM_LIB_PATH=_var/svb_nopfx/libevm.so timeout -k 10 300 python -u bench.py --workload config4 --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/d_c4_nopfx.json 2>> gpurun_out/d.err
