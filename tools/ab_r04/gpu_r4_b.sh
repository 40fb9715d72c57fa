set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# server (config 3 + reingest) and config-5 shape A/Bs of this round's options
timeout -k 10 300 python -u bench.py --workload config4 --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/b_c4.json 2> gpurun_out/b_c4.err &&
timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/b_server.json 2> gpurun_out/b_server.err &&
EVM_LIB_PATH=_var/svb_nopfx/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/b_server_nopfx.json 2>> gpurun_out/b_server.err &&
EVM_LIB_PATH=_var/nocbase/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/b_server_nocbase.json 2>> gpurun_out/b_server.err &&
timeout -k 10 300 python -u bench.py --workload config5shape --steps 5 --warmup 1 > gpurun_out/b_c5s_base.json 2> gpurun_out/b_c5s.err &&
EVM_LIB_PATH=_var/segnofuse/libevm.so timeout -k 10 300 python -u bench.py --workload config5shape --steps 5 --warmup 1 > gpurun_out/b_c5s_nofuse.json 2>> gpurun_out/b_c5s.err &&
timeout -k 10 300 python -u bench.py --workload config5shape --steps 5 --warmup 1 --radix 2 > gpurun_out/b_c5s_r2.json 2>> gpurun_out/b_c5s.err &&
timeout -k 10 300 python -u bench.py --workload config5shape --steps 5 --warmup 1 --server-path 4 > gpurun_out/b_c5s_p4.json 2>> gpurun_out/b_c5s.err
