set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# scans with 16-B accesses, four tiles per workgroup: the whole GPU suite on it, then server A/B
# against the LDS-transposed three launches (scan3) and the one-pass look-back (scanlb)
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/o_pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/o_server.json 2> gpurun_out/o.err &&
EVM_LIB_PATH=_var/scan3/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/o_server_scan3.json 2>> gpurun_out/o.err &&
EVM_LIB_PATH=_var/scanlb/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/o_server_scanlb.json 2>> gpurun_out/o.err &&
timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/o_server2.json 2>> gpurun_out/o.err
