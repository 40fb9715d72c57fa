set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# one-pass look-back scan: the whole GPU suite on it, then server / config-5 shape A/B against the three-launch scan
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/n_pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/n_server.json 2> gpurun_out/n.err &&
EVM_LIB_PATH=_var/scan3/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/n_server_scan3.json 2>> gpurun_out/n.err &&
timeout -k 10 300 python -u bench.py --workload server --zipf 1.2 --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/n_c5.json 2>> gpurun_out/n.err &&
EVM_LIB_PATH=_var/scan3/libevm.so timeout -k 10 300 python -u bench.py --workload server --zipf 1.2 --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/n_c5_scan3.json 2>> gpurun_out/n.err
