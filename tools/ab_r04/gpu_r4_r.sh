set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# empty-store commit by a one-wave-per-segment copy: the whole GPU suite, then config 3 / config-5 shape A/B (nocopy = k_svo_b<false>)
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r_pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/r_server.json 2> gpurun_out/r.err &&
EVM_LIB_PATH=_var/nocopy/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/r_server_nocopy.json 2>> gpurun_out/r.err &&
timeout -k 10 300 python -u bench.py --workload server --zipf 1.2 --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/r_c5.json 2>> gpurun_out/r.err &&
EVM_LIB_PATH=_var/nocopy/libevm.so timeout -k 10 300 python -u bench.py --workload server --zipf 1.2 --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/r_c5_nocopy.json 2>> gpurun_out/r.err
