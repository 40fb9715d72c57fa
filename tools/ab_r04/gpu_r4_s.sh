set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# the empty store's copy writes the tree's prefix XOR (no scan over the leaves): the whole GPU suite, then A/B (nocopy = merge kernel + scan)
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s_pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/s_server.json 2> gpurun_out/s.err &&
EVM_LIB_PATH=_var/nocopy/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/s_server_nocopy.json 2>> gpurun_out/s.err &&
timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/s_server2.json 2>> gpurun_out/s.err &&
timeout -k 10 300 python -u bench.py --workload config5shape --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/s_c5.json 2>> gpurun_out/s.err &&
EVM_LIB_PATH=_var/nocopy/libevm.so timeout -k 10 300 python -u bench.py --workload config5shape --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/s_c5_nocopy.json 2>> gpurun_out/s.err
