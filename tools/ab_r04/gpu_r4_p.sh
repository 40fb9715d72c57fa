set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# merge rows written once through an LDS source map: the whole GPU suite on it, then reingest A/B (src0 = two-pass writes)
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/p_pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/p_server.json 2> gpurun_out/p.err &&
EVM_LIB_PATH=_var/src0/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/p_server_src0.json 2>> gpurun_out/p.err &&
timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/p_server2.json 2>> gpurun_out/p.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/p_pmc_write" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload server --steps 2 --warmup 1 --cpu-seconds 0 > /dev/null &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/p_pmc_fetch" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload server --steps 2 --warmup 1 --cpu-seconds 0 > /dev/null &&
cd "$GRAFT_REPO_ROOT" && python3 tools/pmc_traffic.py gpurun_out/p_pmc_fetch gpurun_out/p_pmc_write > gpurun_out/p_traffic_config3.json
