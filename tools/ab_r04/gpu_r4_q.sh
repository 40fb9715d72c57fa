set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# merge leaves written once through the source map too: server / segment / scale suites, then reingest A/B (rowsonly = leaves in two passes)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_server.py tests/test_gpu_server_segments.py tests/test_gpu_config3_oracle.py tests/test_gpu_scale.py tests/test_gpu_dist_ingest.py > gpurun_out/q_pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/q_server.json 2> gpurun_out/q.err &&
EVM_LIB_PATH=_var/rowsonly/libevm.so timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/q_server_rowsonly.json 2>> gpurun_out/q.err &&
timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/q_server2.json 2>> gpurun_out/q.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/q_pmc_write" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload server --steps 2 --warmup 1 --cpu-seconds 0 > /dev/null &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/q_pmc_fetch" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload server --steps 2 --warmup 1 --cpu-seconds 0 > /dev/null &&
cd "$GRAFT_REPO_ROOT" && python3 tools/pmc_traffic.py gpurun_out/q_pmc_fetch gpurun_out/q_pmc_write > gpurun_out/q_traffic_config3.json
