set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# small scans of one length in one launch (per-owner plan counts, per-segment rows / leaves): the whole GPU suite,
# smoke(), then config 3 and the config-5 shape
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v_pytest.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/v_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/v_server.json 2> gpurun_out/v.err &&
timeout -k 10 300 python -u bench.py --workload config5shape --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/v_c5.json 2>> gpurun_out/v.err &&
timeout -k 10 400 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/v_server2.json 2>> gpurun_out/v.err
