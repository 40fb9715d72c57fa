#!/bin/bash
# Round-2 session A: the new parity tests first, then the full GPU suite, then the benches.
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_apply_stored.py tests/test_gpu_server_atomic.py \
  tests/test_gpu_dist_select.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?
echo "new tests rc=$rc"; tail -15 gpurun_out/pytest_new.log
if fatal $rc; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest.log
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u bench.py --workload server --steps 5 --warmup 2 > gpurun_out/bench_server.json \
  2> gpurun_out/bench_server.err
rc=$?
echo "bench server rc=$rc"; cat gpurun_out/bench_server.json; tail -3 gpurun_out/bench_server.err
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u bench.py --workload server --steps 5 --warmup 2 --zipf 1.2 > gpurun_out/bench_server_zipf.json \
  2> gpurun_out/bench_server_zipf.err
rc=$?
echo "bench server zipf rc=$rc"; cat gpurun_out/bench_server_zipf.json; tail -3 gpurun_out/bench_server_zipf.err
exit $rc
