#!/bin/bash
# Round-2 session B: config-1 parity tests, then the full default bench line.
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_config1.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_c1.log 2>&1
rc=$?
echo "config1 tests rc=$rc"; tail -5 gpurun_out/pytest_c1.log
if fatal $rc; then exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_full.json; tail -5 gpurun_out/bench_full.err
exit $rc
