#!/bin/bash
# N-API (incl. dist) + ragged tc fold + routed client shape at world 1 + config2 bench
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_napi.py tests/test_gpu_dist_abi.py tests/test_gpu_tcpath.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_g.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -15 gpurun_out/pytest_g.log
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u bench.py --shape config4c --steps 10 --warmup 2 --cpu-seconds 0 --extra 0 \
  > gpurun_out/bench_4c.json 2> gpurun_out/bench_4c.err
rc=$?
echo "bench 4c rc=$rc"; tail -1 gpurun_out/bench_4c.json | cut -c1-3000; tail -3 gpurun_out/bench_4c.err
exit $rc
