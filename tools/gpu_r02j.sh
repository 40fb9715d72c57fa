#!/bin/bash
# dist ABI (packed wire) + napi + config4c bench at world 1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_abi.py tests/test_gpu_napi.py tests/test_gpu_dist_select.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_j.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/pytest_j.log
if fatal $rc; then exit $rc; fi
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --shape config4c --steps 10 --warmup 2 --cpu-seconds 0 --extra 0 \
  > gpurun_out/bench_4c.json 2> gpurun_out/bench_4c.err
rc=$?
echo "bench 4c rc=$rc"; python3 -c "
import json;d=json.load(open('gpurun_out/bench_4c.json'));print(d['ms_per_step'], d['route']); print(list(d['pipeline']['kernels_ms_per_step'].items())[:10])"
exit $rc
