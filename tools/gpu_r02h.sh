#!/bin/bash
# server: key-range segments (tests + config 3/5 benches)
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_server_segments.py tests/test_gpu_server.py tests/test_gpu_server_atomic.py tests/test_gpu_adversarial.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_h.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -15 gpurun_out/pytest_h.log
if fatal $rc; then exit $rc; fi
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload server --zipf 1.2 --steps 5 --warmup 2 --cpu-seconds 0 \
  > gpurun_out/bench_z.json 2> gpurun_out/bench_z.err
rc=$?
echo "bench zipf rc=$rc"; python3 -c "
import json;d=json.load(open('gpurun_out/bench_z.json'));print(d['ms_per_step'], d['value']/1e9, d['roofline']['kernel'], d['roofline']['frac']); print(list(d['pipeline']['kernels_ms_per_step'].items())[:16])"
tail -2 gpurun_out/bench_z.err
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 \
  > gpurun_out/bench_s3.json 2> gpurun_out/bench_s3.err
rc=$?
echo "bench config3 rc=$rc"; python3 -c "
import json;d=json.load(open('gpurun_out/bench_s3.json'));print(d['ms_per_step'], d['value']/1e9, d['roofline']['kernel'], d['roofline']['frac']); print(list(d['pipeline']['kernels_ms_per_step'].items())[:16])"
exit $rc
