#!/bin/bash
# One GPU-box session: parity tests, then the bench (and optional extra steps).
# Each GPU step runs under its own time limit; a fault, abort, segfault or
# time limit (124/134/137/139) ends the script; an ordinary test failure
# (exit 1) still lets the bench run so its numbers come back.
#   bash tools/gpu_run.sh [pytest-args...]
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }

timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
  > gpurun_out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest.log
if fatal $rc; then exit $rc; fi

timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
if fatal $rc; then exit $rc; fi

timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --overlap 0 > gpurun_out/bench_no_overlap.json \
  2> gpurun_out/bench_no_overlap.err
rc=$?
echo "bench (one stream) rc=$rc"; cat gpurun_out/bench_no_overlap.json
if fatal $rc; then exit $rc; fi

timeout -k 10 300 python -u bench.py --workload server --steps 5 --warmup 2 > gpurun_out/bench_server.json \
  2> gpurun_out/bench_server.err
rc=$?
echo "bench server rc=$rc"; cat gpurun_out/bench_server.json; tail -3 gpurun_out/bench_server.err
if fatal $rc; then exit $rc; fi

timeout -k 10 300 python -u bench.py --workload server --steps 5 --warmup 2 --request 1 > gpurun_out/bench_server_shuffled.json \
  2> gpurun_out/bench_server_shuffled.err
rc=$?
echo "bench server (per-message shuffle) rc=$rc"; cat gpurun_out/bench_server_shuffled.json
if fatal $rc; then exit $rc; fi

timeout -k 10 300 python -u bench.py --workload server --steps 5 --warmup 2 --zipf 1.2 > gpurun_out/bench_server_zipf.json \
  2> gpurun_out/bench_server_zipf.err
rc=$?
echo "bench server (config 5, Zipf owners) rc=$rc"; cat gpurun_out/bench_server_zipf.json; tail -3 gpurun_out/bench_server_zipf.err
exit $rc
