#!/bin/bash
# Round-2 session C: tc-path tests, the apply tests, a short bench and a kernel trace.
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_tcpath.py tests/test_gpu_apply.py tests/test_gpu_apply_stored.py \
  tests/test_gpu_scale.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_tc.log 2>&1
rc=$?
echo "tc tests rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_tc.log | tail -40
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --extra 0 > gpurun_out/bench_tc.json 2> gpurun_out/bench_tc.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_tc.json; tail -3 gpurun_out/bench_tc.err
if fatal $rc; then exit $rc; fi
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_tc" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 3 --cpu-seconds 0 --extra 0 > "$R/gpurun_out/prof_tc_bench.json"
rc=$?
echo "rocprof rc=$rc"
exit $rc
