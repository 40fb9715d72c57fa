#!/bin/bash
# tc-path tests + short bench + kernel trace (iteration loop)
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_tcpath.py tests/test_gpu_apply.py tests/test_gpu_scale.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_tc.log 2>&1
rc=$?
echo "tc tests rc=$rc"; tail -3 gpurun_out/pytest_tc.log
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --extra 0 > gpurun_out/bench_tc.json 2> gpurun_out/bench_tc.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_tc.json; tail -3 gpurun_out/bench_tc.err
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --extra 0 --overlap 0 > gpurun_out/bench_tc_serial.json 2> gpurun_out/bench_tc_serial.err
rc=$?
echo "bench serial rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/bench_tc_serial.json'));print(d['ms_per_step'], d['pipeline']['kernels_ms_per_step'])"
if fatal $rc; then exit $rc; fi
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_tc" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 3 --cpu-seconds 0 --extra 0 > "$R/gpurun_out/prof_tc_bench.json"
rc=$?
echo "rocprof rc=$rc"
cd "$R" && python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_tc/run_kernel_stats.csv')))
for r in sorted(rows, key=lambda r:-float(r['TotalDurationNs']))[:16]:
    print("%-44s %5s avg %8.1f min %8.1f max %8.1f us" % (r['Name'][:44], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, float(r['MaxNs'])/1e3))
PY
exit $rc
