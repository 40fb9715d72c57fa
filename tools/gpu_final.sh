#!/bin/bash
# The round's final evidence on one box: the default bench line (what the
# driver runs), the same command under rocprofv3 --kernel-trace --stats, and
# the GPU test suite.  -> gpurun_out/final/
R=$(pwd)
O=$R/gpurun_out/final
mkdir -p "$O"
export PYTHONUNBUFFERED=1
set -e
echo "bench"
timeout -k 10 600 python3 -u "$R/bench.py" > "$O/bench.json" 2> "$O/bench.err"
tail -c 600 "$O/bench.json"
echo "rocprof stats"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
  python3 "$R/bench.py" > "$O/prof_bench.json" 2> "$O/prof_bench.err")
find "$O/prof" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
find "$O/prof" -name "*kernel_trace.csv" -delete
echo "pytest"
timeout -k 10 600 python3 -u -m pytest "$R/tests" -m gpu -q --timeout 180 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
tail -2 "$O/pytest_gpu.log"
