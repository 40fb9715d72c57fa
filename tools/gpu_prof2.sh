#!/bin/bash
# Round-2 profiles: kernel trace + stats of the default bench line, and the two
# HBM traffic PMC passes (separate runs, --pmc only), each under its own limit.
R=$(pwd)
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
set -e
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 3 --cpu-seconds 0 > "$R/gpurun_out/prof_bench.json"
B=(python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0)
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch" -o run -- "${B[@]}" > /dev/null
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write" -o run -- "${B[@]}" > /dev/null
cd "$R"
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/traffic.json
echo prof done
