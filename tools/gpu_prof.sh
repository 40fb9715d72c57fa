#!/bin/bash
# Profiles of bench.py on the GPU box (run from the repo root):
#   * kernel trace + stats of the default bench command (every leg):
#     gpurun_out/prof/run_kernel_stats.csv
#   * per workload, the two HBM traffic PMC passes (FETCH_SIZE, WRITE_SIZE;
#     MI355X_MICROARCH.md: separate passes, nothing else on the command line)
#     -> gpurun_out/traffic_<workload>.json (tools/pmc_traffic.py)
#   * with "sq": two SQ counter passes over the headline (pmc_summary.py)
# Every pass has its own time limit; a failed pass ends the script.
R=$(pwd)
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
set -e
# (part "a": the trace + the client / config-3 passes; "b": the config-4 / config-5
# passes -- two calls, each well inside one call's time limit; no part: all)
part=${1:-all}
if [ "$part" != b ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 3 > "$R/gpurun_out/prof_bench.json"
fi
pmc() {  # workload-name, bench args...
  local w=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch_$w" -o run -- \
    python3 "$R/bench.py" "$@" > /dev/null
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_$w" -o run -- \
    python3 "$R/bench.py" "$@" > /dev/null
  python3 "$R/tools/pmc_traffic.py" "$R/gpurun_out/pmc_fetch_$w" "$R/gpurun_out/pmc_write_$w" > "$R/gpurun_out/traffic_$w.json"
}
if [ "$part" != b ]; then
pmc client --extra 0 --steps 3 --warmup 1 --cpu-seconds 0
pmc client_adversarial --workload adversarial --steps 3 --warmup 1
pmc config3 --workload server --steps 2 --warmup 1 --cpu-seconds 0
fi
if [ "$part" != a ]; then
pmc config4 --workload config4 --steps 2 --warmup 1
pmc config5 --workload config5shape --steps 2 --warmup 1
pmc config5n --workload config5 --steps 2 --warmup 1
fi
if [ "$part" = "sq" ]; then
  B=(python3 "$R/bench.py" --extra 0 --steps 3 --warmup 1 --cpu-seconds 0)
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d "$R/gpurun_out/pmc_sq1" -o run -- "${B[@]}" > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE \
    SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM --output-format csv -d "$R/gpurun_out/pmc_sq2" -o run -- "${B[@]}" > /dev/null
  cd "$R" && python3 tools/pmc_summary.py gpurun_out/pmc_sq1 gpurun_out/pmc_sq2 > gpurun_out/pmc_sq.txt
fi
echo prof done
