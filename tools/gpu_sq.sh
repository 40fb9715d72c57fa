#!/bin/bash
# SQ counters + kernel trace of one bench command on the GPU box (run from the
# repo root):  bash tools/gpu_sq.sh NAME [bench args...]
#   gpurun_out/sq_NAME/trace/run_kernel_stats.csv   (kernel trace + stats)
#   gpurun_out/sq_NAME.txt                           (tools/pmc_summary.py over two SQ passes)
# Each pass runs alone under its own time limit (counter passes never combine
# with other tracing); a failed pass ends the script.
set -e
name=$1; shift
R=$(pwd)
O="$R/gpurun_out/sq_$name"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B=(python3 "$R/bench.py" "$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- "${B[@]}" > "$O/bench.json"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
  SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d "$O/pmc1" -o run -- "${B[@]}" > /dev/null
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE \
  SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM --output-format csv -d "$O/pmc2" -o run -- "${B[@]}" > /dev/null
cd "$R" && python3 tools/pmc_summary.py "$O/pmc1" "$O/pmc2" > "gpurun_out/sq_$name.txt"
echo "sq $name done"
