#!/bin/bash
# Profiles of the headline bench on the GPU box (run from the repo root):
#   kernel trace + stats (profiles/*_kernel_stats.csv), the two HBM traffic
#   PMC passes (tools/pmc_traffic.py), and two SQ counter passes for the
#   latency-bound kernels (tools/pmc_summary.py).  Every pass has its own
#   time limit; a failed pass ends the script.
R=$(pwd)
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
B=(python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0)
set -e
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 3 --cpu-seconds 0 > "$R/gpurun_out/prof_bench.json"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch" -o run -- "${B[@]}" > /dev/null
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write" -o run -- "${B[@]}" > /dev/null
if [ "$1" = "sq" ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d "$R/gpurun_out/pmc_sq1" -o run -- "${B[@]}" > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE \
    SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM --output-format csv -d "$R/gpurun_out/pmc_sq2" -o run -- "${B[@]}" > /dev/null
fi
if [ "$2" = "server" ]; then
  S=(python3 "$R/bench.py" --workload server --steps 2 --warmup 1 --owners 20000)
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d "$R/gpurun_out/pmc_sv1" -o run -- "${S[@]}" > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE \
    SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM --output-format csv -d "$R/gpurun_out/pmc_sv2" -o run -- "${S[@]}" > /dev/null
fi
cd "$R"
[ "$2" = "server" ] && python3 tools/pmc_summary.py gpurun_out/pmc_sv1 gpurun_out/pmc_sv2 > gpurun_out/pmc_sv.txt
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/traffic.json
[ "$1" = "sq" ] && python3 tools/pmc_summary.py gpurun_out/pmc_sq1 gpurun_out/pmc_sq2 > gpurun_out/pmc_sq.txt
echo prof done
