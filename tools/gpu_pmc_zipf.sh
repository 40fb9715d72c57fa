#!/bin/bash
# SQ counters for the server kernels on the config-5 shape (two --pmc passes)
R=$(pwd)
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
set -e
S=(python3 "$R/bench.py" --workload server --zipf 1.2 --steps 2 --warmup 1 --owners 20000 --cpu-seconds 0)
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
  SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d "$R/gpurun_out/pmc_z1" -o run -- "${S[@]}" > /dev/null
timeout -s KILL 180 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE \
  SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM --output-format csv -d "$R/gpurun_out/pmc_z2" -o run -- "${S[@]}" > /dev/null
S3=(python3 "$R/bench.py" --workload server --steps 2 --warmup 1 --owners 20000 --cpu-seconds 0)
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
  SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d "$R/gpurun_out/pmc_s1" -o run -- "${S3[@]}" > /dev/null
cd "$R"
python3 tools/pmc_summary.py gpurun_out/pmc_z1 gpurun_out/pmc_z2 > gpurun_out/pmc_zipf.txt
python3 tools/pmc_summary.py gpurun_out/pmc_s1 gpurun_out/pmc_s1 > gpurun_out/pmc_s3.txt
echo pmc done
