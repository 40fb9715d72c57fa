set -o pipefail
export PYTHONUNBUFFERED=1
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
# K5 into an empty store vs into a 100M-row store (reingest), per dispatch: HBM bytes and SQ counters of one server bench
B=(python3 "$R/bench.py" --workload server --steps 2 --warmup 1 --cpu-seconds 0)
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/w_fetch" -o run -- "${B[@]}" > /dev/null &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/w_write" -o run -- "${B[@]}" > /dev/null &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d "$R/gpurun_out/w_sq1" -o run -- "${B[@]}" > /dev/null &&
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM --output-format csv -d "$R/gpurun_out/w_sq2" -o run -- "${B[@]}" > /dev/null &&
cd "$R" && python3 tools/pmc_dispatch.py "k_svo_a<1024u, 1, 256>" gpurun_out/w_fetch gpurun_out/w_write gpurun_out/w_sq1 gpurun_out/w_sq2 > gpurun_out/w_k5_dispatch.txt
