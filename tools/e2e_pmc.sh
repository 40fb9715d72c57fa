#!/bin/bash
# Counter passes over the device-resident sync round (tools/e2e_host.py,
# E2E_OWNERS owners, device rounds only): per-kernel SQ instruction mix and
# waits, then HBM traffic (FETCH_SIZE / WRITE_SIZE alone, as the guide says).
# usage: E2E_OWNERS=20000 tools/e2e_pmc.sh  -> gpurun_out/e2e_pmc/*.txt
R=$(pwd)
O=$R/gpurun_out/e2e_pmc
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
export E2E_HOST=0 E2E_OWNERS=${E2E_OWNERS:-20000}
set -e
n=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  n=$((n + 1))
  echo "pass $n: $pass"
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d "$O/p$n" -o run -- python3 "$R/tools/e2e_host.py" > "$O/run$n.log" 2>&1
  python3 "$R/tools/pmc_sum.py" "$O/p$n" > "$O/pass$n.txt"
  rm -rf "$O/p$n"
  head -20 "$O/pass$n.txt"
done
