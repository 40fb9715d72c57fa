#!/bin/bash
# A/B of the device-resident sync round across variant builds:
#   VARIANTS="base:evolu_amd/libevm.so v1:_var/v1/libevm.so" bash tools/gpu_ab_e2e.sh
# (tools/e2e_host.py, device rounds only; each variant's round times and kernels)
export PYTHONUNBUFFERED=1 E2E_HOST=0
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-1}); do
for vv in $VARIANTS; do
  v=${vv%%:*}; lib=${vv#*:}
  echo "== $v"
  EVM_LIB_PATH=$lib timeout -k 10 300 python -u tools/e2e_host.py > gpurun_out/ab_e2e_$v.log 2>&1 || exit $?
  grep -v "^bodies\|amdgpu.ids" gpurun_out/ab_e2e_$v.log | tail -2 | cut -c1-400
done
done
