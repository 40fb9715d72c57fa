#!/bin/bash
# evm_dist_* ABI on one GPU
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist_abi.py -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_f.log 2>&1
rc=$?
echo "rc=$rc"; tail -30 gpurun_out/pytest_f.log
exit $rc
