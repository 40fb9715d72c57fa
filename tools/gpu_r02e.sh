#!/bin/bash
# N-API (sync + async) and wire-path tests
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_napi.py tests/test_gpu_wire.py -x -v \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_e.log 2>&1
rc=$?
echo "rc=$rc"; tail -30 gpurun_out/pytest_e.log
exit $rc
