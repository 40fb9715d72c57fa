#!/bin/bash
# GPU tests (all, or TESTS=...) then the server legs of the bench (tools/gpu_ab_server.sh)
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_b.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_b.log
[ $rc -eq 0 ] || exit $rc
VARIANTS=${VARIANTS:-cur:evolu_amd/libevm.so} LEGS=${LEGS:-server config4} REPS=${REPS:-1} bash tools/gpu_ab_server.sh
