#!/bin/bash
# The tc path's tests, then the headline bench line only (no extra legs).
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_tcpath.py tests/test_gpu_apply.py tests/test_gpu_scale.py tests/test_gpu_async.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_tc.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_tc.log
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u bench.py --extra 0 --cpu-seconds 0 > gpurun_out/bench_tc.json 2> gpurun_out/bench_tc.err
rc=$?
echo "bench rc=$rc"; python3 -c "
import json;d=json.load(open('gpurun_out/bench_tc.json'))
print('config2 %.4f ms frac %.3f roof %.3f' % (d['ms_per_step'], d['pipeline']['pipeline_hbm_frac'], d['roofline']['frac']))
print(json.dumps(d['pipeline']['kernels_ms_per_step']))"
tail -3 gpurun_out/bench_tc.err
exit $rc
