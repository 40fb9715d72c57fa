#!/bin/bash
# Client-path GPU tests, then the config-2 bench line alone (per-kernel times).
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_tcpath.py tests/test_gpu_apply.py tests/test_gpu_apply_stored.py \
  tests/test_gpu_async.py tests/test_gpu_scale.py tests/test_gpu_core.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_client.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_client.log
if fatal $rc; then exit $rc; fi
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --extra 0 --cpu-seconds 0 ${BENCH_ARGS} > gpurun_out/bench_client.json 2> gpurun_out/bench_client.err
rc=$?
echo "bench rc=$rc"; python3 -c "
import json;d=json.load(open('gpurun_out/bench_client.json'))
print('config2 %.4f ms frac %.3f roof %.3f' % (d['ms_per_step'], d['pipeline']['pipeline_hbm_frac'], d['roofline']['frac']))
for k,v in d['pipeline']['kernels_ms_per_step'].items(): print('  %-24s %.4f' % (k, v))"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --extra 0 --cpu-seconds 0 --depth 1 --overlap 0 --steps 10 > gpurun_out/bench_client_serial.json 2> gpurun_out/bench_client_serial.err
rc=$?
echo "serial bench rc=$rc"; python3 -c "
import json;d=json.load(open('gpurun_out/bench_client_serial.json'))
print('config2 serial %.4f ms' % (d['ms_per_step']))
for k,v in d['pipeline']['kernels_ms_per_step'].items(): print('  %-24s %.4f' % (k, v))"
[ $rc -ne 0 ] && exit $rc
exit 0
