#!/bin/bash
# The small-batch path's tests, then the config-1 leg alone.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_config1.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_small.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_small.log
case $rc in 0) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u bench.py --cpu-seconds 0 --steps 10 --warmup 2 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_small.json'));c=d['config1']
print('config1 %.4f ms' % c['ms_per_batch'], {k:round(v*1e3,1) for k,v in c['kernels_ms_per_batch'].items()})
print({k:round(v['p50_ms'],4) for k,v in c['latency_per_batch'].items()})
print('config2 %.4f ms frac %.3f' % (d['ms_per_step'], d['pipeline']['pipeline_hbm_frac']))"
