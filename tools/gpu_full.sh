#!/bin/bash
# The whole GPU suite, then the default bench line (what the driver runs).
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_full.log
if fatal $rc; then exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?
echo "bench rc=$rc"; python3 -c "
import json;d=json.load(open('gpurun_out/bench_full.json'))
print('config2 %.4f ms frac %.3f roof %.3f' % (d['ms_per_step'], d['pipeline']['pipeline_hbm_frac'], d['roofline']['frac']))
print('config1', d['config1']['ms_per_batch'], d['config1']['value'])
c=d['config3']; print('config3 %.3f ms frac %.3f roof %s %.3f' % (c['ms_per_step'], c['pipeline']['pipeline_hbm_frac'], c['roofline']['kernel'], c['roofline']['frac']))"
tail -3 gpurun_out/bench_full.err
exit $rc
