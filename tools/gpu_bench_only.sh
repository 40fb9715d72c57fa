#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --extra 0 "$@" > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err
rc=$?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_q.json'));p=d['pipeline']
print('ms/step %.4f frac %.3f enqueue %.1f wait %.1f' % (d['ms_per_step'], p['pipeline_hbm_frac'], p['host_enqueue_us_avg'], p['host_wait_us_avg']))
print({k: round(v*1000,1) for k,v in p['kernels_ms_per_step'].items()})"
exit $rc
