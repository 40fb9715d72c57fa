#!/bin/bash
# config-5 shape: segment target sweep (EVM_SEG_TARGET), per-kernel times
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_server_segments.py tests/test_gpu_adversarial.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_seg.log 2>&1 || { tail -20 gpurun_out/pytest_seg.log; exit 1; }
tail -2 gpurun_out/pytest_seg.log
for t in ${TARGETS:-560 680 800 900}; do
  EVM_SEG_TARGET=$t timeout -k 10 300 python -u bench.py --workload server --zipf 1.2 --steps 5 --warmup 2 --cpu-seconds 0 \
    > gpurun_out/sweep_$t.json 2> gpurun_out/sweep_$t.err || exit $?
  python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
print('target %s %.3f ms %.2f G' % (sys.argv[2], d['ms_per_step'], d['value']/1e9))
print('   '+' '.join('%s=%.3f' % (k.replace('k_',''), v) for k,v in list(d['pipeline']['kernels_ms_per_step'].items())[:9]))" gpurun_out/sweep_$t.json $t
done
