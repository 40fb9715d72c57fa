#!/bin/bash
# K5 workgroup-size sweep (EVM_SVO512_THREADS / EVM_SVO1024_THREADS): config 5 and config 3
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_server_segments.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_wg.log 2>&1 || { tail -20 gpurun_out/pytest_wg.log; exit 1; }
EVM_SVO512_THREADS=64 EVM_SVO1024_THREADS=128 timeout -k 10 300 python -u -m pytest tests/test_gpu_server_segments.py \
  tests/test_gpu_adversarial.py tests/test_gpu_server.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_wg2.log 2>&1 || { tail -20 gpurun_out/pytest_wg2.log; exit 1; }
tail -1 gpurun_out/pytest_wg2.log
summ() { python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
print('%s %.3f ms %.2f G' % (sys.argv[2], d['ms_per_step'], d['value']/1e9))
print('   '+' '.join('%s=%.3f' % (k.replace('k_',''), v) for k,v in list(d['pipeline']['kernels_ms_per_step'].items())[:6]))" "$1" "$2"; }
for cfg in "256 256" "128 256" "64 256" "64 128"; do
  set -- $cfg
  EVM_SVO512_THREADS=$1 EVM_SVO1024_THREADS=$2 timeout -k 10 300 python -u bench.py --workload server --zipf 1.2 --steps 5 \
    --warmup 2 --cpu-seconds 0 > gpurun_out/wg5_$1_$2.json 2>/dev/null || exit $?
  summ gpurun_out/wg5_$1_$2.json "c5 512:$1 1024:$2"
done
for t in 256 128; do
  EVM_SVO1024_THREADS=$t timeout -k 10 300 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 \
    > gpurun_out/wg3_$t.json 2>/dev/null || exit $?
  summ gpurun_out/wg3_$t.json "c3 1024:$t"
done
