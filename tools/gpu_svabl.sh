#!/bin/bash
# K5 ablation builds on the config-3 server bench (k_svo_a<1024, true> time per step).
mkdir -p gpurun_out
for lib in evolu_amd/libevm.so "$@"; do
  EVM_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --workload server --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/svabl.json 2>/dev/null || exit $?
  python3 -c "
import json,sys;d=json.load(open('gpurun_out/svabl.json'));k=d['pipeline']['kernels_ms_per_step']
print('%-26s step %.3f ms  k_svo_a %.3f ms' % (sys.argv[1], d['ms_per_step'], k.get('(k_svo_a<1024, true>)', 0)))" $lib
done
