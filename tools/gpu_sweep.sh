#!/bin/bash
# Config-2 bench lines (serial: isolated kernel durations; pipelined: the
# headline) for each value of an engine environment knob:
#   bash tools/gpu_sweep.sh VAR v1 v2 ...
mkdir -p gpurun_out
VAR=$1; shift
summ() { python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
print('%s %.4f ms frac %.3f' % (sys.argv[2], d['ms_per_step'], d['pipeline']['pipeline_hbm_frac']))
print('   '+' '.join('%s=%.1f' % (k.replace('k_',''), v*1e3) for k,v in d['pipeline']['kernels_ms_per_step'].items()))" "$1" "$2"; }
for rep in $(seq ${SW_REPS:-2}); do
for v in "$@"; do
  env $VAR=$v timeout -k 10 200 python -u bench.py --extra 0 --cpu-seconds 0 --depth 1 --overlap 0 --steps 10 > gpurun_out/sw_s.json 2>/dev/null || exit $?
  summ gpurun_out/sw_s.json "$VAR=$v serial"
  [ -n "$SW_SERIAL" ] && continue
  env $VAR=$v timeout -k 10 200 python -u bench.py --extra 0 --cpu-seconds 0 > gpurun_out/sw_p.json 2>/dev/null || exit $?
  summ gpurun_out/sw_p.json "$VAR=$v pipelined"
done
done
