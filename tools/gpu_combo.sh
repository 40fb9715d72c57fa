#!/bin/bash
# Config-2 serial + pipelined lines for "ENV=.. ENV2=.." combos given as arguments.
mkdir -p gpurun_out
summ() { python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
print('%s %.4f ms frac %.3f' % (sys.argv[2], d['ms_per_step'], d['pipeline']['pipeline_hbm_frac']))
print('   '+' '.join('%s=%.1f' % (k.replace('k_',''), v*1e3) for k,v in d['pipeline']['kernels_ms_per_step'].items()))" "$1" "$2"; }
for rep in $(seq ${SW_REPS:-1}); do
for combo in "$@"; do
  env $combo timeout -k 10 200 python -u bench.py --extra 0 --cpu-seconds 0 --depth 1 --overlap 0 --steps 10 > gpurun_out/cb_s.json 2>/dev/null || exit $?
  summ gpurun_out/cb_s.json "[$combo] serial"
  env $combo timeout -k 10 200 python -u bench.py --extra 0 --cpu-seconds 0 > gpurun_out/cb_p.json 2>/dev/null || exit $?
  summ gpurun_out/cb_p.json "[$combo] pipelined"
done
done
