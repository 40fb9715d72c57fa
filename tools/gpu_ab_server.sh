#!/bin/bash
# A/B of server legs across variant builds: VARIANTS="base:path/libevm.so v1:_var/v1/libevm.so ..."
# LEGS="server config4" (bench.py --workload ...), alternating variants, REPS rounds.
# Prints each run's step time and its top kernels; JSON lines under gpurun_out/ab_<leg>_<v>_<rep>.json
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p=d.get('pipeline',{})
print('%s %.3f ms frac %.3f' % (sys.argv[2], d['ms_per_step'], p.get('pipeline_hbm_frac',0)))
print('   '+' '.join('%s=%.3f' % (k, v) for k,v in list(p.get('kernels_ms_per_step',{}).items())[:8]))
sw=d.get('src_wire')
if sw: print('   src_wire K5 %.3f ms' % sw['kernel_ms_avg'])
r=d.get('reingest')
if r: print('   reingest %.3f ms ' % r['ms_per_ingest_median'] + ' '.join('%s=%.3f' % (k,v) for k,v in list(r['kernels_ms'].items())[:4]))
" "$1" "$2"; }
for rep in $(seq 1 ${REPS:-1}); do
for leg in ${LEGS:-server}; do
for vv in $VARIANTS; do
  v=${vv%%:*}; lib=${vv#*:}
  out=gpurun_out/ab_${leg}_${v}_${rep}.json
  EVM_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --workload $leg --steps ${STEPS:-10} --warmup 2 --cpu-seconds 0 ${BENCH_ARGS} > $out 2> ${out%.json}.err || exit $?
  summ $out "$leg $v"
done
done
done
