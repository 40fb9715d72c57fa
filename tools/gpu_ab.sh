#!/bin/bash
# A/B of the config-2 bench: _head/ (a worktree of the last commit, built in
# place) against the working tree, pipelined and serial, alternating.
mkdir -p gpurun_out
R=$(pwd)
summ() { python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
print('%s %.4f ms frac %.3f' % (sys.argv[2], d['ms_per_step'], d['pipeline']['pipeline_hbm_frac']))
print('   '+' '.join('%s=%.1f' % (k.replace('k_',''), v*1e3) for k,v in d['pipeline']['kernels_ms_per_step'].items()))" "$1" "$2"; }
for rep in 1 2; do
for v in head cur; do
  D=$R; [ $v = head ] && D=$R/_head
  (cd $D && timeout -k 10 200 python -u bench.py --extra 0 --cpu-seconds 0 ${BENCH_ARGS} > $R/gpurun_out/ab_${v}_p.json 2>/dev/null) || exit $?
  summ gpurun_out/ab_${v}_p.json "$v pipelined"
  (cd $D && timeout -k 10 200 python -u bench.py --extra 0 --cpu-seconds 0 --depth 1 --overlap 0 --steps 10 ${BENCH_ARGS} > $R/gpurun_out/ab_${v}_s.json 2>/dev/null) || exit $?
  summ gpurun_out/ab_${v}_s.json "$v serial"
done
done
