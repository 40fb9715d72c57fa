#!/bin/bash
# Config 2 only: serial (isolated kernel durations) and pipelined bench lines,
# then a rocprof kernel trace + stats of the pipelined run.
mkdir -p gpurun_out
R=$(pwd)
summ() { python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
print('%s %.4f ms frac %.3f' % (sys.argv[2], d['ms_per_step'], d['pipeline']['pipeline_hbm_frac']))
print('   '+' '.join('%s=%.1f' % (k.replace('k_',''), v*1e3) for k,v in d['pipeline']['kernels_ms_per_step'].items()))" "$1" "$2"; }
timeout -k 10 200 python -u bench.py --extra 0 --cpu-seconds 0 --depth 1 --overlap 0 --steps 10 ${BENCH_ARGS} > gpurun_out/iso_s.json 2>/dev/null || exit $?
summ gpurun_out/iso_s.json serial
timeout -k 10 200 python -u bench.py --extra 0 --cpu-seconds 0 ${BENCH_ARGS} > gpurun_out/iso_p.json 2>/dev/null || exit $?
summ gpurun_out/iso_p.json pipelined
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/iso_prof" -o run -- \
  python3 "$R/bench.py" --extra 0 --cpu-seconds 0 --steps 20 --warmup 3 ${BENCH_ARGS} > "$R/gpurun_out/iso_prof.json" || exit $?
cd "$R" && python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/iso_prof/**/run_kernel_stats.csv',recursive=True)[0]
rows=list(csv.DictReader(open(f)))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print('%-40s calls %6s avg %8.1f us min %8.1f us' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3))
PY
