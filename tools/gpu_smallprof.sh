#!/bin/bash
# rocprof kernel trace + stats of the small-batch path at the config-1 sizes
R=$(pwd); mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/small_prof" -o run -- \
  python3 "$R/tools/small_prof.py" > "$R/gpurun_out/small_prof.json" || exit $?
cd "$R" && python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/small_prof/**/run_kernel_stats.csv',recursive=True)[0]
for r in sorted(csv.DictReader(open(f)),key=lambda r:-float(r['TotalDurationNs']))[:16]:
    print('%-34s calls %6s avg %8.1f us min %8.1f us max %8.1f' % (r['Name'][:34], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, float(r['MaxNs'])/1e3))
PY
