#!/bin/bash
# Config-2 headline at several batch counts in flight (bench.py --depth).
mkdir -p gpurun_out
for rep in 1 2; do
for d in "$@"; do
  timeout -k 10 200 python -u bench.py --extra 0 --cpu-seconds 0 --depth $d > gpurun_out/bd$d.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bd$d.json'));print('depth $d', round(d['ms_per_step'],4), round(d['pipeline']['pipeline_hbm_frac'],3))"
done
done
