#!/bin/bash
mkdir -p gpurun_out
for d in 2 3 4 6; do
  timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --cpu-seconds 0 --extra 0 --depth $d > gpurun_out/bd$d.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bd$d.json'));print('depth $d', round(d['ms_per_step'],4), round(d['pipeline']['pipeline_hbm_frac'],3))"
done
