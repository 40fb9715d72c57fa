#!/bin/bash
# Server-path GPU tests, then the config-3 and config-5-shape server benches
# (per-kernel times).  A/B: SERVER_AB=1 also runs _head/'s build.
mkdir -p gpurun_out
R=$(pwd)
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_server.py tests/test_gpu_server_segments.py tests/test_gpu_server_atomic.py \
  tests/test_gpu_adversarial.py tests/test_gpu_scale.py tests/test_gpu_wire.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_server.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_server.log
if fatal $rc; then exit $rc; fi
[ $rc -ne 0 ] && exit $rc
summ() { python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
print('%s %.3f ms  %.2f G msgs/s' % (sys.argv[2], d['ms_per_step'], d['value']/1e9))
print('   '+' '.join('%s=%.3f' % (k.replace('k_',''), v) for k,v in list(d['pipeline']['kernels_ms_per_step'].items())[:12]))" "$1" "$2"; }
VS="cur"; [ -n "$SERVER_AB" ] && VS="head cur"
for v in $VS; do
  D=$R; [ $v = head ] && D=$R/_head
  (cd $D && timeout -k 10 300 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > $R/gpurun_out/sv3_$v.json 2> $R/gpurun_out/sv3_$v.err) || exit $?
  summ gpurun_out/sv3_$v.json "$v config3"
  (cd $D && timeout -k 10 300 python -u bench.py --workload server --zipf 1.2 --steps 5 --warmup 2 --cpu-seconds 0 > $R/gpurun_out/sv5_$v.json 2> $R/gpurun_out/sv5_$v.err) || exit $?
  summ gpurun_out/sv5_$v.json "$v config5"
done
