#!/bin/bash
# One GPU call: the whole GPU suite, the config-3 server leg alone (K5 and
# the device step), and the config-3 end-to-end rounds (tools/e2e_host.py).
# Every step under its own limit; a step that times out or crashes ends it.
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_full.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload server --steps 10 --warmup 2 --cpu-seconds 0 --e2e 0 \
  > gpurun_out/bench_server.json 2> gpurun_out/bench_server.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/bench_server.json'))
print('config3 ms/step %.3f' % d['ms_per_step'], 'K5 %.3f ms frac %.3f' % (d['roofline']['kernel_ms_avg'], d['roofline']['frac']))"
timeout -k 10 300 python -u tools/e2e_host.py > gpurun_out/e2e_host.log 2>&1 || exit $?
tail -3 gpurun_out/e2e_host.log
