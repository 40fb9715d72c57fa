#!/bin/bash
# GPU-box steps, each under its own time limit.  A fault, abort, segfault or
# time limit (124/134/137/139) ends the script; an ordinary failure (exit 1)
# lets the next step run so its output still comes back.
#   bash tools/gpu_steps.sh 'name|seconds|command' ...
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
worst=0
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "=== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  rc=$?
  echo "--- $name rc=$rc"; tail -c 3000 "gpurun_out/$name.out"; tail -5 "gpurun_out/$name.err"
  [ $rc -ne 0 ] && worst=$rc
  if fatal $rc; then exit $rc; fi
done
exit $worst
