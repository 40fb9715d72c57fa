#!/bin/bash
# Round-end evidence in one call: the whole GPU suite, the default bench line,
# then the rocprof kernel trace + stats of the default bench and the two HBM
# traffic PMC passes (tools/gpu_prof.sh).  Every GPU step has its own limit.
mkdir -p gpurun_out
bash tools/gpu_full.sh || exit $?
bash tools/gpu_prof.sh || exit $?
