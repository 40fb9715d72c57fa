set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
# SQ counters + kernel traces: the server (K5) and the headline (TP1 / XF)
bash tools/gpu_sq.sh server --workload server --steps 2 --warmup 1 --cpu-seconds 0 &&
bash tools/gpu_sq.sh client --extra 0 --steps 3 --warmup 1 --cpu-seconds 0
