#!/bin/bash
# HBM traffic per kernel launch of the server legs at their own sizes
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in separate --pmc passes,
# nothing else on the command line), -> gpurun_out/pmc/traffic_<workload>.json
# (tools/pmc_traffic.py keeps each kernel's full-size launches only).
# usage: tools/gpu_pmc.sh <workload-name>...   (client config3 config4 config5)
R=$(pwd)
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
set -e
pmc() {  # workload-name, bench args...
  local w=$1; shift
  echo "pmc $w fetch"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc/fetch_$w" -o run -- \
    python3 "$R/bench.py" "$@" > "$R/gpurun_out/pmc/bench_$w.json"
  echo "pmc $w write"
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc/write_$w" -o run -- \
    python3 "$R/bench.py" "$@" > /dev/null
  python3 "$R/tools/pmc_traffic.py" "$R/gpurun_out/pmc/fetch_$w" "$R/gpurun_out/pmc/write_$w" \
    > "$R/gpurun_out/pmc/traffic_$w.json"
  rm -rf "$R/gpurun_out/pmc/fetch_$w" "$R/gpurun_out/pmc/write_$w"
}
for w in "$@"; do
  case $w in
    client) pmc client --extra 0 --steps 3 --warmup 1 --cpu-seconds 0 ;;
    client_adversarial) pmc client_adversarial --workload adversarial --steps 3 --warmup 1 ;;
    config3) pmc config3 --workload server --steps 2 --warmup 1 --cpu-seconds 0 ;;
    config4) pmc config4 --workload config4 --steps 2 --warmup 1 ;;
    config5) pmc config5 --workload config5shape --steps 2 --warmup 1 ;;
    *) echo "unknown workload $w"; exit 2 ;;
  esac
done
echo pmc done
