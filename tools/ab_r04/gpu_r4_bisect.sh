set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
T='tests/test_gpu_server_segments.py::test_zipf_segments_vs_sort_path[200-600000-1]'
for v in dbgscan; do
  EVM_LIB_PATH=_var/$v/libevm.so timeout -k 10 120 python -u -m pytest -x -q -s --timeout 100 --timeout-method thread "$T" > gpurun_out/bis_$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
  echo "variant $v passed"
done
