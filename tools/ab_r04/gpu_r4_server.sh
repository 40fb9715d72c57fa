set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_server_segments.py > gpurun_out/t_seg.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_server.py tests/test_gpu_scale.py tests/test_gpu_server_atomic.py tests/test_gpu_wire.py tests/test_gpu_adversarial.py tests/test_gpu_config3_oracle.py tests/test_gpu_dist_loopback.py tests/test_gpu_dist_split_abi.py > gpurun_out/t_server.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload server --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/b_server.json 2> gpurun_out/b_server.err &&
timeout -k 10 400 python -u bench.py --workload config5shape --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/b_c5s.json 2> gpurun_out/b_c5s.err
