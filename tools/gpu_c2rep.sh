mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tcpath.py tests/test_gpu_apply.py tests/test_gpu_async.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_c2.log 2>&1 || { tail -20 gpurun_out/pytest_c2.log; exit 1; }
tail -1 gpurun_out/pytest_c2.log
for rep in 1 2 3; do
timeout -k 10 200 python -u bench.py --extra 0 --cpu-seconds 0 > gpurun_out/c2_$rep.json 2>/dev/null || exit $?
python3 -c "
import json,sys;d=json.load(open(sys.argv[1]));print('%.4f ms frac %.3f roof %.3f'%(d['ms_per_step'],d['pipeline']['pipeline_hbm_frac'],d['roofline']['frac']))" gpurun_out/c2_$rep.json
done
