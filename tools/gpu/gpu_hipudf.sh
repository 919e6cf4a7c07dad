set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hip_udf.py tests/test_e2e_flows.py tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/hipudf_tests.log 2>&1 || { tail -30 gpurun_out/hipudf_tests.log; exit 1; }
tail -1 gpurun_out/hipudf_tests.log
timeout -k 10 400 python bench.py --flow full --steps 30 > gpurun_out/hipudf_full.log 2>&1 || { tail -20 gpurun_out/hipudf_full.log; exit 1; }
grep metric gpurun_out/hipudf_full.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('full', round(d['value']/1e6,2), round(d['ms_per_step'],2), d['last_batch_outputs'])"
