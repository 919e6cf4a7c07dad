set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_e2e_flows.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ser_tests.log 2>&1 || { tail -40 gpurun_out/ser_tests.log; exit 1; }
tail -1 gpurun_out/ser_tests.log
for f in passthrough window; do
  timeout -k 10 420 python bench.py --flow $f --steps 20 > gpurun_out/bench_$f.log 2>&1 || { tail -20 gpurun_out/bench_$f.log; exit 1; }
  grep metric gpurun_out/bench_$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['p99_latency_process_ms'],2))"
done
