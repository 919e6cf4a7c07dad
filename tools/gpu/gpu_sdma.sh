# D2H of rendered output on SDMA vs the blit kernel: serializer GPU tests, passthrough + window benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_e2e_flows.py -x -q -m gpu -k "serial or e2e or flow" --timeout 120 --timeout-method thread > gpurun_out/sdma_tests.log 2>&1 || { tail -30 gpurun_out/sdma_tests.log; exit 1; }
tail -1 gpurun_out/sdma_tests.log
for f in passthrough window; do
  for v in 1 0; do
    export DXA_D2H_SDMA=$v
    timeout -k 10 400 python bench.py --flow $f --steps 30 > gpurun_out/sdma_${f}_$v.log 2>&1 || { tail -20 gpurun_out/sdma_${f}_$v.log; exit 1; }
    grep metric gpurun_out/sdma_${f}_$v.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f sdma=$v', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['p99_latency_process_ms'],2))"
  done
done
