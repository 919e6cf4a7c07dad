# parse-ahead + carved gather outputs: GPU tests, then flows with DXA_PARSE_AHEAD on/off
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_kafka.py tests/test_kafka_device.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ahead_tests.log 2>&1 || { tail -30 gpurun_out/ahead_tests.log; exit 1; }
tail -1 gpurun_out/ahead_tests.log
for flow in full window groupby; do
  for a in 0 1; do
    DXA_PARSE_AHEAD=$a timeout -k 10 420 python bench.py --flow $flow --steps 30 > gpurun_out/ahead_${flow}_$a.log 2>&1 || { tail -20 gpurun_out/ahead_${flow}_$a.log; exit 1; }
    grep metric gpurun_out/ahead_${flow}_$a.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$flow ahead=$a', round(d['value']/1e6,2), round(d['ms_per_step'],2), 'p50', round(d['p50_latency_process_ms'],2), 'p99', round(d['p99_latency_process_ms'],2))"
  done
done
