# Generator / serializer (word-packed emitter): differential tests, generator micro-bench, window + passthrough benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "datagen or serializer or java_double" --timeout 120 --timeout-method thread > gpurun_out/gen_tests.log 2>&1 || { tail -40 gpurun_out/gen_tests.log; exit 1; }
tail -3 gpurun_out/gen_tests.log
timeout -k 10 120 python tools/gen_bench.py > gpurun_out/gen_bench.log 2>&1 || { tail -20 gpurun_out/gen_bench.log; exit 1; }
cat gpurun_out/gen_bench.log
for f in ${FLOWS:-window passthrough}; do
  timeout -k 10 420 python bench.py --flow $f --steps 20 > gpurun_out/bench_$f.log 2>&1 || { tail -20 gpurun_out/bench_$f.log; exit 1; }
  grep metric gpurun_out/bench_$f.log | python -c "
import sys,json
d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2),'M ev/s', round(d['ms_per_step'],2),'ms p99', round(d['p99_latency_process_ms'],2), d['config'].get('source'))"
done
