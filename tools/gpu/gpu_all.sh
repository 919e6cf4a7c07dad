# Full GPU validation: all gpu tests, then the default bench and every flow (each step time-limited)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
grep metric gpurun_out/bench_default.log
for f in ${FLOWS:-join passthrough full window}; do
  timeout -k 10 420 python bench.py --flow $f --steps 20 > gpurun_out/bench_$f.log 2>&1 || { tail -20 gpurun_out/bench_$f.log; exit 1; }
  grep metric gpurun_out/bench_$f.log | python -c "
import sys,json
d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2),'M ev/s', round(d['ms_per_step'],2),'ms p99', round(d['p99_latency_process_ms'],2), d['config'].get('source'), d.get('max_hbm_allocated_gb'))"
done
