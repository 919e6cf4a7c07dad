# final round-5 tree (third pass, gpu-sim event-time fix): GPU suite, smoke, default bench, all five flows x2
set -o pipefail
mkdir -p gpurun_out/final7
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/final7/tests.log 2>&1 || { tail -40 gpurun_out/final7/tests.log; exit 1; }
tail -2 gpurun_out/final7/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final7/smoke.log 2>&1 || { tail -20 gpurun_out/final7/smoke.log; exit 1; }
tail -1 gpurun_out/final7/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final7/bench_default.log 2>&1 || { tail -20 gpurun_out/final7/bench_default.log; exit 1; }
echo "default $(grep -o '"value": [0-9.]*' gpurun_out/final7/bench_default.log | cut -d' ' -f2)"
for rep in 1 2; do
  for f in groupby join window full passthrough; do
    st=60; [ $f = groupby ] && st=100
    timeout -k 10 400 python bench.py --flow $f --steps $st > gpurun_out/final7/${f}_$rep.log 2>&1 || { tail -20 gpurun_out/final7/${f}_$rep.log; exit 1; }
    grep '"metric"' gpurun_out/final7/${f}_$rep.log | python -c "
import sys,json
d=json.loads(sys.stdin.readline()); print('$f $rep', round(d['value']/1e6,2),'M ev/s', round(d['ms_per_step'],2),'ms p99', round(d['p99_latency_process_ms'],1), 'hbm', d.get('max_hbm_allocated_gb'))"
  done
done
