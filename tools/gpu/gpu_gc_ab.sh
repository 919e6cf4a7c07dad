# Latency-Process tail with and without the GC settling (dxa.utils.settle_gc): 100 timed steps, per-batch latencies
set -o pipefail
mkdir -p gpurun_out
for flow in groupby window; do
  for g in 0 1; do
    DXA_GC_TUNE=$g DXA_BENCH_HOST_TRACE=1 timeout -k 10 400 python bench.py --flow $flow --steps 100 > gpurun_out/gc_${flow}_$g.log 2>&1 || { tail -20 gpurun_out/gc_${flow}_$g.log; exit 1; }
    grep metric gpurun_out/gc_${flow}_$g.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); l=d['latency_trace_ms']; print('$flow gc=$g', round(d['value']/1e6,2), round(d['ms_per_step'],2), 'p50', round(d['p50_latency_process_ms'],2), 'p99', round(d['p99_latency_process_ms'],2), 'max', max(l), 'top', sorted(range(len(l)), key=lambda i:-l[i])[:5])"
  done
done
