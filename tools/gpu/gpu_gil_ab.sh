# Latency-Process of pipelined outputs vs collector settling and the GIL switch interval (groupby, 60 steps)
set -o pipefail
mkdir -p gpurun_out
for cfg in "0 5" "1 5" "0 0.5" "1 0.5"; do
  set -- $cfg
  DXA_GC_TUNE=$1 DXA_SWITCH_INTERVAL_MS=$2 DXA_BENCH_HOST_TRACE=1 timeout -k 10 300 python bench.py --steps 60 > gpurun_out/gil_$1_$2.log 2>&1 || { tail -20 gpurun_out/gil_$1_$2.log; exit 1; }
  grep metric gpurun_out/gil_$1_$2.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('gc=$1 sw=$2', round(d['value']/1e6,2), round(d['ms_per_step'],2), 'p50', round(d['p50_latency_process_ms'],2), 'p99', round(d['p99_latency_process_ms'],2))"
done
