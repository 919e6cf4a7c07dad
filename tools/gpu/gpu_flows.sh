# all bench flows, 30 timed steps each
set -o pipefail
mkdir -p gpurun_out
for f in ${FLOWS:-full window join passthrough groupby}; do
  timeout -k 10 420 python bench.py --flow $f --steps 30 > gpurun_out/flows_$f.log 2>&1 || { tail -20 gpurun_out/flows_$f.log; exit 1; }
  grep metric gpurun_out/flows_$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2), round(d['ms_per_step'],2), 'p50', round(d['p50_latency_process_ms'],2), 'p99', round(d['p99_latency_process_ms'],2), d.get('max_hbm_allocated_gb'))"
done
