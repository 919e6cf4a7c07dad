# Round 4: output pipeline depth 1 vs 2 (two batches' outputs in flight) on every flow
set -o pipefail
mkdir -p gpurun_out/r4bb
run() { name=$1; flow=$2; shift 2; env "$@" timeout -k 10 300 python bench.py --flow $flow --steps 100 > gpurun_out/r4bb/$name.log 2>&1 || { tail -20 gpurun_out/r4bb/$name.log; exit 1; }
  grep metric gpurun_out/r4bb/$name.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$name', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms p50', round(d['p50_latency_process_ms'],2), 'p99', round(d['p99_latency_process_ms'],2), 'max hbm', d.get('max_hbm_allocated_gb'))"; }
for f in passthrough full window groupby; do
  run ${f}_d1 $f DXA_OUTPUT_DEPTH=1
  run ${f}_d2 $f DXA_OUTPUT_DEPTH=2
done
run passthrough_d2b passthrough DXA_OUTPUT_DEPTH=2
run passthrough_d3 passthrough DXA_OUTPUT_DEPTH=3
