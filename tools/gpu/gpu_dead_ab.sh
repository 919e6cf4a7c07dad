# dead-view elimination A/B on the full flow (two runs each, alternating)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for d in 0 1; do
    DXA_DEAD_VIEWS=$d timeout -k 10 420 python bench.py --flow full --steps 30 > gpurun_out/dead_${d}_$r.log 2>&1 || { tail -20 gpurun_out/dead_${d}_$r.log; exit 1; }
    grep metric gpurun_out/dead_${d}_$r.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('dead=$d run $r', round(d['value']/1e6,2), round(d['ms_per_step'],2), 'p50', round(d['p50_latency_process_ms'],2), 'p99', round(d['p99_latency_process_ms'],2))"
  done
done
