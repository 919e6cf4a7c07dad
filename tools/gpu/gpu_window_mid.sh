# window / full flows: complete pane blocks merged per batch (DXA_WINDOW_MID=0) vs pre-combined into one table (1)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for f in window full; do
    for m in 0 1; do
      DXA_WINDOW_MID=$m timeout -k 10 300 python bench.py --flow $f --steps 40 > gpurun_out/wmid_${f}_${m}_$r.log 2>&1 || { tail -20 gpurun_out/wmid_${f}_${m}_$r.log; exit 1; }
      grep metric gpurun_out/wmid_${f}_${m}_$r.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f mid=$m run $r', round(d['value']/1e6,2), round(d['ms_per_step'],2), 'p50', round(d['p50_latency_process_ms'],2), 'p99', round(d['p99_latency_process_ms'],2))"
    done
  done
done
