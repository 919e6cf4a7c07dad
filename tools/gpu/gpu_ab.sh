# A/B of bench flags: FLOWS x VARIANTS (';'-separated bench argument sets), REPS runs each.  OUT=<dir>
set -o pipefail
O=gpurun_out/${OUT:-ab}
mkdir -p $O
IFS=';' read -ra VARS <<< "${VARIANTS:-}"
for rep in $(seq 1 ${REPS:-2}); do
  for f in ${FLOWS:-window full}; do
    k=0
    for v in "${VARS[@]}"; do
      k=$((k+1))
      timeout -k 10 420 python bench.py --flow $f --steps ${STEPS:-60} $v > $O/${f}_v${k}_$rep.log 2>&1 || { tail -20 $O/${f}_v${k}_$rep.log; exit 1; }
      grep '"metric"' $O/${f}_v${k}_$rep.log | python -c "
import sys,json
d=json.loads(sys.stdin.readline()); print('$f', 'v$k [$v]', 'rep $rep', round(d['value']/1e6,2),'M ev/s', round(d['ms_per_step'],2),'ms p99', round(d['p99_latency_process_ms'],1))"
    done
  done
done
