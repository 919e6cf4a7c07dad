# Same-box A/B of whole source trees: TREES="tools/_ab/base ." (each a directory holding bench.py + dxa/ with its
# built libraries), FLOWS, REPS alternating rounds.  A tree under tools/_ab/ is `git archive <commit> bench.py dxa`
# built in place (python -c "from dxa.ops.build import build; build()").  OUT=<dir>
set -o pipefail
O=gpurun_out/${OUT:-ab_trees}
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for f in ${FLOWS:-window full}; do
    k=0
    for t in ${TREES:-.}; do
      k=$((k+1))
      timeout -k 10 420 python $t/bench.py --flow $f --steps ${STEPS:-60} ${ARGS:-} > $O/${f}_t${k}_$rep.log 2>&1 || { tail -20 $O/${f}_t${k}_$rep.log; exit 1; }
      grep '"metric"' $O/${f}_t${k}_$rep.log | python -c "
import sys,json
d=json.loads(sys.stdin.readline()); print('$f', 't$k [$t]', 'rep $rep', round(d['value']/1e6,2),'M ev/s', round(d['ms_per_step'],2),'ms p99', round(d['p99_latency_process_ms'],1))"
    done
  done
done
