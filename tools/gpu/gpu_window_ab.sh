# window flow: this tree vs the end-of-round-2 tree (_ab_r2, a git worktree built in place), alternating
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
for r in 1 2; do
  for t in cur r2; do
    d=$R; [ $t = r2 ] && d=$R/_ab_r2
    (cd $d && timeout -k 10 300 python bench.py --flow window --steps 30) > gpurun_out/wab_${t}_$r.log 2>&1 || { tail -20 gpurun_out/wab_${t}_$r.log; exit 1; }
    grep metric gpurun_out/wab_${t}_$r.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$t run $r', round(d['value']/1e6,2), round(d['ms_per_step'],2), 'p50', round(d['p50_latency_process_ms'],2), 'p99', round(d['p99_latency_process_ms'],2))"
  done
done
