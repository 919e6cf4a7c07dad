# Same-box A/B of env settings: ABFLOW flow, ABVARS = space-separated "NAME=VAL,NAME=VAL" configs, 2 rounds each
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in $ABVARS; do
    envs=$(echo $cfg | tr ',' ' ')
    env $envs timeout -k 10 420 python bench.py --flow ${ABFLOW:-window} --steps 30 > gpurun_out/ab_$r.log 2>&1 || { tail -20 gpurun_out/ab_$r.log; exit 1; }
    grep metric gpurun_out/ab_$r.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$cfg run $r', round(d['value']/1e6,2), round(d['ms_per_step'],2), 'p50', round(d['p50_latency_process_ms'],2), 'p99', round(d['p99_latency_process_ms'],2))"
  done
done
