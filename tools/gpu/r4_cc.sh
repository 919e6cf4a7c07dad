# Round 4: host sections of the join and groupby flows (same Kafka ingest; join is ~1 ms slower per step)
set -o pipefail
mkdir -p gpurun_out/r4cc
for f in join groupby; do
DXA_HOST_TIMERS=1 timeout -k 10 300 python bench.py --flow $f --steps 60 --profile-stages > gpurun_out/r4cc/$f.log 2>&1 || { tail -20 gpurun_out/r4cc/$f.log; exit 1; }
grep metric gpurun_out/r4cc/$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2)); print('  ', d.get('host_ms_per_step')); print('  ', d.get('host_sections_ms_per_step'))"
done
