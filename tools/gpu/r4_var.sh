# Round 4: run-to-run spread on one box (same tree, same settings) — window and full x4, groupby x2
set -o pipefail
mkdir -p gpurun_out/var
for k in 1 2 3 4; do for f in window full; do
  timeout -k 10 300 python bench.py --flow $f --steps 100 > gpurun_out/var/${f}_$k.log 2>&1 || { tail -20 gpurun_out/var/${f}_$k.log; exit 1; }
  grep metric gpurun_out/var/${f}_$k.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f#$k', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms p50', round(d['p50_latency_process_ms'],2))"
done; done
for k in 1 2 3 4; do
  DXA_OUTPUT_DEPTH=2 timeout -k 10 300 python bench.py --flow full --steps 100 > gpurun_out/var/full_d2_$k.log 2>&1 || { tail -20 gpurun_out/var/full_d2_$k.log; exit 1; }
  grep metric gpurun_out/var/full_d2_$k.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('full_d2#$k', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms p50', round(d['p50_latency_process_ms'],2))"
done
for k in 1 2; do
  timeout -k 10 300 python bench.py --flow groupby --steps 100 > gpurun_out/var/groupby_$k.log 2>&1 || { tail -20 gpurun_out/var/groupby_$k.log; exit 1; }
  grep metric gpurun_out/var/groupby_$k.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('groupby#$k', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2))"
done
