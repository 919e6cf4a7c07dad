# A/B on one box: new renumber / pane-stats kernels on and off, window and full, twice each (interleaved)
set -o pipefail
mkdir -p gpurun_out/r4ab
for rep in 1 2; do
  for v in 1 0; do
    for f in window full; do
      DXA_RENUMBER_KERNEL=$v DXA_TS_STATS_KERNEL=$v timeout -k 10 300 python bench.py --flow $f --steps 30 > gpurun_out/r4ab/${f}_$v.log 2>&1 || { tail -20 gpurun_out/r4ab/${f}_$v.log; exit 1; }
      grep metric gpurun_out/r4ab/${f}_$v.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('rep $rep kernels=$v $f', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms')"
    done
  done
done
