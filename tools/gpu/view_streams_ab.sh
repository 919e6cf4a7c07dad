#!/bin/bash
# A/B of concurrent views on the full flow (window filled: default warmup): DXA_VIEW_STREAMS=0 (statement order, one
# stream) vs streams vs threads, alternating, two repetitions on one box.
set -o pipefail
mkdir -p gpurun_out/vs
for rep in 1 2; do
  for v in 0 streams threads; do
    DXA_VIEW_STREAMS=$v timeout -k 10 240 python bench.py --flow full --steps 30 \
      > gpurun_out/vs/full_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/vs/full_${v}_$rep.log; exit 1; }
    grep metric gpurun_out/vs/full_${v}_$rep.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('full views=$v rep $rep', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms')"
  done
done
