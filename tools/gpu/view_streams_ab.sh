#!/bin/bash
# A/B of concurrent views on the full flow: DXA_VIEW_STREAMS=0 (statement order, one stream) vs streams vs threads.
set -o pipefail
mkdir -p gpurun_out/vs
export DXA_VIEW_STREAMS
for rep in 1 2; do
  for v in 0 streams threads; do
    DXA_VIEW_STREAMS=$v timeout -k 10 180 python bench.py --flow full --steps 40 --warmup 8 \
      > gpurun_out/vs/full_${v}_$rep.log 2>&1 || exit $?
    echo "full $v rep$rep: $(tail -1 gpurun_out/vs/full_${v}_$rep.log | cut -c90-200)"
  done
done
