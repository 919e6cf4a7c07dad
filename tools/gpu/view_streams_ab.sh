#!/bin/bash
# A/B of concurrent views (side HIP streams) on the window and full flows: DXA_VIEW_STREAMS=1 (default) vs 0.
set -o pipefail
mkdir -p gpurun_out/vs
export DXA_VIEW_STREAMS
for flow in full window; do
  for v in 1 0; do
    DXA_VIEW_STREAMS=$v timeout -k 10 180 python bench.py --flow $flow --steps 40 --warmup 8 \
      > gpurun_out/vs/${flow}_vs$v.log 2>&1 || exit $?
    tail -1 gpurun_out/vs/${flow}_vs$v.log | cut -c1-200
  done
done
