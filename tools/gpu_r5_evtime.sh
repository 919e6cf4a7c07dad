# window / full flows after the gpu-sim event-time fix (events in the second before their batch time)
set -o pipefail
O=gpurun_out/r5_evtime; mkdir -p $O
for rep in 1 2; do
  for f in window full; do
    DXA_BENCH_HOST_TRACE=1 timeout -k 10 300 python bench.py --flow $f --steps 60 > $O/${f}_$rep.log 2>&1 || exit 1
  done
done
