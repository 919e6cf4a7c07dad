# host-side timing of the full / window flows: per-step host ms (stage, process_batch) and per-stage wall times
set -o pipefail
O=gpurun_out/r5_host5; mkdir -p $O
DXA_HOST_TIMERS=1 DXA_BENCH_HOST_TRACE=1 timeout -k 10 300 python bench.py --flow full --steps 60 --profile-stages > $O/full_trace.log 2>&1 && \
DXA_HOST_TIMERS=1 DXA_BENCH_HOST_TRACE=1 timeout -k 10 300 python bench.py --flow window --steps 60 --profile-stages > $O/window_trace.log 2>&1
for rep in 1 2; do
  for f in window full; do
    [ -z "$HOST_ONLY" ] && { timeout -k 10 300 python bench.py --flow $f --steps 60 > $O/${f}_$rep.log 2>&1 || exit 1; }
  done
done
