# Output-stream priority A/B: Latency-Process and throughput (groupby 60 steps, window/full 20 steps)
set -o pipefail
mkdir -p gpurun_out
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for flow in groupby window full; do
  for p in 0 1; do
    DXA_SINK_STREAM_PRIORITY=$p timeout -k 10 420 python bench.py --flow $flow --steps 40 > gpurun_out/prio_${flow}_$p.log 2>&1 || { tail -20 gpurun_out/prio_${flow}_$p.log; exit 1; }
    grep metric gpurun_out/prio_${flow}_$p.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$flow prio=$p', round(d['value']/1e6,2), round(d['ms_per_step'],2), 'p50', round(d['p50_latency_process_ms'],2), 'p99', round(d['p99_latency_process_ms'],2))"
  done
done
