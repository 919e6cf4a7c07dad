# GPU validation: kernel tests, then one bench per BASELINE flow (each step time-limited, stop on first failure)
set -o pipefail
mkdir -p gpurun_out
python -m dxa.ops.build || exit 1
timeout -k 10 300 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for f in groupby join window full passthrough; do
  timeout -k 10 420 python bench.py --flow $f --steps 20 --profile-stages > gpurun_out/bench_$f.log 2>&1 || { tail -20 gpurun_out/bench_$f.log; exit 1; }
  grep metric gpurun_out/bench_$f.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$f', round(d['value']/1e6,2),'M ev/s', round(d['ms_per_step'],2),'ms p99', round(d['p99_latency_process_ms'],2), d.get('max_hbm_allocated_gb'), d.get('stage_s'), d.get('reference_build_s'), d.get('window_panes'))"
done
for f in window passthrough; do
  DXA_SYNC_STAGES=1 timeout -k 10 420 python bench.py --flow $f --steps 10 --profile-stages > gpurun_out/bench_sync_$f.log 2>&1 || { tail -20 gpurun_out/bench_sync_$f.log; exit 1; }
  grep metric gpurun_out/bench_sync_$f.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('sync $f', round(d['ms_per_step'],2), {k: round(v*1000,2) for k,v in d['stage_s'].items()})"
done
