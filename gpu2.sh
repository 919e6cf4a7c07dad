set -o pipefail
mkdir -p gpurun_out
R=$PWD
python -m dxa.ops.build
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
DXA_SYNC_STAGES=1 timeout -k 10 400 python bench.py --steps 10 --warmup 3 --profile-stages > gpurun_out/bench_sync.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --profile-stages > gpurun_out/bench1.log 2>&1 || exit 1
tail -2 gpurun_out/gpu_tests.log; cat gpurun_out/bench_sync.log gpurun_out/bench1.log | grep metric | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(round(d['value']/1e6,2),'M ev/s', round(d['ms_per_step'],1),'ms', d.get('stage_s'), d['p99_latency_process_ms'])"
