# Round 4: inference mode for the batch thread — full GPU suite + full/window benches
set -o pipefail
mkdir -p gpurun_out/r4x
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4x/tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r4x/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4x/tests.log
run() { name=$1; flow=$2; shift 2; env "$@" timeout -k 10 300 python bench.py --flow $flow --steps 100 --profile-stages > gpurun_out/r4x/$name.log 2>&1 || { tail -20 gpurun_out/r4x/$name.log; exit 1; }
  grep metric gpurun_out/r4x/$name.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); h=d.get('host_ms_per_step',{}); print('$name', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms p50', round(d['p50_latency_process_ms'],2), 'route', h.get('route'), 'DW', h.get('sql:DeviceWindow'))"; }
run full_inf full DXA_INFERENCE_MODE=1
run full_grad full DXA_INFERENCE_MODE=0
run window_inf window DXA_INFERENCE_MODE=1
run window_grad window DXA_INFERENCE_MODE=0
run full_inf2 full DXA_INFERENCE_MODE=1
run full_grad2 full DXA_INFERENCE_MODE=0
