# Round 4: parse-ahead on its own stream (queued before the previous batch's processing) — tests + A/B
set -o pipefail
mkdir -p gpurun_out/r4q
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_flows_gpu.py -x -q -m gpu -k "prepare or flow or concurrent" --timeout 300 --timeout-method thread > gpurun_out/r4q/tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r4q/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4q/tests.log
run() { name=$1; flow=$2; shift 2; env "$@" timeout -k 10 300 python bench.py --flow $flow --steps 100 --profile-stages > gpurun_out/r4q/$name.log 2>&1 || { tail -20 gpurun_out/r4q/$name.log; exit 1; }
  grep metric gpurun_out/r4q/$name.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); h=d.get('host_ms_per_step',{}); print('$name', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms p50', round(d['p50_latency_process_ms'],2), 'project', h.get('project'), 'route', h.get('route'))"; }
run full_side full DXA_X=0
run full_cur full DXA_PARSE_STREAM=0
run window_side window DXA_X=0
run window_cur window DXA_PARSE_STREAM=0
run full_side2 full DXA_X=0
run window_side2 window DXA_X=0
run groupby groupby DXA_X=0
