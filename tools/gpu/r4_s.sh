# Round 4: vectorised concat segments — tests + full/window benches with host breakdown
set -o pipefail
mkdir -p gpurun_out/r4s
timeout -k 10 500 python -u -m pytest tests/test_copybatch.py tests/test_flows_gpu.py tests/test_window_stats.py tests/test_decimal.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4s/tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r4s/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4s/tests.log
run() { name=$1; flow=$2; shift 2; env "$@" timeout -k 10 300 python bench.py --flow $flow --steps 100 --profile-stages > gpurun_out/r4s/$name.log 2>&1 || { tail -20 gpurun_out/r4s/$name.log; exit 1; }
  grep metric gpurun_out/r4s/$name.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); h=d.get('host_ms_per_step',{}); print('$name', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms p50', round(d['p50_latency_process_ms'],2)); print('  ', h)"; }
run full full DXA_X=0
run window window DXA_X=0
run full2 full DXA_X=0
run window2 window DXA_X=0
