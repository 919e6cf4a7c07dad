# Round 4: pane-partial concatenation cache — flow tests + full/window benches with host sections
set -o pipefail
mkdir -p gpurun_out/r4u
timeout -k 10 500 python -u -m pytest tests/test_flows_gpu.py tests/test_window_stats.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4u/tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r4u/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4u/tests.log
for f in full window full window; do
DXA_HOST_TIMERS=1 timeout -k 10 300 python bench.py --flow $f --steps 100 --profile-stages > gpurun_out/r4u/$f.log 2>&1 || { tail -20 gpurun_out/r4u/$f.log; exit 1; }
grep metric gpurun_out/r4u/$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2)); print('  ', d.get('host_ms_per_step')); print('  ', d.get('host_sections_ms_per_step'))"
done
