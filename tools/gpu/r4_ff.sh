# Round 4: pane compaction total read with the pane statistics (one host read fewer per batch) — tests + benches
set -o pipefail
mkdir -p gpurun_out/r4ff
timeout -k 10 500 python -u -m pytest tests/test_flows_gpu.py tests/test_window_stats.py tests/test_gpu_kernels.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4ff/tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r4ff/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4ff/tests.log
for f in window full window full; do
DXA_HOST_TIMERS=1 timeout -k 10 300 python bench.py --flow $f --steps 100 --profile-stages > gpurun_out/r4ff/$f.log 2>&1 || { tail -20 gpurun_out/r4ff/$f.log; exit 1; }
grep metric gpurun_out/r4ff/$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); h=d.get('host_sections_ms_per_step',{}); print('$f', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'windows', d['host_ms_per_step'].get('windows'), 'stats', h.get('windows:stats'), 'compact', h.get('windows:compact'))"
done
