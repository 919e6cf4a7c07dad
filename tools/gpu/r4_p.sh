# Round 4: full flow host-bound knobs A/B (GIL switch interval) + per-statement host time of the planning thread
set -o pipefail
mkdir -p gpurun_out/r4p
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py --flow full --steps 100 --profile-stages > gpurun_out/r4p/$name.log 2>&1 || { tail -20 gpurun_out/r4p/$name.log; exit 1; }
  grep metric gpurun_out/r4p/$name.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$name', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms p50', round(d['p50_latency_process_ms'],2)); print('   host ms/step', d.get('host_ms_per_step'))"; }
run default DXA_X=0
run sw05 DXA_SWITCH_INTERVAL_MS=0.5
run sw1 DXA_SWITCH_INTERVAL_MS=1
run default2 DXA_X=0
timeout -k 10 300 python bench.py --flow window --steps 100 --profile-stages > gpurun_out/r4p/window.log 2>&1 || { tail -20 gpurun_out/r4p/window.log; exit 1; }
grep metric gpurun_out/r4p/window.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('window', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms'); print('   host ms/step', d.get('host_ms_per_step'))"
