# Round 4: cProfile of the full flow's timed steps (host time by function: syncs vs Python)
set -o pipefail
mkdir -p gpurun_out/r4r
DXA_BENCH_CPROFILE=gpurun_out/r4r/full.prof timeout -k 10 420 python bench.py --flow full --steps 60 > gpurun_out/r4r/bench_full.log 2>&1 || { tail -20 gpurun_out/r4r/bench_full.log; exit 1; }
python tools/pstats_report.py gpurun_out/r4r/full.prof 60 > gpurun_out/r4r/cprof_full.txt
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4r/bench_full.log | head -1
run() { name=$1; flow=$2; shift 2; env "$@" timeout -k 10 300 python bench.py --flow $flow --steps 100 --profile-stages > gpurun_out/r4r/$name.log 2>&1 || { tail -20 gpurun_out/r4r/$name.log; exit 1; }
  grep metric gpurun_out/r4r/$name.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); h=d.get('host_ms_per_step',{}); print('$name', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms p50', round(d['p50_latency_process_ms'],2), 'route', h.get('route'), 'DW', h.get('sql:DeviceWindow'))"; }
run full_hp full DXA_BENCH_HIPRIO=1
run full_np full DXA_BENCH_HIPRIO=0
run full_hp2 full DXA_BENCH_HIPRIO=1
run full_np2 full DXA_BENCH_HIPRIO=0
run window_hp window DXA_BENCH_HIPRIO=1
run window_np window DXA_BENCH_HIPRIO=0
