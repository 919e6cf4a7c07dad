# Round 4: GPU suite, benches (100 steps), launch attribution + kernel-trace stats of full
set -o pipefail
mkdir -p gpurun_out/r4m
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4m/tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r4m/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4m/tests.log
for f in groupby window full; do
  timeout -k 10 300 python bench.py --flow $f --steps 100 > gpurun_out/r4m/bench_$f.log 2>&1 || { tail -20 gpurun_out/r4m/bench_$f.log; exit 1; }
  grep metric gpurun_out/r4m/bench_$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms', 'p50', round(d['p50_latency_process_ms'],2))"
done
ATTRIB_DEPTH=3 timeout -k 10 400 python tools/launch_attrib.py --flow full --batches 6 --top 80 > gpurun_out/r4m/attrib_full.txt 2>&1 || { tail -20 gpurun_out/r4m/attrib_full.txt; exit 1; }
head -3 gpurun_out/r4m/attrib_full.txt | tail -1
FLOWS="window full" bash tools/gpu/gpu_prof.sh > gpurun_out/r4m/prof.txt 2>&1 || { tail -20 gpurun_out/r4m/prof.txt; exit 1; }
echo prof ok
