# Round 4: unhex debug on the test's data, benches, launch attribution with call chains, then the GPU tests
set -o pipefail
mkdir -p gpurun_out/r4j
timeout -k 10 300 python tools/gpu/dbg_unhex.py > gpurun_out/r4j/dbg_unhex.txt 2>&1; tail -8 gpurun_out/r4j/dbg_unhex.txt
for f in groupby window full; do
  timeout -k 10 300 python bench.py --flow $f --steps 30 > gpurun_out/r4j/bench_$f.log 2>&1 || { tail -20 gpurun_out/r4j/bench_$f.log; exit 1; }
  grep metric gpurun_out/r4j/bench_$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms')"
done
for f in window full; do
  ATTRIB_DEPTH=3 timeout -k 10 400 python tools/launch_attrib.py --flow $f --batches 6 --top 80 > gpurun_out/r4j/attrib_$f.txt 2>&1 || { tail -20 gpurun_out/r4j/attrib_$f.txt; exit 1; }
  head -3 gpurun_out/r4j/attrib_$f.txt | tail -1
done
timeout -k 10 900 python -u -m pytest tests/test_window_stats.py tests/test_copybatch.py tests/test_packing.py tests/test_strfuncs.py tests/test_decimal.py tests/test_flows_gpu.py tests/test_distributed.py tests/test_jit.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4j/tests.log 2>&1 || { grep -E "PASS|FAIL|Error" gpurun_out/r4j/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4j/tests.log
