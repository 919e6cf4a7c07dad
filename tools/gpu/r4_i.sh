# Round 4: unhex debug, benches + launch attribution (independent of the test suite), then the GPU tests
set -o pipefail
mkdir -p gpurun_out/r4i
timeout -k 10 120 python tools/gpu/dbg_unhex.py > gpurun_out/r4i/dbg_unhex.txt 2>&1; cat gpurun_out/r4i/dbg_unhex.txt | tail -8
for f in groupby window full; do
  timeout -k 10 300 python bench.py --flow $f --steps 30 > gpurun_out/r4i/bench_$f.log 2>&1 || { tail -20 gpurun_out/r4i/bench_$f.log; exit 1; }
  grep metric gpurun_out/r4i/bench_$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms')"
done
for f in window full; do
  timeout -k 10 400 python tools/launch_attrib.py --flow $f --batches 6 > gpurun_out/r4i/attrib_$f.txt 2>&1 || { tail -20 gpurun_out/r4i/attrib_$f.txt; exit 1; }
  head -2 gpurun_out/r4i/attrib_$f.txt
done
timeout -k 10 900 python -u -m pytest tests/test_packing.py tests/test_spark_docs_examples.py tests/test_strfuncs.py tests/test_arrayfuncs.py tests/test_decimal.py tests/test_flows_gpu.py tests/test_jit.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4i/tests.log 2>&1 || { grep -E "PASS|FAIL|Error" gpurun_out/r4i/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4i/tests.log
