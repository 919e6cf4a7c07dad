# Round 4: decimal + array GPU tests, flow differentials, benches, per-site launch attribution of window/full
set -o pipefail
mkdir -p gpurun_out/r4g
timeout -k 10 900 python -u -m pytest tests/test_packing.py tests/test_spark_docs_examples.py tests/test_strfuncs.py tests/test_arrayfuncs.py tests/test_decimal.py tests/test_flows_gpu.py tests/test_jit.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4g/tests.log 2>&1 || { tail -60 gpurun_out/r4g/tests.log; exit 1; }
tail -1 gpurun_out/r4g/tests.log
for f in groupby window full; do
  timeout -k 10 300 python bench.py --flow $f --steps 30 > gpurun_out/r4g/bench_$f.log 2>&1 || { tail -20 gpurun_out/r4g/bench_$f.log; exit 1; }
  grep metric gpurun_out/r4g/bench_$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms')"
done
for f in window full; do
  timeout -k 10 400 python tools/launch_attrib.py --flow $f --batches 6 > gpurun_out/r4g/attrib_$f.txt 2>&1 || { tail -20 gpurun_out/r4g/attrib_$f.txt; exit 1; }
  head -2 gpurun_out/r4g/attrib_$f.txt
done
