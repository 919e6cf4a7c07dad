set -o pipefail
mkdir -p gpurun_out/r4d
timeout -k 10 600 python -u -m pytest tests/test_arrayfuncs.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4d/tests.log 2>&1 || { tail -60 gpurun_out/r4d/tests.log; exit 1; }
tail -1 gpurun_out/r4d/tests.log
for f in window full groupby; do
  timeout -k 10 300 python bench.py --flow $f --steps 30 > gpurun_out/r4d/bench_$f.log 2>&1 || { tail -20 gpurun_out/r4d/bench_$f.log; exit 1; }
  grep metric gpurun_out/r4d/bench_$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms')"
done
