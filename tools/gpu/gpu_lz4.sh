set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lz4.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lz4_tests.log 2>&1 || { tail -30 gpurun_out/lz4_tests.log; exit 1; }
tail -1 gpurun_out/lz4_tests.log
for L in 0 9; do
  timeout -k 10 200 python tools/lz4_bench.py --level $L > gpurun_out/lz4_micro_L$L.log 2>&1 || { tail -20 gpurun_out/lz4_micro_L$L.log; exit 1; }
  echo "level $L $(grep gbps gpurun_out/lz4_micro_L$L.log)"
done
for f in groupby join; do
  timeout -k 10 300 python bench.py --flow $f --steps 20 > gpurun_out/bench_$f.log 2>&1 || { tail -20 gpurun_out/bench_$f.log; exit 1; }
  grep metric gpurun_out/bench_$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', d['value']/1e6, d['ms_per_step'], d['p99_latency_process_ms'], d['config'].get('lz4_ratio'), d['generation_s'])"
done
