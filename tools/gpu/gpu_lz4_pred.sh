# LZ4 decoder A/B: predicated fast path (default) vs the branching group kernel (DXA_LZ4_LANES=17)
set -o pipefail
mkdir -p gpurun_out
for v in pred group; do
  if [ $v = group ]; then export DXA_LZ4_LANES=17; else unset DXA_LZ4_LANES; fi
  timeout -k 10 300 python -u -m pytest tests/test_lz4.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lz4p_tests_$v.log 2>&1 || { tail -30 gpurun_out/lz4p_tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/lz4p_tests_$v.log)"
  timeout -k 10 200 python tools/lz4_bench.py --level 9 > gpurun_out/lz4p_micro_$v.log 2>&1 || { tail -20 gpurun_out/lz4p_micro_$v.log; exit 1; }
  echo "$v $(grep gbps gpurun_out/lz4p_micro_$v.log)"
done
for v in pred group; do
  if [ $v = group ]; then export DXA_LZ4_LANES=17; else unset DXA_LZ4_LANES; fi
  timeout -k 10 300 python bench.py --steps 30 > gpurun_out/lz4p_bench_$v.log 2>&1 || { tail -20 gpurun_out/lz4p_bench_$v.log; exit 1; }
  grep metric gpurun_out/lz4p_bench_$v.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('groupby $v', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['p99_latency_process_ms'],2))"
done
