set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "json or full_query" --timeout 120 --timeout-method thread > gpurun_out/parse_tests.log 2>&1 || { tail -40 gpurun_out/parse_tests.log; exit 1; }
tail -1 gpurun_out/parse_tests.log
for v in ${VARIANTS:-base w4}; do
  DXA_NATIVE_LIB=$PWD/tools/_cmp/libdxa_kernels_$v.so timeout -k 10 200 python tools/parse_bench.py > gpurun_out/parse_$v.log 2>&1 || { tail -20 gpurun_out/parse_$v.log; exit 1; }
  echo "$v $(grep gbps gpurun_out/parse_$v.log)"
done
for v in ${VARIANTS:-base w4}; do
  DXA_NATIVE_LIB=$PWD/tools/_cmp/libdxa_kernels_$v.so timeout -k 10 300 python bench.py --steps 20 > gpurun_out/parse_bench_$v.log 2>&1 || { tail -20 gpurun_out/parse_bench_$v.log; exit 1; }
  grep metric gpurun_out/parse_bench_$v.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('groupby $v', round(d['value']/1e6,2), round(d['ms_per_step'],2))"
done
