# Parser variants: json GPU tests + parse micro-bench each, then groupby bench for the first two
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for v in ${VARIANTS:-ld w5 w6 w5t48 w5t32 reg}; do
  export DXA_NATIVE_LIB=$R/tools/_cmp/libdxa_kernels_$v.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "json or parse or full_query" --timeout 120 --timeout-method thread > gpurun_out/pab2_tests_$v.log 2>&1 || { tail -30 gpurun_out/pab2_tests_$v.log; exit 1; }
  timeout -k 10 200 python tools/parse_bench.py > gpurun_out/pab2_parse_$v.log 2>&1 || { tail -20 gpurun_out/pab2_parse_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/pab2_tests_$v.log) $(grep gbps gpurun_out/pab2_parse_$v.log)"
done
for v in ${BVARIANTS:-ld w5 reg}; do
  export DXA_NATIVE_LIB=$R/tools/_cmp/libdxa_kernels_$v.so
  for f in groupby window; do
  timeout -k 10 300 python bench.py --flow $f --steps 30 > gpurun_out/pab2_bench_${f}_$v.log 2>&1 || { tail -20 gpurun_out/pab2_bench_${f}_$v.log; exit 1; }
  grep metric gpurun_out/pab2_bench_${f}_$v.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f $v', round(d['value']/1e6,2), round(d['ms_per_step'],2))"
  done
done
