# Parser A/B: correctness (json GPU tests) + parse micro-bench + groupby bench + one PMC pass per variant
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for v in ${VARIANTS:-base ldswin}; do
  export DXA_NATIVE_LIB=$R/tools/_cmp/libdxa_kernels_$v.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_e2e_flows.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pab_tests_$v.log 2>&1 || { tail -30 gpurun_out/pab_tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/pab_tests_$v.log)"
  timeout -k 10 200 python tools/parse_bench.py > gpurun_out/pab_parse_$v.log 2>&1 || { tail -20 gpurun_out/pab_parse_$v.log; exit 1; }
  echo "$v $(grep gbps gpurun_out/pab_parse_$v.log)"
  timeout -k 10 300 python bench.py --steps 30 > gpurun_out/pab_bench_$v.log 2>&1 || { tail -20 gpurun_out/pab_bench_$v.log; exit 1; }
  grep metric gpurun_out/pab_bench_$v.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('groupby $v', round(d['value']/1e6,2), round(d['ms_per_step'],2))"
done
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
for v in ${VARIANTS:-base ldswin}; do
  export DXA_NATIVE_LIB=$R/tools/_cmp/libdxa_kernels_$v.so
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $R/gpurun_out/pab_pmc_$v -o p1 -- python3 $R/tools/parse_bench.py --reps 1 > $R/gpurun_out/pab_pmc_$v.log 2>&1 || { tail -20 $R/gpurun_out/pab_pmc_$v.log; exit 1; }
  find $R/gpurun_out/pab_pmc_$v -name "*kernel_trace*" -delete
  python3 $R/tools/pmc_summary.py $R/gpurun_out/pab_pmc_$v.md $R/gpurun_out/pab_pmc_$v
  grep json_parse $R/gpurun_out/pab_pmc_$v.md | cut -c1-400
done
