set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_e2e_flows.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/agg_tests.log 2>&1 || { tail -40 gpurun_out/agg_tests.log; exit 1; }
tail -1 gpurun_out/agg_tests.log
for f in groupby window full; do
  timeout -k 10 300 python bench.py --flow $f --steps 20 > gpurun_out/bench_$f.log 2>&1 || { tail -20 gpurun_out/bench_$f.log; exit 1; }
  grep metric gpurun_out/bench_$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['p50_latency_process_ms'],2), round(d['p99_latency_process_ms'],2))"
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/groupby -o groupby -- python3 $R/bench.py --flow groupby --steps 20 > $R/gpurun_out/prof_groupby.log 2>&1 || exit 1
find $R/gpurun_out/prof/groupby -name "*kernel_trace*" -delete
head -25 $R/gpurun_out/prof/groupby/groupby_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
