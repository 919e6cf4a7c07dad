# cProfile of the timed steps of bench flows (host overhead), summarised by tools/pstats_report.py
set -o pipefail
mkdir -p gpurun_out
for f in ${FLOWS:-full window}; do
  DXA_BENCH_CPROFILE=gpurun_out/cprof_$f.prof timeout -k 10 420 python bench.py --flow $f --steps 20 > gpurun_out/cprof_bench_$f.log 2>&1 || { tail -20 gpurun_out/cprof_bench_$f.log; exit 1; }
  python tools/pstats_report.py gpurun_out/cprof_$f.prof 20 > gpurun_out/cprof_$f.txt
  grep metric gpurun_out/cprof_bench_$f.log | cut -c1-300
done
