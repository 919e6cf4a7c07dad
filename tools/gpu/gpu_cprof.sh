# host profile (cProfile) of the timed steps of FLOWS; OUT=<dir>
set -o pipefail
O=gpurun_out/${OUT:-cprof}
mkdir -p $O
for f in ${FLOWS:-full}; do
  DXA_BENCH_CPROFILE=$O/$f.prof timeout -k 10 420 python bench.py --flow $f --steps ${STEPS:-60} > $O/$f.log 2>&1 || { tail -20 $O/$f.log; exit 1; }
  python tools/pstats_report.py $O/$f.prof ${STEPS:-60} > $O/${f}_report.txt 2>&1 || { tail -20 $O/${f}_report.txt; exit 1; }
  head -5 $O/$f.log | grep -o '"value": [0-9.]*'
done
