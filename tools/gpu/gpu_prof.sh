# Kernel-level profiles (kernel trace + stats only) of every bench flow; keeps only the stats CSVs
set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for f in ${FLOWS:-groupby join window full}; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/$f -o $f -- python3 $R/bench.py --flow $f --steps 60 > $R/gpurun_out/prof_$f.log 2>&1 || { tail -20 $R/gpurun_out/prof_$f.log; exit 1; }
  find $R/gpurun_out/prof/$f -name "*kernel_trace*" -delete
done
for f in groupby join window full; do echo "== $f"; head -12 $R/gpurun_out/prof/$f/${f}_kernel_stats.csv | cut -d, -f1-5 | cut -c1-150; grep -h metric $R/gpurun_out/prof_$f.log | cut -c1-200; done
