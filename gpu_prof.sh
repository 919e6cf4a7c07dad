# Kernel-level profiles of the windowed flows (kernel trace + stats only)
set -o pipefail
mkdir -p gpurun_out/prof
python -m dxa.ops.build || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for f in window full; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/$f -o $f -- python3 $R/bench.py --flow $f --steps 20 > $R/gpurun_out/prof_$f.log 2>&1 || { tail -20 $R/gpurun_out/prof_$f.log; exit 1; }
done
find $R/gpurun_out/prof -name "*stats*" | head
find $R/gpurun_out/prof -name "*kernel_trace*" -delete
for f in window full; do echo "== $f"; head -25 $R/gpurun_out/prof/$f/${f}_kernel_stats.csv | cut -d, -f1-8; tail -1 $R/gpurun_out/prof_$f.log | cut -c1-300; done
