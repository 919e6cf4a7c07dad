# roctx stage ranges (DXA_TRACE=1) + kernel trace → per-stage host time and GPU-busy share
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/marker
cd /tmp && export TMPDIR=/tmp
for f in ${FLOWS:-full window}; do
  DXA_TRACE=1 timeout -k 10 400 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $R/gpurun_out/marker/$f -o m -- python3 $R/bench.py --flow $f --steps 15 --warmup 40 > $R/gpurun_out/marker_$f.log 2>&1 || { tail -20 $R/gpurun_out/marker_$f.log; exit 1; }
  (cd $R && python3 tools/marker_summary.py gpurun_out/marker/$f --skip 40 > gpurun_out/marker_$f.txt && cat gpurun_out/marker_$f.txt)
  find $R/gpurun_out/marker/$f -name "*.csv" -size +20M -delete
done
