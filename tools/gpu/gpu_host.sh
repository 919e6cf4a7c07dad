# host-side attribution of the window / full flows: host sections, sync audit, and a rocprofv3 kernel trace of the
# 300-pane window with its idle-gap summary.  OUT=<dir under gpurun_out>
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-host}
mkdir -p $O
for f in ${FLOWS:-window full}; do
  DXA_HOST_TIMERS=1 DXA_BENCH_HOST_TRACE=1 timeout -k 10 420 python bench.py --flow $f --steps 40 --profile-stages > $O/host_$f.log 2>&1 || { tail -20 $O/host_$f.log; exit 1; }
  timeout -k 10 300 python tools/sync_audit.py --flow $f > $O/sync_$f.txt 2>$O/sync_$f.err || { tail -20 $O/sync_$f.err; exit 1; }
  head -20 $O/sync_$f.txt
done
[ -n "$NOPROF" ] && exit 0
for f in ${PROF_FLOWS:-window}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof_$f -o run -- python3 bench.py --flow $f --steps 30 > $O/prof_$f.log 2>&1 || { tail -20 $O/prof_$f.log; exit 1; }
  python tools/gap_summary.py $O/prof_$f --last-ms 200 > $O/gaps_$f.txt 2>&1 || { tail -20 $O/gaps_$f.txt; exit 1; }
  head -30 $O/gaps_$f.txt
done
