# Round-4 first GPU session: GPU suite + smoke, then window/full benches (slotted vs two-pass generator) and a
# kernel-trace profile of the full flow
set -o pipefail
mkdir -p gpurun_out/r4
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r4/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.log 2>&1 || { tail -20 gpurun_out/r4/smoke.log; exit 1; }
echo smoke ok
for v in 0 1; do
  for f in window full; do
    DXA_GEN_SLOTTED=$v timeout -k 10 300 python bench.py --flow $f --steps 30 > gpurun_out/r4/${f}_slot$v.log 2>&1 || { tail -20 gpurun_out/r4/${f}_slot$v.log; exit 1; }
    grep metric gpurun_out/r4/${f}_slot$v.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f slotted=$v', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms')"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4/prof_full -o full -- python3 $R/bench.py --flow full --steps 20 > $R/gpurun_out/r4/prof_full.log 2>&1 || { tail -20 $R/gpurun_out/r4/prof_full.log; exit 1; }
find $R/gpurun_out/r4/prof_full -name "*kernel_trace*" -delete
echo prof done
