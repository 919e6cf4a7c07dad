# Round 4: new GPU tests (exchange pack kernels, 2-rank flows on one GPU, SQL clauses) + host profiles
set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 900 python -u -m pytest tests/test_packing.py tests/test_sql_clauses24.py tests/test_distributed.py tests/test_flows_dist.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4b/tests.log 2>&1 || { tail -60 gpurun_out/r4b/tests.log; exit 1; }
tail -1 gpurun_out/r4b/tests.log
for f in full window; do
  timeout -k 10 300 python tools/host_profile.py --flow $f > gpurun_out/r4b/hprof_$f.txt 2>gpurun_out/r4b/hprof_$f.err || { tail -20 gpurun_out/r4b/hprof_$f.err; exit 1; }
  echo "$f profiled"
done
timeout -k 10 120 python tools/gpu/h2d_sync_probe.py > gpurun_out/r4b/h2d_probe.txt 2>&1 || { tail -20 gpurun_out/r4b/h2d_probe.txt; exit 1; }
cat gpurun_out/r4b/h2d_probe.txt
