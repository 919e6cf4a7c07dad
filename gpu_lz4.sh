set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_lz4.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lz4_tests.log 2>&1 || { tail -30 gpurun_out/lz4_tests.log; exit 1; }
mkdir -p gpurun_out
for C in 1 4 8; do
  DXA_BENCH_HOST_TRACE=1 timeout -k 10 300 python bench.py --flow groupby --source pinned-lz4 --lz4-chunks $C --steps 12 > gpurun_out/lz4b_$C.log 2>&1 || { tail -20 gpurun_out/lz4b_$C.log; exit 1; }
  grep metric gpurun_out/lz4b_$C.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['ms_per_step'], d['host_trace_ms'])"
done
DXA_BENCH_HOST_TRACE=1 timeout -k 10 300 python bench.py --flow groupby --source pinned --steps 12 > gpurun_out/rawb.log 2>&1 || { tail -20 gpurun_out/rawb.log; exit 1; }
grep metric gpurun_out/rawb.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['ms_per_step'], d['host_trace_ms'])"
