set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lz4.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lz4_tests.log 2>&1 || { tail -30 gpurun_out/lz4_tests.log; exit 1; }
tail -1 gpurun_out/lz4_tests.log
timeout -k 10 200 python tools/lz4_bench.py > gpurun_out/lz4_micro_16.log 2>&1 || { tail -20 gpurun_out/lz4_micro_16.log; exit 1; }
grep gbps gpurun_out/lz4_micro_16.log
timeout -k 10 300 python bench.py --steps 20 > gpurun_out/lz4b.log 2>&1 || { tail -20 gpurun_out/lz4b.log; exit 1; }
grep metric gpurun_out/lz4b.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value']/1e6, d['ms_per_step'], d['p99_latency_process_ms'])"
