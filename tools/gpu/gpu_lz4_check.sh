# LZ4 decoder: GPU correctness tests, micro-bench, groupby bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lz4.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lz4_check.log 2>&1 || { tail -30 gpurun_out/lz4_check.log; exit 1; }
tail -1 gpurun_out/lz4_check.log
timeout -k 10 300 python tools/lz4_bench.py > gpurun_out/lz4_micro.json 2>&1 || { tail -20 gpurun_out/lz4_micro.json; exit 1; }
tail -1 gpurun_out/lz4_micro.json
timeout -k 10 300 python bench.py --steps 20 > gpurun_out/bench_lz4check.log 2>&1 || { tail -20 gpurun_out/bench_lz4check.log; exit 1; }
grep metric gpurun_out/bench_lz4check.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('groupby', round(d['value']/1e6,2), round(d['ms_per_step'],2))"
