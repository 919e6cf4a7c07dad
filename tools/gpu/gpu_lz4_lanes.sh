# LZ4 decoder group-width A/B: correctness tests and micro-bench per DXA_LZ4_LANES, then the groupby bench
set -o pipefail
mkdir -p gpurun_out
for L in 8 17; do
  DXA_LZ4_LANES=$L timeout -k 10 300 python -u -m pytest tests/test_lz4.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lz4_lanes_$L.log 2>&1 || { tail -30 gpurun_out/lz4_lanes_$L.log; exit 1; }
  echo "lanes $L: $(tail -1 gpurun_out/lz4_lanes_$L.log)"
done
for L in 16 17 8; do
  DXA_LZ4_LANES=$L timeout -k 10 300 python tools/lz4_bench.py > gpurun_out/lz4_micro_$L.json 2>&1 || { tail -20 gpurun_out/lz4_micro_$L.json; exit 1; }
  echo "lanes $L: $(tail -1 gpurun_out/lz4_micro_$L.json)"
done
for L in 16 8; do
  DXA_LZ4_LANES=$L timeout -k 10 300 python bench.py --steps 20 > gpurun_out/bench_lanes_$L.log 2>&1 || { tail -20 gpurun_out/bench_lanes_$L.log; exit 1; }
  grep metric gpurun_out/bench_lanes_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('groupby lanes $L', round(d['value']/1e6,2), round(d['ms_per_step'],2))"
done
