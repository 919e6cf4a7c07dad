# LZ4 frame block size: decoder micro-bench and groupby bench at 16 / 32 / 64 KiB blocks
set -o pipefail
mkdir -p gpurun_out
for b in ${BLOCKS:-16384 32768 65536}; do
  timeout -k 10 200 python tools/lz4_bench.py --block $b > gpurun_out/lz4_block_$b.log 2>&1 || { tail -20 gpurun_out/lz4_block_$b.log; exit 1; }
  echo "micro $b $(grep ratio gpurun_out/lz4_block_$b.log)"
  timeout -k 10 300 python bench.py --lz4-block $b > gpurun_out/bench_block_$b.log 2>&1 || { tail -20 gpurun_out/bench_block_$b.log; exit 1; }
  grep metric gpurun_out/bench_block_$b.log | python -c "
import sys,json
d=json.loads(sys.stdin.readline()); print('bench $b', round(d['value']/1e6,2),'M ev/s', round(d['ms_per_step'],2),'ms', d['config'].get('lz4_ratio'), d['config'].get('ingest_bytes_per_event'))"
done
