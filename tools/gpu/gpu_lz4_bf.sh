# group decoder: branching (DXA_LZ4_BF=0) vs branch-free masked stores/loads, 16 KiB and 64 KiB frame blocks
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lz4.py tests/test_kafka_device.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lz4bf_tests.log 2>&1 || { tail -30 gpurun_out/lz4bf_tests.log; exit 1; }
tail -1 gpurun_out/lz4bf_tests.log
for blk in 16384 65536; do
  for bf in 0 1; do
    DXA_LZ4_BF=$bf timeout -k 10 300 python tools/lz4_bench.py --block $blk --reps 10 > gpurun_out/lz4bf_${blk}_$bf.log 2>&1 || { tail -10 gpurun_out/lz4bf_${blk}_$bf.log; exit 1; }
    echo "block=$blk bf=$bf $(tail -1 gpurun_out/lz4bf_${blk}_$bf.log)"
  done
done
