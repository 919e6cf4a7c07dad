# groupby bench with / without the device CRC check (A/B, twice each), and a kernel-stats profile
set -o pipefail
mkdir -p gpurun_out/crc
timeout -k 10 300 python -u -m pytest tests/test_kafka_device.py tests/test_kafka.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/crc/tests.log 2>&1 || { tail -30 gpurun_out/crc/tests.log; exit 1; }
tail -1 gpurun_out/crc/tests.log
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in crc nocrc; do
    flag=""; [ $v = nocrc ] && flag="--no-crc"
    timeout -k 10 240 python bench.py --steps 30 --warmup 5 $flag > gpurun_out/crc/bench_$v.log 2>&1 || { tail -20 gpurun_out/crc/bench_$v.log; exit 1; }
    grep metric gpurun_out/crc/bench_$v.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],3), d.get('p99_latency_batch_ms'))"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/crc/prof -o gb -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/crc/prof.log 2>&1 || { tail -20 $R/gpurun_out/crc/prof.log; exit 1; }
find $R/gpurun_out/crc/prof -name "*kernel_stats.csv" -exec head -14 {} \;
find $R/gpurun_out/crc/prof -name "*kernel_trace.csv" -delete
