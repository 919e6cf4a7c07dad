# Kafka record batches decoded on the GPU: tests, then the groupby bench with the kafka source vs pinned-lz4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kafka_device.py tests/test_kafka.py tests/test_lz4.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/kafka_tests.log 2>&1 || { tail -30 gpurun_out/kafka_tests.log; exit 1; }
tail -1 gpurun_out/kafka_tests.log
for src in kafka pinned-lz4; do
  timeout -k 10 400 python bench.py --source $src --steps 30 > gpurun_out/kafka_bench_$src.log 2>&1 || { tail -20 gpurun_out/kafka_bench_$src.log; exit 1; }
  grep metric gpurun_out/kafka_bench_$src.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$src', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['p99_latency_process_ms'],2), d['config'].get('ingest_bytes_per_event'), d['generation_s'])"
done
