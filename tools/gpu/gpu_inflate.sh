# gzip Kafka batches inflated on the GPU: kernel tests, then the groupby bench with gzip vs LZ4 record batches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kafka_device.py tests/test_lz4.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/inflate_tests.log 2>&1 || { tail -40 gpurun_out/inflate_tests.log; exit 1; }
tail -1 gpurun_out/inflate_tests.log
summ() { grep metric $1 | python -c "
import sys,json
d=json.loads(sys.stdin.readline()); c=d['config']; print('$2', round(d['value']/1e6,2),'M ev/s', round(d['ms_per_step'],2),'ms', c.get('ingest_bytes_per_event'),'B/ev ratio', c.get('lz4_ratio'), 'recs', c.get('kafka_batch_records'))"; }
for cfg in "gzip --kafka-codec gzip" "gzip_bs16k --kafka-codec gzip --kafka-batch-size 16384" "lz4"; do
  set -- $cfg; tag=$1; shift
  timeout -k 10 300 python bench.py --flow groupby --steps 20 "$@" > gpurun_out/codec_$tag.log 2>&1 || { tail -20 gpurun_out/codec_$tag.log; exit 1; }
  summ gpurun_out/codec_$tag.log $tag
done
