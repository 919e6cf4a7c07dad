# groupby over Kafka record batches: producer batching (fixed records per batch, or bsN = the Java producer's
# batch.size=N with its compression-ratio estimator) x LZ4 block size x LZ4 decoder lanes per block x history ring
set -o pipefail
mkdir -p gpurun_out
summ() { grep metric $1 | python -c "
import sys,json
d=json.loads(sys.stdin.readline()); c=d['config']; print('$2', round(d['value']/1e6,2),'M ev/s', round(d['ms_per_step'],2),'ms', c.get('ingest_bytes_per_event'),'B/ev ratio', c.get('lz4_ratio'), 'recs', c.get('kafka_batch_records'))"; }
# KB_CFGS: space-separated configs, each records_block_lanes[_ring]
for cfg in ${KB_CFGS:-26_16384_16 bs16384_65536_16 bs16384_65536_8 105_65536_16}; do
  set -- ${cfg//_/ }
  case $1 in bs*) sel="--kafka-batch-size ${1#bs}";; *) sel="--kafka-batch-records $1";; esac
  DXA_LZ4_LANES=$3 DXA_LZ4_RING=${4:-2048} timeout -k 10 300 python bench.py --flow groupby --steps 20 $sel --lz4-block $2 > gpurun_out/kb_$1_$2_$3_${4:-2048}.log 2>&1 || { tail -20 gpurun_out/kb_$1_$2_$3_${4:-2048}.log; exit 1; }
  summ gpurun_out/kb_$1_$2_$3_${4:-2048}.log "$1 block=$2 lanes=$3 ring=${4:-2048}"
done
