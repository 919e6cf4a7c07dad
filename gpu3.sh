# LZ4 ingest check: kernel tests, then groupby/join with raw vs LZ4-compressed pinned ingest, plus window/full
set -o pipefail
mkdir -p gpurun_out
python -m dxa.ops.build || exit 1
timeout -k 10 300 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 420 python bench.py "$@" > gpurun_out/b3_$name.log 2>&1 || { tail -20 gpurun_out/b3_$name.log; exit 1; }
  grep metric gpurun_out/b3_$name.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); c=d['config']; print('$name', round(d['value']/1e6,2),'M ev/s', round(d['ms_per_step'],2),'ms p99', round(d['p99_latency_process_ms'],2), c.get('ingest_bytes_per_event'), c.get('lz4_ratio'), d.get('stage_s'))"
}
run groupby_raw --flow groupby --steps 20 --profile-stages
run groupby_lz4 --flow groupby --source pinned-lz4 --steps 20 --profile-stages
run join_lz4 --flow join --source pinned-lz4 --steps 20 --profile-stages
run window --flow window --steps 20 --profile-stages
run full --flow full --steps 20 --profile-stages
