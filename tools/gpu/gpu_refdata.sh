# Device CSV reference data: differential tests, then the join bench at 100M rows (CSV written once, loaded through
# datax.job.input.default.referencedata.*)
set -o pipefail
mkdir -p gpurun_out/refdata
timeout -k 10 300 python -u -m pytest tests/test_refdata.py tests/test_kafka.py tests/test_kafka_device.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/refdata/tests.log 2>&1 || { tail -40 gpurun_out/refdata/tests.log; exit 1; }
tail -1 gpurun_out/refdata/tests.log
timeout -k 10 500 python bench.py --flow join --steps 20 > gpurun_out/refdata/bench_join.log 2>&1 || { tail -30 gpurun_out/refdata/bench_join.log; exit 1; }
grep metric gpurun_out/refdata/bench_join.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('join', round(d['value']/1e6,2), round(d['ms_per_step'],3), d.get('p99_latency_batch_ms'), d['reference_build_s'], d['reference_load'], d.get('max_hbm_allocated_gb'))"
timeout -k 10 300 python bench.py --steps 20 > gpurun_out/refdata/bench_groupby.log 2>&1 || { tail -30 gpurun_out/refdata/bench_groupby.log; exit 1; }
grep metric gpurun_out/refdata/bench_groupby.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('groupby', round(d['value']/1e6,2), round(d['ms_per_step'],3), d.get('p99_latency_batch_ms'))"
