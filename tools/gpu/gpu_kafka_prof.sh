set -o pipefail
mkdir -p gpurun_out
DXA_BENCH_HOST_TRACE=1 timeout -k 10 300 python bench.py --source kafka --steps 30 > gpurun_out/kprof_ht.log 2>&1 || { tail -20 gpurun_out/kprof_ht.log; exit 1; }
grep metric gpurun_out/kprof_ht.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print(round(d['value']/1e6,2), d.get('host_trace_ms'))"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/kafka -o kafka -- python3 $R/bench.py --source kafka --steps 20 > $R/gpurun_out/prof_kafka.log 2>&1 || exit 1
find $R/gpurun_out/prof/kafka -name "*kernel_trace*" -delete
head -16 $R/gpurun_out/prof/kafka/kafka_kernel_stats.csv | cut -d, -f1-4 | cut -c1-140
