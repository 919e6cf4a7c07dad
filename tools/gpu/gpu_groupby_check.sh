# groupby flow: two plain runs (variance), one stage-timed run, one rocprofv3 kernel-stats run
set -o pipefail
mkdir -p gpurun_out
for k in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 > gpurun_out/gb_run$k.log 2>&1 || { tail -20 gpurun_out/gb_run$k.log; exit 1; }
  grep metric gpurun_out/gb_run$k.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('run$k', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['p99_latency_process_ms'],2), d['max_hbm_allocated_gb'])"
done
timeout -k 10 300 python bench.py --steps 20 --profile-stages > gpurun_out/gb_stages.log 2>&1 || { tail -20 gpurun_out/gb_stages.log; exit 1; }
grep metric gpurun_out/gb_stages.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('stages', round(d['value']/1e6,2), d.get('stage_s'))"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/groupby -o groupby -- python3 $R/bench.py --flow groupby --steps 20 > $R/gpurun_out/prof_groupby.log 2>&1 || exit 1
find $R/gpurun_out/prof/groupby -name "*kernel_trace*" -delete
head -30 $R/gpurun_out/prof/groupby/groupby_kernel_stats.csv | cut -d, -f1-4 | cut -c1-140
