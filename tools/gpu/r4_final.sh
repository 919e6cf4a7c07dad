# Round 4 final: GPU suite, smoke, default bench, all five flows, kernel-trace launch counts + idle gaps of full
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/final/tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/final/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/final/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > gpurun_out/final/bench_default.log 2>&1 || { tail -20 gpurun_out/final/bench_default.log; exit 1; }
for f in groupby join window full passthrough; do
  timeout -k 10 300 python bench.py --flow $f --steps 100 > gpurun_out/final/bench_$f.log 2>&1 || { tail -20 gpurun_out/final/bench_$f.log; exit 1; }
  grep metric gpurun_out/final/bench_$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms p50', round(d['p50_latency_process_ms'],2), 'p99', round(d['p99_latency_process_ms'],2))"
done
FLOWS="window full" bash tools/gpu/gpu_prof.sh > gpurun_out/final/prof.txt 2>&1 || { tail -20 gpurun_out/final/prof.txt; exit 1; }
python - <<'PY'
import csv, json
for f in ["window", "full"]:
    rows = list(csv.DictReader(open(f"gpurun_out/prof/{f}/{f}_kernel_stats.csv")))
    d = json.loads([l for l in open(f"gpurun_out/prof_{f}.log") if l.startswith("{")][0])
    nb = d["steps"] + d["warmup"]
    calls = sum(int(r["Calls"]) for r in rows); ns = sum(int(r["TotalDurationNs"]) for r in rows)
    print(f, "calls/batch", round(calls / nb, 1), "GPU ms/batch", round(ns / nb / 1e6, 3), "step ms", round(d["ms_per_step"], 2))
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/final/trace -o full -- python3 $R/bench.py --flow full --steps 40 > $R/gpurun_out/final/trace.log 2>&1 || { tail -20 $R/gpurun_out/final/trace.log; exit 1; }
cd $R
python tools/gap_summary.py gpurun_out/final/trace --last-ms 150 --top 20 > gpurun_out/final/gaps_full.txt && head -3 gpurun_out/final/gaps_full.txt
rm -rf gpurun_out/final/trace
