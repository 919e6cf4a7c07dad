# Round 4: fused group-table init — tests, launches per batch (full/window), benches of all five flows
set -o pipefail
mkdir -p gpurun_out/r4y
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_flows_gpu.py tests/test_decimal.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4y/tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r4y/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4y/tests.log
for f in groupby join window full passthrough; do
  timeout -k 10 300 python bench.py --flow $f --steps 100 > gpurun_out/r4y/bench_$f.log 2>&1 || { tail -20 gpurun_out/r4y/bench_$f.log; exit 1; }
  grep metric gpurun_out/r4y/bench_$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms p50', round(d['p50_latency_process_ms'],2), 'p99', round(d['p99_latency_process_ms'],2))"
done
FLOWS="window full" bash tools/gpu/gpu_prof.sh > gpurun_out/r4y/prof.txt 2>&1 || { tail -20 gpurun_out/r4y/prof.txt; exit 1; }
python - <<'PY'
import csv, json
for f in ["window", "full"]:
    rows = list(csv.DictReader(open(f"gpurun_out/prof/{f}/{f}_kernel_stats.csv")))
    d = json.loads([l for l in open(f"gpurun_out/prof_{f}.log") if l.startswith("{")][0])
    nb = d["steps"] + d["warmup"]
    calls = sum(int(r["Calls"]) for r in rows); ns = sum(int(r["TotalDurationNs"]) for r in rows)
    print(f, "calls/batch", round(calls / nb, 1), "GPU ms/batch", round(ns / nb / 1e6, 3), "step ms", round(d["ms_per_step"], 2))
    for r in sorted(rows, key=lambda r: -int(r["Calls"]))[:10]:
        print("  ", round(int(r["Calls"]) / nb, 1), r["Name"][:90])
PY
