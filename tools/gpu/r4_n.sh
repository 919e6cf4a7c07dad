# Round 4: batched output rendering (one launch pair per batch) + LDS-staged emitter writes (A/B vs unstaged build)
set -o pipefail
mkdir -p gpurun_out/r4n
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_flows_gpu.py tests/test_decimal.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4n/tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r4n/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4n/tests.log
summ() { grep metric $1 | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$2', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms', d.get('output_d2h'))"; }
for f in full passthrough window; do
  timeout -k 10 300 python bench.py --flow $f --steps 100 > gpurun_out/r4n/bench_$f.log 2>&1 || { tail -20 gpurun_out/r4n/bench_$f.log; exit 1; }
  summ gpurun_out/r4n/bench_$f.log "$f staged"
  DXA_NATIVE_LIB=$R/tools/_cmp/libdxa_kernels_nostage.so timeout -k 10 300 python bench.py --flow $f --steps 100 > gpurun_out/r4n/bench_${f}_nostage.log 2>&1 || { tail -20 gpurun_out/r4n/bench_${f}_nostage.log; exit 1; }
  summ gpurun_out/r4n/bench_${f}_nostage.log "$f unstaged"
done
cd /tmp && export TMPDIR=/tmp
for v in staged nostage; do
  LIBV=""; [ $v = nostage ] && LIBV=$R/tools/_cmp/libdxa_kernels_nostage.so
  DXA_NATIVE_LIB=$LIBV timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_MISS_sum --output-format csv -d $R/gpurun_out/r4n/pmc_$v -o w -- python3 $R/bench.py --flow passthrough --steps 4 --warmup 2 > $R/gpurun_out/r4n/pmc_$v.log 2>&1 || { tail -20 $R/gpurun_out/r4n/pmc_$v.log; exit 1; }
  find $R/gpurun_out/r4n/pmc_$v -name "*kernel_trace*" -delete
done
cd $R
python - <<'PY'
import csv, glob, collections
for v in ["staged", "nostage"]:
    acc = collections.defaultdict(list); dur = collections.defaultdict(list)
    for p in glob.glob(f"gpurun_out/r4n/pmc_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "")
            if ("gen_write" in k or "ser_write" in k) and r["Counter_Name"] == "WRITE_SIZE":
                acc[k].append(float(r["Counter_Value"])); dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for k in acc:
        print(v, k[-30:], "WRITE MB/dispatch", round(sum(acc[k]) / len(acc[k]) * 1024 / 1e6, 1), "median us", sorted(dur[k])[len(dur[k]) // 2] / 1e3)
PY
FLOWS="full" bash tools/gpu/gpu_prof.sh > gpurun_out/r4n/prof.txt 2>&1 || { tail -20 gpurun_out/r4n/prof.txt; exit 1; }
python - <<'PY'
import csv, json
for f in ["full"]:
    rows = list(csv.DictReader(open(f"gpurun_out/prof/{f}/{f}_kernel_stats.csv")))
    d = json.loads([l for l in open(f"gpurun_out/prof_{f}.log") if l.startswith("{")][0])
    nb = d["steps"] + d["warmup"]
    calls = sum(int(r["Calls"]) for r in rows); ns = sum(int(r["TotalDurationNs"]) for r in rows)
    print(f, "calls/batch", round(calls / nb, 1), "GPU ms/batch", round(ns / nb / 1e6, 3))
    for r in sorted(rows, key=lambda r: -int(r["Calls"]))[:14]:
        print("  ", round(int(r["Calls"]) / nb, 1), r["Name"][:90])
    for r in sorted(rows, key=lambda r: -int(r["TotalDurationNs"]))[:8]:
        print("  us/batch", round(int(r["TotalDurationNs"]) / nb / 1e3, 1), r["Name"][:90])
PY
