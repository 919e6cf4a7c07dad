# Host CPU budget of the box vs the bench's threads: the cgroup quota, CPU throttling counters around a full-flow run,
# and the same run with OpenMP / Arrow pools held to one thread.  OUT=<dir>
set -o pipefail
O=gpurun_out/${OUT:-cpu_diag}
mkdir -p $O
CG=/sys/fs/cgroup
{ echo "cpu.max: $(cat $CG/cpu.max 2>/dev/null)"; echo "nproc: $(nproc)"; python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; env | grep -E "OMP|THREADS|MAX_JOBS" ; } > $O/box.txt 2>&1
cat $O/box.txt
for v in default omp1; do
  cat $CG/cpu.stat > $O/stat_${v}_before.txt 2>/dev/null
  if [ $v = omp1 ]; then export OMP_NUM_THREADS=1 ARROW_NUM_THREADS=1; fi
  TIMEFORMAT="%R %U %S"
  { time timeout -k 10 420 python bench.py --flow ${FLOW:-full} --steps 60 > $O/bench_$v.log 2> $O/err_$v.txt ; } 2> $O/time_$v.txt || { tail -20 $O/err_$v.txt; exit 1; }
  cat $CG/cpu.stat > $O/stat_${v}_after.txt 2>/dev/null
  python - $O $v <<'PY'
import json, sys
o, v = sys.argv[1], sys.argv[2]
d = json.loads([l for l in open(f"{o}/bench_{v}.log") if l.startswith("{")][0])
def stat(p):
    try:
        return {l.split()[0]: int(l.split()[1]) for l in open(p)}
    except OSError:
        return {}
b, a = stat(f"{o}/stat_{v}_before.txt"), stat(f"{o}/stat_{v}_after.txt")
real, user, sys_ = (float(x) for x in open(f"{o}/time_{v}.txt").read().split()[-3:])
print(v, round(d["value"] / 1e6, 1), "M ev/s", round(d["ms_per_step"], 2), "ms", "p99", round(d["p99_latency_process_ms"], 1),
      "| throttled periods", a.get("nr_throttled", 0) - b.get("nr_throttled", 0), "of", a.get("nr_periods", 0) - b.get("nr_periods", 0),
      "throttled ms", round((a.get("throttled_usec", 0) - b.get("throttled_usec", 0)) / 1e3, 1),
      "| wall", real, "s, cpu", round(user + sys_, 1), "s =", round((user + sys_) / real, 1), "CPUs")
PY
done
