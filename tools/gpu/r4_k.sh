set -o pipefail
mkdir -p gpurun_out/r4k
timeout -k 10 300 python tools/gpu/dbg_unhex2.py > gpurun_out/r4k/dbg.txt 2>&1; tail -12 gpurun_out/r4k/dbg.txt
timeout -k 10 900 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4k/tests.log 2>&1 || { grep -E "PASS|FAIL|Error" gpurun_out/r4k/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4k/tests.log
for f in window full; do
  timeout -k 10 300 python bench.py --flow $f --steps 30 > gpurun_out/r4k/bench_$f.log 2>&1 || { tail -20 gpurun_out/r4k/bench_$f.log; exit 1; }
  grep metric gpurun_out/r4k/bench_$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms')"
done
for v in 1; do
  for f in window full; do
    DXA_GEN_SLOTTED=$v timeout -k 10 300 python bench.py --flow $f --steps 30 > gpurun_out/r4k/bench_${f}_slot$v.log 2>&1 || { tail -20 gpurun_out/r4k/bench_${f}_slot$v.log; exit 1; }
    grep metric gpurun_out/r4k/bench_${f}_slot$v.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f slotted', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms')"
  done
done
