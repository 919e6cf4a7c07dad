# Slotted (one-pass) vs packed (two-pass) GPU generator on the window / full flows, same box, alternating runs
set -o pipefail
mkdir -p gpurun_out/gen_slot
for r in 1 2; do
  for v in 1 0; do
    for f in ${FLOWS:-window full}; do
      DXA_GEN_SLOTTED=$v timeout -k 10 300 python bench.py --flow $f --steps 30 > gpurun_out/gen_slot/${f}_slot${v}_r$r.log 2>&1 || { tail -20 gpurun_out/gen_slot/${f}_slot${v}_r$r.log; exit 1; }
      grep metric gpurun_out/gen_slot/${f}_slot${v}_r$r.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f slotted=$v run $r', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms')"
    done
  done
done
