# torch.profiler op/stage tables for the given flows (default: all bench flows), written to gpurun_out/tprof_<flow>.txt
set -o pipefail
mkdir -p gpurun_out
python -m dxa.ops.build || exit 1
FLOWS=${FLOWS:-"groupby window full passthrough"}
for f in $FLOWS; do
  timeout -k 10 420 python bench.py --flow $f --steps 10 --torch-profile gpurun_out/tprof_$f.txt > gpurun_out/tprof_$f.log 2>&1 || { tail -20 gpurun_out/tprof_$f.log; exit 1; }
  echo "== $f"; head -45 gpurun_out/tprof_$f.txt | cut -c1-190
done
