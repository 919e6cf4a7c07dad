# Reference cycles holding device memory, per flow (see tools/gc_cycles.py)
set -o pipefail
mkdir -p gpurun_out
for flow in groupby window full; do
  timeout -k 10 300 python -u tools/gc_cycles.py --flow $flow --steps 6 --warmup 3 > gpurun_out/gccyc_$flow.log 2>&1 || { tail -20 gpurun_out/gccyc_$flow.log; exit 1; }
  grep -v '^{"metric' gpurun_out/gccyc_$flow.log | grep -v amdgpu.ids | tail -40
done
