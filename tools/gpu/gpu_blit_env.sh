# passthrough (large D2H of rendered JSON): does the HIP blit engine choice change the step?
set -o pipefail
mkdir -p gpurun_out
for v in default 1 2 3; do
  if [ $v = default ]; then unset GPU_BLIT_ENGINE_TYPE; else export GPU_BLIT_ENGINE_TYPE=$v; fi
  timeout -k 10 240 python bench.py --flow passthrough --steps 20 > gpurun_out/blit_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/blit_$v.log; continue; }
  grep metric gpurun_out/blit_$v.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('blit $v', round(d['value']/1e6,2), round(d['ms_per_step'],2))"
done
