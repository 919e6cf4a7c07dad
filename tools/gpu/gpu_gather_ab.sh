# string gather: GPU tests, then window/full flows with the lane-per-string kernel vs the wave-per-string one
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gather_tests.log 2>&1 || { tail -30 gpurun_out/gather_tests.log; exit 1; }
tail -1 gpurun_out/gather_tests.log
for f in window full; do
  for v in lane wave; do
    if [ $v = wave ]; then export DXA_STR_GATHER_WAVE=1; else unset DXA_STR_GATHER_WAVE; fi
    timeout -k 10 300 python bench.py --flow $f --steps 30 > gpurun_out/gather_${f}_$v.log 2>&1 || { tail -20 gpurun_out/gather_${f}_$v.log; exit 1; }
    grep metric gpurun_out/gather_${f}_$v.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f $v', round(d['value']/1e6,2), round(d['ms_per_step'],2))"
  done
done
