set -o pipefail
mkdir -p gpurun_out
for J in 1 0; do
  DXA_JIT=$J DXA_BENCH_HOST_TRACE=1 timeout -k 10 420 python bench.py --flow full --steps 10 --torch-profile gpurun_out/tprof_full_jit$J.txt > gpurun_out/bench_full_jit$J.log 2>&1 || { tail -20 gpurun_out/bench_full_jit$J.log; exit 1; }
  grep metric gpurun_out/bench_full_jit$J.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('jit=$J', round(d['value']/1e6,2), round(d['ms_per_step'],2), d['host_trace_ms'][-3:])"
done
