# Round 4: host profile after (cProfile of process_batch) + host sections of full / window
set -o pipefail
mkdir -p gpurun_out/r4aa
for f in full window; do
  timeout -k 10 300 python tools/host_profile.py --flow $f > gpurun_out/r4aa/hprof_$f.txt 2>gpurun_out/r4aa/hprof_$f.err || { tail -20 gpurun_out/r4aa/hprof_$f.err; exit 1; }
  DXA_HOST_TIMERS=1 timeout -k 10 300 python bench.py --flow $f --steps 100 --profile-stages > gpurun_out/r4aa/$f.log 2>&1 || { tail -20 gpurun_out/r4aa/$f.log; exit 1; }
  grep metric gpurun_out/r4aa/$f.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2)); print('  ', d.get('host_ms_per_step')); print('  ', d.get('host_sections_ms_per_step'))"
done
