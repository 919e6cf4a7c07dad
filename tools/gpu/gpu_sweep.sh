# groupby bench parameter sweep: LZ4 chunks per batch x ingest prefetch depth
set -o pipefail
mkdir -p gpurun_out
for c in ${CHUNKS:-2 4 8}; do for pf in ${PREFETCH:-2 3}; do
  timeout -k 10 300 python bench.py --steps 20 --lz4-chunks $c --prefetch $pf > gpurun_out/sweep_${c}_$pf.log 2>&1 || { tail -20 gpurun_out/sweep_${c}_$pf.log; exit 1; }
  grep metric gpurun_out/sweep_${c}_$pf.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('chunks $c prefetch $pf', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['p99_latency_process_ms'],1))"
done; done
