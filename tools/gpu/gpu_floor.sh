# groupby step floors: bytes already in HBM (no ingest) vs pinned-lz4, host-side timings per step
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for v in ${VARIANTS:-base ldswin}; do
  export DXA_NATIVE_LIB=$R/tools/_cmp/libdxa_kernels_$v.so
  for src in device pinned-lz4; do
    DXA_BENCH_HOST_TRACE=1 timeout -k 10 300 python bench.py --steps 30 --source $src > gpurun_out/floor_${v}_$src.log 2>&1 || { tail -20 gpurun_out/floor_${v}_$src.log; exit 1; }
    grep metric gpurun_out/floor_${v}_$src.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$v $src', round(d['value']/1e6,2), round(d['ms_per_step'],2), d.get('host_trace_ms'))"
  done
done
