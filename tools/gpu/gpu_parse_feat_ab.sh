# isolated parse throughput per parser feature variant (tools/_cmp/libdxa_kernels_<v>.so)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for r in 1 2; do
  for v in ${VARIANTS:-oldparse cur noctl noesc oldskip noseen}; do
    DXA_NATIVE_LIB=$R/tools/_cmp/libdxa_kernels_$v.so timeout -k 10 200 python tools/parse_bench.py > gpurun_out/pfeat_$v.log 2>&1 || { tail -20 gpurun_out/pfeat_$v.log; exit 1; }
    echo "$v $(tail -1 gpurun_out/pfeat_$v.log)"
  done
done
