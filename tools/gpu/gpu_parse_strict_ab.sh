# isolated parse throughput: strict parser (current) vs the pre-strictness kernel (tools/_cmp/libdxa_kernels_oldparse.so)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for r in 1 2; do
  timeout -k 10 200 python tools/parse_bench.py > gpurun_out/pstrict_new_$r.log 2>&1 || { tail -20 gpurun_out/pstrict_new_$r.log; exit 1; }
  echo "new $(tail -1 gpurun_out/pstrict_new_$r.log)"
  DXA_NATIVE_LIB=$R/tools/_cmp/libdxa_kernels_oldparse.so timeout -k 10 200 python tools/parse_bench.py > gpurun_out/pstrict_old_$r.log 2>&1 || { tail -20 gpurun_out/pstrict_old_$r.log; exit 1; }
  echo "old $(tail -1 gpurun_out/pstrict_old_$r.log)"
done
