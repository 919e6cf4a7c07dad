# A/B of emitter store variants: generator micro-bench + window/passthrough benches per variant
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-nt wb}; do
  DXA_NATIVE_LIB=$PWD/tools/_cmp/libdxa_kernels_$v.so timeout -k 10 120 python tools/gen_bench.py > gpurun_out/genab_$v.log 2>&1 || { tail -20 gpurun_out/genab_$v.log; exit 1; }
  echo "$v $(cat gpurun_out/genab_$v.log | grep events)"
done
VARIANTS="${VARIANTS:-nt wb}" FLOWS="${FLOWS:-passthrough window}" bash tools/gpu/gpu_variants.sh
