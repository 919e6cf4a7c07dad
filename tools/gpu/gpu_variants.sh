# A/B of prebuilt kernel-library variants (tools/_cmp/libdxa_kernels_<v>.so) on chosen flows
set -o pipefail
mkdir -p gpurun_out
for f in ${FLOWS:-window passthrough}; do
for v in ${VARIANTS:-base}; do
  DXA_NATIVE_LIB=$PWD/tools/_cmp/libdxa_kernels_$v.so timeout -k 10 300 python bench.py --flow $f --steps 20 > gpurun_out/var_${f}_$v.log 2>&1 || { tail -20 gpurun_out/var_${f}_$v.log; exit 1; }
  grep metric gpurun_out/var_${f}_$v.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f $v', round(d['value']/1e6,2), round(d['ms_per_step'],2))"
done
done
