# Round 4 profiles: kernel-trace stats of every flow, launch attribution, PMC counter passes (parser/serializer)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4p
for f in window full; do
  ATTRIB_DEPTH=3 timeout -k 10 400 python tools/launch_attrib.py --flow $f --batches 6 --top 80 > gpurun_out/r4p/attrib_$f.txt 2>&1 || { tail -20 gpurun_out/r4p/attrib_$f.txt; exit 1; }
  head -3 gpurun_out/r4p/attrib_$f.txt | tail -1
done
FLOWS="full window" bash tools/gpu/gpu_host_profile.sh || exit 1
FLOWS="window full passthrough groupby join" bash tools/gpu/gpu_prof.sh || exit 1
