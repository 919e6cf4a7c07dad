# Round 4: launch attribution (ATen ops / native launches / host syncs per batch) on the final tree
set -o pipefail
mkdir -p gpurun_out/r4ee
for f in full window; do
  DXA_INFERENCE_MODE=0 ATTRIB_DEPTH=3 timeout -k 10 400 python tools/launch_attrib.py --flow $f --batches 6 --top 80 > gpurun_out/r4ee/attrib_$f.txt 2>&1 || { tail -20 gpurun_out/r4ee/attrib_$f.txt; exit 1; }
  head -3 gpurun_out/r4ee/attrib_$f.txt | tail -1
done
