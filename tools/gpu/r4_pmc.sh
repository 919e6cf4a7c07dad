# Round 4 PMC tables: parser / serializer / aggregation kernels of the device-resident flows against the roofline
set -o pipefail
for F in full window passthrough; do
  FLOW=$F bash tools/gpu/gpu_pmc.sh || exit 1
  echo "pmc $F done"
done
