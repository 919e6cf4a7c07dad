set -o pipefail
mkdir -p gpurun_out
for f in ${FLOWS:-groupby window full passthrough}; do
  timeout -k 10 300 python tools/sync_audit.py --flow $f > gpurun_out/sync_$f.txt 2>gpurun_out/sync_$f.err || { tail -20 gpurun_out/sync_$f.err; exit 1; }
  head -30 gpurun_out/sync_$f.txt
done
