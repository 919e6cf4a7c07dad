set -o pipefail
mkdir -p gpurun_out
for f in ${FLOWS:-full window groupby}; do
  timeout -k 10 300 python tools/host_profile.py --flow $f > gpurun_out/hprof_$f.txt 2>gpurun_out/hprof_$f.err || { tail -20 gpurun_out/hprof_$f.err; exit 1; }
  echo "$f done"
done
