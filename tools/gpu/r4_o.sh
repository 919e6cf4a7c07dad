# Round 4: idle-gap attribution of the full flow (kernel + memory-copy trace), host profile
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4o
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/r4o/trace -o full -- python3 $R/bench.py --flow full --steps 40 > $R/gpurun_out/r4o/trace.log 2>&1 || { tail -20 $R/gpurun_out/r4o/trace.log; exit 1; }
cd $R
python tools/gap_summary.py gpurun_out/r4o/trace --last-ms 200 --top 30 > gpurun_out/r4o/gaps_full.txt && cat gpurun_out/r4o/gaps_full.txt
rm -rf gpurun_out/r4o/trace
