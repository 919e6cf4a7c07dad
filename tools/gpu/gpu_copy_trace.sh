# Which copies run as blit kernels (__amd_rocclr_copyBuffer) vs SDMA in the groupby flow: kernel + memory-copy trace
set -o pipefail
mkdir -p gpurun_out/ctrace
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/ctrace -o gb -- python3 $R/bench.py --flow groupby --steps 10 --warmup 3 > $R/gpurun_out/ctrace.log 2>&1 || { tail -20 $R/gpurun_out/ctrace.log; exit 1; }
cd $R && python3 tools/copy_trace_summary.py gpurun_out/ctrace > gpurun_out/ctrace_summary.txt && cat gpurun_out/ctrace_summary.txt
find $R/gpurun_out/ctrace -name "*.csv" -size +20M -delete
