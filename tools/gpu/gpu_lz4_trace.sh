# Kernel + memory-copy timeline of the chunked LZ4 groupby bench (no counters)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/trace_lz4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/trace_lz4 -o t -- python3 $R/bench.py --flow groupby --source pinned-lz4 --lz4-chunks ${C:-4} --steps 8 --warmup 3 --prefetch ${PF:-2} > $R/gpurun_out/trace_lz4.log 2>&1 || { tail -20 $R/gpurun_out/trace_lz4.log; exit 1; }
ls -la $R/gpurun_out/trace_lz4/
grep metric $R/gpurun_out/trace_lz4.log | cut -c1-200
