# passthrough flow with gzip blob outputs: device gzip (default) vs host zlib (DXA_GPU_GZIP=0)
set -o pipefail
mkdir -p gpurun_out
summ() { grep metric $1 | python -c "
import sys,json
d=json.loads(sys.stdin.readline()); print('$1', round(d['value']/1e6,2),'M ev/s', round(d['ms_per_step'],2),'ms p99', round(d['p99_latency_process_ms'],2))"; }
timeout -k 10 300 python bench.py --flow passthrough --sink blob --workdir /tmp/dxa_bench_passthrough --steps 10 > gpurun_out/pt_blob.log 2>&1 || { tail -20 gpurun_out/pt_blob.log; exit 1; }
du -sh /tmp/dxa_bench_passthrough_0/out; ls /tmp/dxa_bench_passthrough_0/out/Tagged | head -3
rm -rf /tmp/dxa_bench_passthrough_0/out
summ gpurun_out/pt_blob.log
DXA_GPU_GZIP=0 timeout -k 10 300 python bench.py --flow passthrough --sink blob --workdir /tmp/dxa_bench_passthrough --steps 5 > gpurun_out/pt_blob_host.log 2>&1 || { tail -20 gpurun_out/pt_blob_host.log; exit 1; }
du -sh /tmp/dxa_bench_passthrough_0/out
rm -rf /tmp/dxa_bench_passthrough_0/out
summ gpurun_out/pt_blob_host.log
DXA_GZIP_DYNAMIC=1 timeout -k 10 300 python bench.py --flow passthrough --sink blob --workdir /tmp/dxa_bench_passthrough --steps 10 > gpurun_out/pt_blob_dyn.log 2>&1 || { tail -20 gpurun_out/pt_blob_dyn.log; exit 1; }
du -sh /tmp/dxa_bench_passthrough_0/out
rm -rf /tmp/dxa_bench_passthrough_0/out
summ gpurun_out/pt_blob_dyn.log
