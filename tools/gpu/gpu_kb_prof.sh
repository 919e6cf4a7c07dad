# rocprofv3 kernel stats of the groupby flow at two producer batchings: 26 records / 16 KiB blocks vs the Java
# producer's batch.size=16384 (84 records, one ~51 KB LZ4 block per batch)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for cfg in "r26 --kafka-batch-records 26 --lz4-block 16384" "bs16k --kafka-batch-size 16384 --lz4-block 65536"; do
  set -- $cfg
  tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kbprof/$tag -o $tag -- python3 $R/bench.py --flow groupby --steps 10 "$@" > $R/gpurun_out/kbprof_$tag.log 2>&1 || { tail -20 $R/gpurun_out/kbprof_$tag.log; exit 1; }
  find $R/gpurun_out/kbprof/$tag -name "*kernel_trace*" -delete
  echo "== $tag"; head -12 $R/gpurun_out/kbprof/$tag/${tag}_kernel_stats.csv | cut -d, -f1-5 | cut -c1-150
done
