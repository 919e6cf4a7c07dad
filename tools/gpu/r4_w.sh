# Round 4: stage-1 structural index prototype — correctness vs host scan, timing vs json_parse, PMC counters
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4w
timeout -k 10 300 python -u -m pytest tests/test_json_index.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4w/tests.log 2>&1 || { tail -30 gpurun_out/r4w/tests.log; exit 1; }
tail -1 gpurun_out/r4w/tests.log
for ps in 16 64 256; do
  timeout -k 10 300 python tools/json_index_bench.py --per-seg $ps > gpurun_out/r4w/bench_$ps.json 2>&1 || { tail -20 gpurun_out/r4w/bench_$ps.json; exit 1; }
  tail -1 gpurun_out/r4w/bench_$ps.json
done
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $R/gpurun_out/r4w/pmc/p$i -o p$i -- python3 $R/tools/json_index_bench.py --reps 3 > $R/gpurun_out/r4w/pmc_p$i.log 2>&1 || { tail -20 $R/gpurun_out/r4w/pmc_p$i.log; exit 1; }
  find $R/gpurun_out/r4w/pmc/p$i -name "*kernel_trace*" -delete
done
cd $R
python tools/pmc_roofline.py gpurun_out/r4w/index_roofline.md "json_index prototype vs json_parse (1 M IoT events)" gpurun_out/r4w/pmc/p1 gpurun_out/r4w/pmc/p2 gpurun_out/r4w/pmc/p3
head -14 gpurun_out/r4w/index_roofline.md | tail -6
