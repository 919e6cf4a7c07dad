# zstd decoder on the in-tree library: tools/zstd_bench.py at levels 1 and 3 (phase cycles per frame), two rocprofv3
# counter passes over one level-3 launch, and (FLOW=1) the groupby flow with --kafka-codec zstd.  OUT=<dir>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-zstd_pmc}
mkdir -p $O
cd $R
for lvl in 1 3; do
  timeout -k 10 180 python tools/zstd_bench.py --level $lvl > $O/zstd_$lvl.json 2> $O/zstd_$lvl.err || { tail $O/zstd_$lvl.err; exit 1; }
  cat $O/zstd_$lvl.json
done
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $O/p$i -o p$i -- python3 $R/tools/zstd_bench.py --reps 1 --level 3 > $O/pmc_p$i.log 2>&1 || { tail -20 $O/pmc_p$i.log; exit 1; }
  find $O/p$i -name "*kernel_trace*" -delete
done
python3 $R/tools/pmc_summary.py $O/pmc_zstd.md $O/p1 $O/p2
head -4 $O/pmc_zstd.md
cd $R
[ -z "$FLOW" ] && exit 0
timeout -k 10 420 python bench.py --steps ${STEPS:-30} --kafka-codec zstd > $O/bench_zstd.log 2>&1 || { tail -20 $O/bench_zstd.log; exit 1; }
grep -o '"value": [0-9.]*' $O/bench_zstd.log | head -1
