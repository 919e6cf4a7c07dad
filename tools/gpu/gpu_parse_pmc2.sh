# PMC passes over the parse micro-bench (default library); OUT=<dir under gpurun_out>
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=${OUT:-pmc_parse2}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
P3="FETCH_SIZE TCC_HIT_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $R/gpurun_out/$O/p$i -o p$i -- python3 $R/tools/parse_bench.py --reps 1 > $R/gpurun_out/${O}_p$i.log 2>&1 || { tail -20 $R/gpurun_out/${O}_p$i.log; exit 1; }
  find $R/gpurun_out/$O/p$i -name "*kernel_trace*" -delete
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/$O.md $R/gpurun_out/$O/p1 $R/gpurun_out/$O/p2 $R/gpurun_out/$O/p3
head -4 $R/gpurun_out/$O.md
