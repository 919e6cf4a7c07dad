# PMC passes over the LZ4 decode micro-bench (kernel trace + counters only)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_lz4
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $R/gpurun_out/pmc_lz4/p$i -o p$i -- python3 $R/tools/lz4_bench.py --reps 1 > $R/gpurun_out/pmc_lz4_p$i.log 2>&1 || { tail -20 $R/gpurun_out/pmc_lz4_p$i.log; exit 1; }
  find $R/gpurun_out/pmc_lz4/p$i -name "*kernel_trace*" -delete
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_lz4.md $R/gpurun_out/pmc_lz4/p1 $R/gpurun_out/pmc_lz4/p2
grep -A4 -i "lz4_decode" $R/gpurun_out/pmc_lz4.md | head -40
