# PMC counter passes (kernel trace + counters only; no runtime/sys tracing) for one bench flow; summary → gpurun_out/pmc_<flow>.md
set -o pipefail
F=${FLOW:-groupby}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_$F
# (extensions are built in-tree before the call; nothing is compiled on the box)
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P3="FETCH_SIZE TCC_HIT_sum"
P4="WRITE_SIZE TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $R/gpurun_out/pmc_$F/p$i -o p$i -- python3 $R/bench.py --flow $F --steps 4 --warmup 2 > $R/gpurun_out/pmc_${F}_p$i.log 2>&1 || { tail -20 $R/gpurun_out/pmc_${F}_p$i.log; exit 1; }
  find $R/gpurun_out/pmc_$F/p$i -name "*kernel_trace*" -delete
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_$F.md $R/gpurun_out/pmc_$F/p1 $R/gpurun_out/pmc_$F/p2 $R/gpurun_out/pmc_$F/p3 $R/gpurun_out/pmc_$F/p4
