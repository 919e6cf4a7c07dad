# PMC counters of the generator micro-bench (gen_len / gen_write kernels); one rocprofv3 pass per counter group
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P3="SQ_INSTS_SMEM SQ_IFETCH SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $R/gpurun_out/pmc_gen/p$i -o p$i -- python3 $R/tools/gen_bench.py --reps 1 > $R/gpurun_out/pmc_gen_p$i.log 2>&1 || { tail -20 $R/gpurun_out/pmc_gen_p$i.log; [ $i = 3 ] || exit 1; }
  find $R/gpurun_out/pmc_gen/p$i -name "*kernel_trace*" -delete
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_gen.md $R/gpurun_out/pmc_gen/p1 $R/gpurun_out/pmc_gen/p2 $R/gpurun_out/pmc_gen/p3
head -5 $R/gpurun_out/pmc_gen.md | cut -c1-1500
