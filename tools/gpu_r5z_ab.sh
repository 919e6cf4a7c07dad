# A/B of in-kernel validity zeroing: previous commit (scratch/t_head) vs working tree, alternating, one box
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r5z_ab3; mkdir -p $O
pb() { (cd "$1" && timeout -k 10 120 python tools/parse_bench.py --reps 20 $3 > $O/$2.log 2>&1); }
H=$R/scratch/t_head
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_parse_fuzz.py tests/test_column_pruning.py \
  tests/test_flows_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/sel_tests.log 2>&1 && \
pb $R new_pb_full && pb $H head_pb_full && pb $H head_pb_full2 && pb $R new_pb_full2 && \
pb $R new_pb_pruned --pruned && pb $H head_pb_pruned --pruned
