# A/B of in-kernel string-slot zeroing: committed tree (scratch/t_head) vs working tree, alternating, one box
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r5z_ab2; mkdir -p $O
pb() { (cd "$1" && timeout -k 10 120 python tools/parse_bench.py --reps 20 $3 > $O/$2.log 2>&1); }
run() { (cd "$1" && timeout -k 10 300 python bench.py --flow $2 --steps 400 > $O/$3.log 2>&1); }
H=$R/scratch/t_head
pb $R new_pb_full && pb $H head_pb_full && pb $H head_pb_full2 && pb $R new_pb_full2 && \
pb $R new_pb_pruned --pruned && pb $H head_pb_pruned --pruned && \
run $H full head_full_1 && run $R full new_full_1 && run $R full new_full_2 && run $H full head_full_2 && \
run $H full head_full_3 && run $R full new_full_3 && \
run $R window new_window_1 && run $H window head_window_1 && run $H window head_window_2 && run $R window new_window_2
