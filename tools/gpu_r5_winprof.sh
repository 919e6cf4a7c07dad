# window flow (300-pane window) kernel trace: per-kernel stats and GPU idle gaps
set -o pipefail
O=gpurun_out/r5_winprof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o win -- python3 bench.py --flow window --steps 40 > $O/prof.log 2>&1
