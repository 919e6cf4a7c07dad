# round-5 check of in-kernel string-slot zeroing: GPU suite, window / full / groupby benches, window kernel stats
set -o pipefail
O=gpurun_out/r5z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 240 python bench.py --flow window --steps 60 > $O/window_1.log 2>&1 && \
timeout -k 10 240 python bench.py --flow full --steps 60 > $O/full_1.log 2>&1 && \
timeout -k 10 240 python bench.py --steps 100 --warmup 5 > $O/groupby_1.log 2>&1 && \
timeout -k 10 240 python bench.py --flow window --steps 60 > $O/window_2.log 2>&1 && \
timeout -k 10 240 python bench.py --flow full --steps 60 > $O/full_2.log 2>&1 && \
timeout -k 10 240 python bench.py --steps 100 --warmup 5 > $O/groupby_2.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o win -- python3 bench.py --flow window --steps 40 > $O/prof.log 2>&1
