# host-8 feasibility: 8 concurrent rank planners with host CRC (within the box's 16-CPU share), and one rank's
# thread scaling.  OUT=<dir>
set -o pipefail
O=gpurun_out/${OUT:-host8}
mkdir -p $O
nproc > $O/nproc.txt; python -c "import os; print(len(os.sched_getaffinity(0)))" >> $O/nproc.txt
timeout -k 10 600 python tools/host8_bench.py --ranks 1 --threads 1,2,4,8,16 --seconds 5 > $O/rank1.jsonl 2> $O/rank1.err || { tail -20 $O/rank1.err; exit 1; }
cat $O/rank1.jsonl
timeout -k 10 600 python tools/host8_bench.py --ranks 8 --threads 1,2 --seconds 8 > $O/rank8.jsonl 2> $O/rank8.err || { tail -20 $O/rank8.err; exit 1; }
cat $O/rank8.jsonl
