# rocprofv3 counter passes over the device gzip kernel (one pass per counter group, each time-limited)
set -o pipefail
mkdir -p gpurun_out/gzpmc
export PYTHONPATH=$PWD
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/gzpmc/trace -o trace -- python3 $R/tools/gpu/gzip_once.py > $R/gpurun_out/gzpmc/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/gzpmc/p1 -o p1 -- python3 $R/tools/gpu/gzip_once.py > $R/gpurun_out/gzpmc/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY -d $R/gpurun_out/gzpmc/p2 -o p2 -- python3 $R/tools/gpu/gzip_once.py > $R/gpurun_out/gzpmc/p2.log 2>&1 || exit 1
cd $R && python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/gzpmc/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "gzip_chunks" in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f, dict(agg))
for f in glob.glob("gpurun_out/gzpmc/trace/**/*kernel_stats.csv", recursive=True):
    print(open(f).read()[:600])
PY
