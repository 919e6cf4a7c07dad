# Round 4: full GPU suite + smoke on the current tree
set -o pipefail
mkdir -p gpurun_out/r4v
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4v/tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r4v/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4v/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4v/smoke.log 2>&1 || { tail -20 gpurun_out/r4v/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > gpurun_out/r4v/bench_default.log 2>&1 || { tail -20 gpurun_out/r4v/bench_default.log; exit 1; }
grep metric gpurun_out/r4v/bench_default.log | cut -c1-200
