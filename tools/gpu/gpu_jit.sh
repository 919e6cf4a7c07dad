set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_jit.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/jit_tests.log 2>&1 || { tail -40 gpurun_out/jit_tests.log; exit 1; }
tail -1 gpurun_out/jit_tests.log
timeout -k 10 300 python tools/jit_bench.py > gpurun_out/jit_bench.log 2>&1 || { tail -20 gpurun_out/jit_bench.log; exit 1; }
cat gpurun_out/jit_bench.log | grep expr
