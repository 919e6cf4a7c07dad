# targeted GPU tests, then the whole GPU suite, smoke and the flows; OUT=<dir under gpurun_out>
set -o pipefail
O=gpurun_out/${OUT:-check}
mkdir -p $O
# TESTS: test files; K: an optional -k expression
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${K:+-k "$K"} ${TESTS:-tests/test_windows.py tests/test_kafka_codecs.py tests/test_spark_int_widths.py tests/test_jit.py} > $O/targeted.log 2>&1 || { tail -60 $O/targeted.log; exit 1; }
tail -2 $O/targeted.log
[ -n "$QUICK" ] && exit 0
OUT=${OUT:-check} bash tools/gpu/gpu_baseline.sh
