# one iteration: targeted GPU tests, then an A/B of bench variants, then the host attribution (no profile)
set -o pipefail
TESTS="${TESTS:-tests/test_windows.py tests/test_flows_gpu.py tests/test_e2e_flows.py}" QUICK=1 OUT=${OUT} bash tools/gpu/gpu_r6_check.sh && \
OUT=${OUT}/ab bash tools/gpu/gpu_ab.sh && \
NOPROF=1 OUT=${OUT} bash tools/gpu/gpu_r6_host.sh
