# cycles first (what the collector still frees on the GPU path), then the settle_gc latency A/B
set -o pipefail
bash tools/gpu/gpu_gc_cycles.sh && bash tools/gpu/gpu_gc_ab.sh
