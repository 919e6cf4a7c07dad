# window / full flows: staging depth 2 (default) vs 3, alternating on one box
set -o pipefail
O=gpurun_out/r5_prefetch; mkdir -p $O
for rep in 1 2; do
  for f in window full; do
    for d in 2 3; do
      timeout -k 10 300 python bench.py --flow $f --steps 60 --prefetch $d > $O/${f}_d${d}_$rep.log 2>&1 || exit 1
    done
  done
done
grep -H -o '"value": [0-9.]*' $O/*.log
