# last check of the round-5 tree: GPU suite, smoke, default bench, window and full once
set -o pipefail
O=gpurun_out/final8; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
for f in window full; do
  timeout -k 10 400 python bench.py --flow $f --steps 60 > $O/${f}_1.log 2>&1 || { tail -20 $O/${f}_1.log; exit 1; }
done
grep -h -o '"metric": "[^"]*", "value": [0-9.]*' $O/*.log
