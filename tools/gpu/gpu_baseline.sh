# GPU suite, smoke, then each flow once (window/full at the 300-pane default); OUT=<dir under gpurun_out>
set -o pipefail
O=gpurun_out/${OUT:-base}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
for f in ${FLOWS:-groupby window full join passthrough}; do
  timeout -k 10 420 python bench.py --flow $f --steps 40 > $O/$f.log 2>&1 || { tail -20 $O/$f.log; exit 1; }
  grep '"metric"' $O/$f.log | python -c "
import sys,json
d=json.loads(sys.stdin.readline()); print('$f', round(d['value']/1e6,2),'M ev/s', round(d['ms_per_step'],2),'ms p99', round(d['p99_latency_process_ms'],1), 'h2d', d.get('h2d_gb_s'), 'pcie', d.get('pcie_fraction'), 'panes', d.get('window_panes'))"
done
