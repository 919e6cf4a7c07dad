# Round 4: passthrough A/B — parse-ahead stream on/off (D2H-bound flow)
set -o pipefail
mkdir -p gpurun_out/r4z
run() { name=$1; flow=$2; shift 2; env "$@" timeout -k 10 300 python bench.py --flow $flow --steps 100 > gpurun_out/r4z/$name.log 2>&1 || { tail -20 gpurun_out/r4z/$name.log; exit 1; }
  grep metric gpurun_out/r4z/$name.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$name', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms p50', round(d['p50_latency_process_ms'],2), d.get('output_d2h'))"; }
run pt_side passthrough DXA_PARSE_STREAM=1
run pt_cur passthrough DXA_PARSE_STREAM=0
run pt_side2 passthrough DXA_PARSE_STREAM=1
run pt_cur2 passthrough DXA_PARSE_STREAM=0
run join_side join DXA_PARSE_STREAM=1
run join_cur join DXA_PARSE_STREAM=0
