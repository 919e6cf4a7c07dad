# Round 4: slotted one-pass generator vs two-pass on the now GPU-bound window flow (and full)
set -o pipefail
mkdir -p gpurun_out/r4dd
run() { name=$1; flow=$2; shift 2; env "$@" timeout -k 10 300 python bench.py --flow $flow --steps 100 > gpurun_out/r4dd/$name.log 2>&1 || { tail -20 gpurun_out/r4dd/$name.log; exit 1; }
  grep metric gpurun_out/r4dd/$name.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$name', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms p50', round(d['p50_latency_process_ms'],2))"; }
run window_2p window DXA_GEN_SLOTTED=0
run window_slot window DXA_GEN_SLOTTED=1
run full_2p full DXA_GEN_SLOTTED=0
run full_slot full DXA_GEN_SLOTTED=1
run window_2p_b window DXA_GEN_SLOTTED=0
run window_slot_b window DXA_GEN_SLOTTED=1
