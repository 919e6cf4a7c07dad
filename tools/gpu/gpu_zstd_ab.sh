# zstd decoder A/B over variant builds (tools/_cmp/libdxa_kernels_<v>.so, dxa.ops.build.build_variant): codec GPU
# tests on the in-tree library, then tools/zstd_bench.py (bytes checked against the input) at levels 1 and 3 per
# variant, REPS alternating rounds; FLOW=1 adds the groupby flow with --kafka-codec zstd per variant.
# VARIANTS="zstd_base zstd_zg32 ..."  OUT=<dir>
set -o pipefail
O=gpurun_out/${OUT:-zstd_ab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kafka_codecs.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in $(seq 1 ${REPS:-1}); do
  for v in ${VARIANTS:-zstd_base}; do
    for lvl in 1 3; do
      DXA_NATIVE_LIB=tools/_cmp/libdxa_kernels_$v.so timeout -k 10 180 python tools/zstd_bench.py --level $lvl \
        > $O/${v}_${lvl}_$rep.json 2> $O/${v}_${lvl}_$rep.err || { tail $O/${v}_${lvl}_$rep.err; exit 1; }
      python -c "
import json; d=json.load(open('$O/${v}_${lvl}_$rep.json')); p=d['per_frame']
print('$v', 'L$lvl', 'rep $rep', 'ok' if d['ok'] else 'MISMATCH', d['best_ms'], 'ms', d['gbps'], 'GB/s',
      round(p['seq_loop'] / max(1, p['sequences'])), 'cyc/seq', round(p['literals']), 'lit cyc')"
    done
  done
done
[ -z "$FLOW" ] && exit 0
for v in ${VARIANTS:-zstd_base}; do
  DXA_NATIVE_LIB=tools/_cmp/libdxa_kernels_$v.so timeout -k 10 420 python bench.py --steps ${STEPS:-30} \
    --kafka-codec zstd > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  grep '"metric"' $O/bench_$v.log | python -c "
import sys,json
d=json.loads(sys.stdin.readline()); print('zstd groupby', '$v', round(d['value']/1e6,2),'M ev/s', round(d['ms_per_step'],2),'ms')"
done
