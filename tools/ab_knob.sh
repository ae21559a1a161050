#!/bin/bash
# Same-box A/B of rtw_tuning knobs on one config with the in-tree library: ROUNDS x tunings,
# full bench.py lines (every tuning renders the same image), and the walk diagnostics of
# build/rtw_diag.so under each tuning when DIAG=1.
# usage: CONFIG=c2 ROUNDS=2 STEPS=5 DIAG=1 bash tools/ab_knob.sh '' '{"hoist": 0}'
# BENCH_EXTRA: more bench.py arguments (e.g. '--shard 8,3': one rank's shard)
set -u
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
CONFIG=${CONFIG:-c2}; ROUNDS=${ROUNDS:-2}; STEPS=${STEPS:-5}
n=0
if [ "${DIAG:-0}" = 1 ]; then
  for tu in "$@"; do
    n=$((n+1))
    RTW_LIB=build/rtw_diag.so timeout -k 10 200 python tools/diag_walk.py $CONFIG ${DIAG_SPP:-32} ${tu:+"$tu"} \
      > "$OUT/diag_${CONFIG}_$n.json" 2> "$OUT/diag.err" || { echo "diag $tu failed"; tail -5 "$OUT/diag.err"; exit 1; }
    echo "diag '$tu': $(cat $OUT/diag_${CONFIG}_$n.json)"
  done
fi
for r in $(seq $ROUNDS); do
  n=0
  for tu in "$@"; do
    n=$((n+1))
    timeout -k 10 400 python bench.py --config $CONFIG --no-cpu-baseline --steps $STEPS --warmup 1 ${BENCH_EXTRA:-} ${tu:+--tuning "$tu"} \
      > "$OUT/${CONFIG}_t${n}_$r.json" 2> "$OUT/ab.err" || { echo "bench '$tu' failed"; tail -5 "$OUT/ab.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/${CONFIG}_t${n}_$r.json'));print('$CONFIG', '''$tu''', $r, d['value'], d['roofline']['kernel_ms_per_step'])"
  done
done
