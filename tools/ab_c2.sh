#!/bin/bash
# Same-box A/B of library builds on the headline config: ROUNDS x libs, full bench.py lines
# (C2 unless CONFIG), alternating, plus the walk diagnostics of each diag build.
# usage: ROUNDS=2 STEPS=5 DIAGS="build/rtw_diag_base.so build/rtw_diag_tight.so" bash tools/ab_c2.sh "" build/rtw_base.so
set -u
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
CONFIG=${CONFIG:-c2}; ROUNDS=${ROUNDS:-2}; STEPS=${STEPS:-5}
for d in ${DIAGS:-}; do
  RTW_LIB=$d timeout -k 10 200 python tools/diag_walk.py $CONFIG ${DIAG_SPP:-32} > "$OUT/diag_$(basename $d .so).json" 2> "$OUT/diag.err" \
    || { echo "diag $d failed"; cat "$OUT/diag.err"; exit 1; }
  echo "diag $d: $(cat $OUT/diag_$(basename $d .so).json)"
done
for r in $(seq $ROUNDS); do
  for lib in "$@"; do
    tag=$(basename "${lib:-default}" .so)
    RTW_LIB=$lib timeout -k 10 400 python bench.py --config $CONFIG --no-cpu-baseline --steps $STEPS --warmup 1 \
      > "$OUT/${CONFIG}_${tag}_$r.json" 2> "$OUT/ab.err" || { echo "bench $lib failed"; tail -5 "$OUT/ab.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/${CONFIG}_${tag}_$r.json'));print('$CONFIG', '$tag', $r, d['value'], d['roofline']['kernel_ms_per_step'])"
  done
done
