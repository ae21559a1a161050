#!/bin/bash
# Same-box A/B of library builds (RTW_LIB; "" = the in-tree product library) on one config: ROUNDS x libs,
# alternating, one bench.py line each (per-kernel times), saved as $OUT/<config>_<k>_<round>.json (k = the
# position of the library in the argument list).
# usage: CONFIG=c2 [SPP=0 (the config's)] [ROUNDS=2] [STEPS=5] [OUT=gpurun_out/ab] bash tools/ab_lib.sh "" build/rtw_x.so ...
set -o pipefail
CONFIG=${CONFIG:-c2}; SPP=${SPP:-0}; ROUNDS=${ROUNDS:-2}; STEPS=${STEPS:-5}; OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
for r in $(seq $ROUNDS); do
  k=0
  for lib in "$@"; do
    k=$((k+1))
    f="$OUT/${CONFIG}_${k}_${r}.json"
    RTW_LIB=$lib timeout -k 10 300 python bench.py --config $CONFIG --spp $SPP --no-cpu-baseline --steps $STEPS \
      --warmup 1 > "$f" 2> "$OUT/ab.err" || { echo "bench $lib failed"; tail -5 "$OUT/ab.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$f'));print('$CONFIG', repr('$lib'), $r, d['value'], d['roofline']['kernel_ms_per_step'])"
  done
done
