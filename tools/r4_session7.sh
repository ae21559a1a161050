#!/bin/bash
# Round-4 session 7 (final build): GPU suite, quick bench lines of C2 / C4 / C5, then the build-stamped
# VALU + traffic PMC passes of CFGS (tools/final_r4.sh with SKIP_BENCH=1).
set -u
OUT=gpurun_out/s7
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1; rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc = 0 ] || exit $rc
for c in c2 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/${c}_bench.json" 2> "$OUT/$c.err" || exit $?
  python3 -c "import json;d=json.loads([l for l in open('$OUT/${c}_bench.json') if l.startswith('{')][-1]);print('$c', d['value'], d['roofline']['kernel_ms_per_step'])"
done
CFGS=${CFGS:-"c2 c3 c4"} SKIP_BENCH=1 bash tools/final_r4.sh || exit $?
