#!/bin/bash
# A/B of library builds (RTW_LIB) on one config: rounds x libs, bench.py per-kernel times.
# usage: CONFIG=c2 SPP=64 ROUNDS=2 bash tools/ab_lib.sh "" build/prev.so ...
set -o pipefail
CONFIG=${CONFIG:-c2}; SPP=${SPP:-64}; ROUNDS=${ROUNDS:-2}
for r in $(seq $ROUNDS); do
  for lib in "$@"; do
    RTW_LIB=$lib timeout -k 10 300 python bench.py --config $CONFIG --spp $SPP --no-cpu-baseline --steps 2 \
      > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$CONFIG', repr('$lib'), d['value'], d['roofline']['kernel_ms_per_step'])"
  done
done
