#!/bin/bash
# PMC passes (VALU issue + HBM traffic) of bench.py for several configs; summaries under
# gpurun_out/pmc_<config>/, copied by hand to profiles/pmc_{valu,traffic}_<config>_sah.json.
set -u
for c in ${CONFIGS:-c3 c4 c5}; do
  steps=2; [ "$c" = c3 ] && steps=1
  OUT=gpurun_out/pmc_$c/valu BENCH_ARGS="--config $c --no-cpu-baseline --steps 1 --warmup 0" bash tools/pmc_valu.sh || exit $?
  OUT=gpurun_out/pmc_$c/traffic BENCH_ARGS="--config $c --no-cpu-baseline --steps 1 --warmup 0" bash tools/pmc_traffic.sh || exit $?
done
