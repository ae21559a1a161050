#!/bin/bash
# Round 5: full GPU suite on the auto deal (dynamic only for batches of >= 192 chunks per wave), + simple_light / c2 A/B
set -u
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5/gpu12_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/gpu12_tests.txt; [ $rc = 0 ] || exit $rc
for cfg in simple_light c2; do
  OUT=gpurun_out/r5/ab_deal4_$cfg CONFIG=$cfg ROUNDS=2 STEPS=3 bash tools/ab_knob.sh '{"deal": 0}' '' || exit 1
done
