#!/bin/bash
# Round 5: the deal modes (tuning.deal bits) on every config, same box: 0 static, 1 iteration 0 only,
# 3 + the tail from one counter (default), 5 + the tail per stripe group
set -u
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "knobs_invariant or fused_step_bit or c3_geometry or shard" > gpurun_out/r5/gpu11_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/gpu11_tests.txt; [ $rc = 0 ] || exit $rc
for cfg in simple_light c2 c4 c5 cornell cornell_smoke; do
  OUT=gpurun_out/r5/ab_deal3_$cfg CONFIG=$cfg ROUNDS=2 STEPS=3 bash tools/ab_knob.sh '{"deal": 0}' '{"deal": 1}' '' '{"deal": 5}' || exit 1
done
