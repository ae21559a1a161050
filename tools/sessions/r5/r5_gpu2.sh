#!/bin/bash
# Round 5: the 4-copy stage's block shapes (tuning.clds_shape) -- bit-identity, then a same-box A/B.
set -u
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "four_copy or knobs_invariant" > gpurun_out/r5/gpu2_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/gpu2_tests.txt; [ $rc = 0 ] || exit $rc
OUT=gpurun_out/r5/ab2 CONFIG=c2 ROUNDS=2 STEPS=5 bash tools/ab_knob.sh '' '{"bvh_orders": 4, "clds_shape": 2}' \
  '{"bvh_orders": 4, "clds_shape": 3}' '{"bvh_orders": 4, "clds_shape": 4}'
