#!/bin/bash
# Round 5, first GPU session: the 4-copy compact stage (tuning.bvh_orders 4) and its two-block shape,
# checked for bit-identity by the GPU tests that cover it, then a same-box A/B against the 8-copy stage.
set -u
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "knobs_invariant or compact_nodes_are_exact or four_copy or concurrency or tile_lists_random" \
  > gpurun_out/r5/gpu1_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/gpu1_tests.txt; [ $rc = 0 ] || exit $rc
OUT=gpurun_out/r5/ab1 CONFIG=c2 ROUNDS=2 STEPS=5 bash tools/ab_knob.sh '' '{"bvh_orders": 4}' \
  '{"bvh_orders": 4, "clds_blocks": 1}'
