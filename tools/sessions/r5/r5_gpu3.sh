#!/bin/bash
# Round 5: the 32-B fp32-box compact nodes (compact_nodes 2, with bvh_orders 4) -- bit-identity, then A/B.
set -u
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "four_copy or knobs_invariant or compact_nodes_are_exact or tile_lists_random" > gpurun_out/r5/gpu3_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5/gpu3_tests.txt; [ $rc = 0 ] || exit $rc
OUT=gpurun_out/r5/ab3 CONFIG=c2 ROUNDS=2 STEPS=5 bash tools/ab_knob.sh '' '{"bvh_orders": 4, "compact_nodes": 2}' \
  '{"bvh_orders": 4, "clds_shape": 4}'
