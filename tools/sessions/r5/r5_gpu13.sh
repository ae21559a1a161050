#!/bin/bash
# Round 5: the compact-stage variants again on the deal-3 default, same box, 3 rounds
set -u
OUT=gpurun_out/r5/ab_stage_c2 CONFIG=c2 ROUNDS=3 STEPS=4 bash tools/ab_knob.sh '' '{"bvh_orders": 4, "compact_nodes": 2}' \
  '{"bvh_orders": 4, "clds_shape": 4}' '{"bvh_orders": 4}' || exit 1
