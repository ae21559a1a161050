#!/bin/bash
# Round 5: same-box A/B of the dynamic deal (tuning.deal 1, the new default) against the static deal (0)
set -u
for cfg in simple_light cornell_smoke c2 c5; do
  OUT=gpurun_out/r5/ab_deal2_$cfg CONFIG=$cfg ROUNDS=2 STEPS=3 bash tools/ab_knob.sh '{"deal": 0}' '' || exit 1
done
