#!/bin/bash
# Round 5: emitter scenes -- 3 iterations, and the static tail (deal 57 = 59 without bit 2)
set -u
for cfg in cornell cornell_smoke simple_light; do
  st=3; [ $cfg = simple_light ] && st=5
  OUT=gpurun_out/r5/ab_light_$cfg CONFIG=$cfg ROUNDS=2 STEPS=$st bash tools/ab_knob.sh '' '{"wf_iters": 3}' '{"deal": 57}' || exit 1
done
