#!/bin/bash
# Round 5: fewer wavefront iterations before the dynamically fed tail, every config, same box
set -u
for cfg in c2 c4 cornell cornell_smoke c5 simple_light; do
  st=3; [ $cfg = c4 ] && st=2; [ $cfg = c5 ] && st=2
  OUT=gpurun_out/r5/ab_iters2_$cfg CONFIG=$cfg ROUNDS=2 STEPS=$st bash tools/ab_knob.sh '' '{"wf_iters": 3}' '{"wf_iters": 4}' '{"wf_iters": 5}' || exit 1
done
