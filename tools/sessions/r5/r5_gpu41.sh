#!/bin/bash
# Round 5: C5 at 24 / 32 / 50 iterations, and simple_light (noise texture, no image) at 4 / 9 / 16
set -u
OUT=gpurun_out/r5/ab_iters7_c5 CONFIG=c5 ROUNDS=2 STEPS=2 bash tools/ab_knob.sh '{"wf_iters": 24}' '{"wf_iters": 32}' '{"wf_iters": 50}' || exit 1
OUT=gpurun_out/r5/ab_iters7_simple_light CONFIG=simple_light ROUNDS=2 STEPS=5 bash tools/ab_knob.sh '' '{"wf_iters": 9}' '{"wf_iters": 16}' || exit 1
