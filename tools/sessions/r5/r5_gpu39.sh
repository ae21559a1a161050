#!/bin/bash
# Round 5: C5's iteration count under deal 59 (auto: 9 on image-textured scenes)
set -u
OUT=gpurun_out/r5/ab_iters5_c5 CONFIG=c5 ROUNDS=2 STEPS=2 bash tools/ab_knob.sh '' '{"wf_iters": 4}' '{"wf_iters": 6}' '{"wf_iters": 12}' || exit 1
