#!/bin/bash
# Round 5: C5 at 12 / 16 / 24 iterations vs the default 9
set -u
OUT=gpurun_out/r5/ab_iters6_c5 CONFIG=c5 ROUNDS=2 STEPS=2 bash tools/ab_knob.sh '' '{"wf_iters": 12}' '{"wf_iters": 16}' '{"wf_iters": 24}' || exit 1
