#!/bin/bash
# Round 5: wavefront iterations before the (now dynamically fed) tail, same box, C2 and C4
set -u
OUT=gpurun_out/r5/ab_iters_c2 CONFIG=c2 ROUNDS=2 STEPS=4 bash tools/ab_knob.sh '' '{"wf_iters": 5}' '{"wf_iters": 6}' '{"wf_iters": 7}' || exit 1
OUT=gpurun_out/r5/ab_iters_c4 CONFIG=c4 ROUNDS=1 STEPS=2 bash tools/ab_knob.sh '' '{"wf_iters": 6}' '{"wf_iters": 12}' || exit 1
OUT=gpurun_out/r5/ab_iters_cornell CONFIG=cornell ROUNDS=1 STEPS=2 bash tools/ab_knob.sh '' '{"wf_iters": 6}' '{"wf_iters": 12}' || exit 1
