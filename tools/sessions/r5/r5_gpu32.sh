#!/bin/bash
# Round 5: wavefront iterations for C4 (tree through L1/L2, split kernels) under deal 59
set -u
OUT=gpurun_out/r5/ab_iters4_c4 CONFIG=c4 ROUNDS=2 STEPS=2 bash tools/ab_knob.sh '' '{"wf_iters": 6}' '{"wf_iters": 9}' '{"wf_iters": 3}' || exit 1
