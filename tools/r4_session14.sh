#!/bin/bash
# Round-4 session 14: wavefront iterations before the tail on the final build, C2 and C3 (knob sweep).
set -u
OUT=gpurun_out/s14
mkdir -p "$OUT"
CONFIG=c2 ROUNDS=2 STEPS=5 OUT=$OUT bash tools/ab_knob.sh '' '{"wf_iters": 12}' '{"wf_iters": 16}' '{"wf_iters": 7}' || exit $?
