#!/bin/bash
# Round-4 session 6: C4 bisect of the split trace's slowdown since the sphere-filter build:
# in-tree, build/rtw_head.so (sphere-filter build), rtw_hstruct (that + one rtw_wf field),
# rtw_nopk (in-tree with the split kernels' packed branches compiled out).
set -u
OUT=gpurun_out/s6
mkdir -p "$OUT"
CONFIG=c4 ROUNDS=${ROUNDS:-1} STEPS=2 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_head.so build/rtw_hstruct.so build/rtw_nopk.so || exit $?
# C2 and C5: the wave-cooperative rejection loop in the sphere-scene steps and tails (build/rtw_coop.so)
ROUNDS=2 STEPS=5 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_coop.so || exit $?
CONFIG=c5 ROUNDS=1 STEPS=3 OUT=$OUT bash tools/ab_c2.sh "" build/rtw_coop.so || exit $?
